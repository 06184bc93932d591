#!/bin/bash
# Roofline evidence for the shipped kernels, one gpurun call: for every leg in $LEGS (default: all),
#   1. rocprofv3 --kernel-trace --stats of that leg's bench run (its own bench line beside the trace),
#      reduced per (kernel, grid size) by scripts/trace_summary.py, and
#   2. the PMC passes of scripts/pmc.sh on the same workload, merged into one summary.
# Outputs: gpurun_out/prof_$TAG/<leg>/{bench.json, stats/, trace.json, trace.txt}, gpurun_out/prof_$TAG/pmc_summary.json
# usage: TAG=r06 LEGS="C2_bf16x6 C2_fp32" bash scripts/gpu_profile.sh  (NO_PMC=1: traces only; PMC_ONLY=1: PMC only)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
TAG=${TAG:-r06}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
NOX="--no-cpu-baseline --no-c3 --no-alt-dtypes"
declare -A A
A[C2_f16x3]="--ensemble-dtype f16x3 --train-epochs 0 --sac-steps 16"
A[C2_bf16x6]="--ensemble-dtype bf16x6 --train-epochs 2"
A[C2_fp32]="--ensemble-dtype fp32 --train-epochs 0 --sac-steps 16"
A[C3_bf16]="--config C3 --ensemble-dtype bf16 --train-epochs 0 --sac-steps 16"
A[N2_bf16x6]="--config N2 --ensemble-dtype bf16x6 --train-epochs 0 --sac-steps 16"
A[C5_fp32]="--config C5 --shards 8 --ensemble-dtype fp32 --train-epochs 0 --sac-steps 16 --steps 5 --warmup 2"
A[C5_f16x3]="--config C5 --shards 8 --ensemble-dtype f16x3 --train-epochs 0 --sac-steps 16 --steps 5 --warmup 2"
A[C5_bf16]="--config C5 --shards 8 --ensemble-dtype bf16 --train-epochs 0 --sac-steps 16 --steps 5 --warmup 2"
LEGS=${LEGS:-"C2_bf16x6 C2_f16x3 C2_fp32 N2_bf16x6 C3_bf16 C5_fp32 C5_f16x3 C5_bf16"}
for L in $LEGS; do
  [ -n "$PMC_ONLY" ] && break
  D=$R/$OUT/$L
  rm -rf $D && mkdir -p $D
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D/stats -o run -- \
     python $R/bench.py $NOX ${A[$L]} > $D/bench.json 2> $D/bench.err)
  rc=$?
  echo "$L trace rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $D/bench.err; exit $rc; }
  python scripts/trace_summary.py $D/stats --json $D/trace.json > $D/trace.txt
  head -12 $D/trace.txt
done
[ -n "$NO_PMC" ] && exit 0
for L in $LEGS; do
  # the PMC passes time a short bench of the same workload (the train leg only where it was traced)
  EXTRA=""
  [ "$L" = "C2_bf16x6" ] && EXTRA="--train-epochs 1 --sac-steps 200"
  bash scripts/pmc.sh $OUT/pmc_summary.json ${A[$L]} --steps 3 --warmup 1 --prof-steps 2 $EXTRA || exit $?
done
