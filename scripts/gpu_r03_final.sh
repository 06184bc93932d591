#!/bin/bash
# Round-3 final measurement, call 1: the GPU parity suite + the default bench line (scripts/gpu_r03.sh),
# then rocprofv3 kernel stats of $STATS (scripts/profile_r03.sh), the SAC kernel trace and the BNN.train
# kernel stats.  Call 2 runs the PMC passes (PMC=... bash scripts/profile_r03.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_r03.sh; rc=$?
[ $rc -gt 1 ] && exit $rc
STATS="${STATS:-C2:f16x3 C2:fp32 C3:bf16}" PMC="" bash scripts/profile_r03.sh || exit $?
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/sacprof" -o run -- \
  python "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --sac-steps 300 --train-epochs 0 --no-c3 --no-alt-dtypes \
  > "$R/gpurun_out/sacprof.json" 2> "$R/gpurun_out/sacprof.err") || { tail -5 gpurun_out/sacprof.err; exit 1; }
python scripts/sac_trace.py gpurun_out/sacprof/run_kernel_trace.csv > gpurun_out/sac_trace.txt 2>&1
bash scripts/gpu_trainprof.sh || exit $?
exit $rc
