#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --kernel-trace only besides --pmc) over a short
# bench: HBM bytes (FETCH_SIZE, WRITE_SIZE separately, per MI355X_MICROARCH.md §HBM), MFMA busy, wait share,
# L2 hit rate and the VALU / MFMA / LDS instruction mix.
# usage: scripts/pmc.sh OUT.json [extra bench.py args selecting the workload, e.g. --ensemble-dtype fp32]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
OUT=${1:-gpurun_out/pmc_summary.json}
shift
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --sac-steps 50 --no-c3 --no-alt-dtypes --train-epochs 0 --prof-steps 2 $*"
KEY=$(python -c "import sys; sys.argv=['bench.py'] + sys.argv[1:]; import bench; print(bench.workload_key(bench.parse()))" $ARGS)
TAG=$(echo "$KEY" | tr ' =' '__')
# one stream: every ensemble launch is the full-batch launch bench.py prices (roofline.avg_launch_ms)
export MOPO_ROLLOUT_SPLIT=1
cd /tmp
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES" "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" \
         "TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_$TAG/pmc$i" -o run -- python "$R/bench.py" $ARGS > "$R/gpurun_out/pmc_${TAG}_$i.log" 2>&1
  rc=$?
  echo "$KEY pass $i ($C) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$R/gpurun_out/pmc_${TAG}_$i.log"; exit $rc; fi
done
cd "$R" && python scripts/pmc_summary.py "$OUT" "gpurun_out/pmc_$TAG" "$KEY"
