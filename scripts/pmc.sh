#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --kernel-trace only besides --pmc) over a short
# bench: HBM bytes (FETCH_SIZE, WRITE_SIZE separately, per MI355X_MICROARCH.md §HBM) and MFMA busy.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --sac-steps 50 --no-c3 --no-alt-dtypes --train-epochs 0"
# one stream: every ensemble launch is the 50k-row launch bench.py prices (roofline.avg_launch_ms)
export MOPO_ROLLOUT_SPLIT=1
cd /tmp
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES" "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$R/gpurun_out/pmc$i" -o run -- python "$R/bench.py" $ARGS > "$R/gpurun_out/pmc$i.log" 2>&1
  rc=$?
  echo "pass $i ($C) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$R/gpurun_out/pmc$i.log"; exit $rc; fi
done
cd "$R" && python scripts/pmc_summary.py gpurun_out/pmc_summary.json gpurun_out \
  "$(python -c 'import sys; sys.argv=["bench.py"]; import bench; print(bench.workload_key(bench.parse()))')"
