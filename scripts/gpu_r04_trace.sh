#!/bin/bash
# Kernel trace of the headline bench (the timed rollouts run split over two streams) for timeline analysis.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/trace" -o run -- \
  python "$R/bench.py" --steps 6 --warmup 4 --no-cpu-baseline --no-c3 --no-alt-dtypes --sac-steps 16 --train-epochs 0 \
  --prof-steps 1 > "$R/gpurun_out/trace_bench.json" 2> "$R/gpurun_out/trace_bench.err"
rc=$?
echo "rocprof rc=$rc"
ls -R "$R/gpurun_out/trace" | head
exit $rc
