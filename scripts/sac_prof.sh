#!/bin/bash
# SAC parity tests + a kernel-trace of the SAC leg (per-position durations: scripts/sac_trace.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_sac.py -q -x -p no:cacheprovider > gpurun_out/sac_tests.log 2>&1
rc=$?
tail -3 gpurun_out/sac_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/sacprof" -o run -- python "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --sac-steps 300 --train-epochs 0 --no-c3 > "$R/gpurun_out/sacprof.json" 2> "$R/gpurun_out/sacprof.err"
rc=$?
echo "rocprof rc=$rc"
[ $rc -eq 0 ] && python "$R/scripts/sac_trace.py" "$R/gpurun_out/sacprof/run_kernel_trace.csv"
exit $rc
