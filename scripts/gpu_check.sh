#!/bin/bash
# One gpurun call: GPU parity tests, then (only if no crash) bench + rocprof kernel-trace.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
[ -n "$NO_BENCH" ] && exit $rc
timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
brc=$?
cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
if [ $brc -ne 0 ]; then echo "bench rc=$brc: stopping"; exit $brc; fi
[ -n "$NO_PROF" ] && exit $rc
cd /tmp && MOPO_ROLLOUT_SPLIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof" -o run -- python "${GRAFT_REPO_ROOT:-/root/repo}/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof_bench.json" 2> "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof.err"
prc=$?
echo "rocprof rc=$prc"
exit $rc
