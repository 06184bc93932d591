#!/bin/bash
# One gpurun call: the GPU parity suite, then (if it did not crash) the default bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${TEST_LIMIT:-840} python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -25 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
[ -n "$NO_BENCH" ] && exit $rc
timeout -k 10 ${BENCH_LIMIT:-300} python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
brc=$?
tail -c 3000 gpurun_out/bench.json; tail -5 gpurun_out/bench.err
[ $brc -ne 0 ] && { echo "bench rc=$brc"; exit $brc; }
exit $rc
