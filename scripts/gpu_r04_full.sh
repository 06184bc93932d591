#!/bin/bash
# The whole -m gpu suite on the current build, then (if it passed) the A/B of $AB under $BENCH_ARGS and
# one default bench run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
if [ -n "$AB" ]; then
  cp mopo_amd/libmopo_hip.so /tmp/lib_keep.so
  bash scripts/ab.sh; r=$?
  cp /tmp/lib_keep.so mopo_amd/libmopo_hip.so
  [ $r -ne 0 ] && exit $r
fi
timeout -k 10 400 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
r=$?
tail -c 600 gpurun_out/bench_full.json
exit $r
