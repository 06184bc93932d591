#!/bin/bash
# Parity of an ensemble-kernel variant (ab/$V.so swapped in for the ensemble / rollout GPU tests), then
# the A/B of $AB (scripts/ab.sh).  usage: V=r2 AB="r2 base" bash scripts/gpu_ens_ab.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
cp ab/$V.so mopo_amd/libmopo_hip.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_ref.py tests/test_gpu_rollout.py -q -x -p no:cacheprovider \
  --timeout 200 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/ens_tests.log 2>&1
rc=$?
tail -15 gpurun_out/ens_tests.log
[ $rc -ne 0 ] && exit $rc
bash scripts/ab.sh
