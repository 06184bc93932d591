#!/bin/bash
# Ensemble parity (reference-graph + oracle cases, f16x3 rollouts) on ab/$TESTV.so, then the headline
# A/B over ab/$AB.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
cp mopo_amd/libmopo_hip.so /tmp/lib_keep.so
for v in $TESTV; do
  cp ab/$v.so mopo_amd/libmopo_hip.so
  timeout -k 10 600 python -u -m pytest tests/test_gpu_ref.py tests/test_gpu_rollout.py -q -x -p no:cacheprovider \
    -k "bnn or f16x3 or split or full_size or fused" --timeout 300 --timeout-method thread > gpurun_out/ens_tests_$v.log 2>&1
  rc=$?
  echo "== $v parity rc=$rc: $(tail -1 gpurun_out/ens_tests_$v.log)"
  [ $rc -ne 0 ] && { cp /tmp/lib_keep.so mopo_amd/libmopo_hip.so; exit $rc; }
done
bash scripts/ab.sh; r=$?
cp /tmp/lib_keep.so mopo_amd/libmopo_hip.so
exit $r
