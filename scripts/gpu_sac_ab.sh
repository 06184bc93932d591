#!/bin/bash
# SAC parity (tests/test_gpu_sac.py + test_gpu_ref.py SAC cases) on each ab/<v>.so of $AB, then the
# same-box step-time A/B (scripts/ab_sac.sh) over those that passed.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
cp mopo_amd/libmopo_hip.so /tmp/lib_keep_s.so
ok=""
for v in $AB; do
  cp ab/$v.so mopo_amd/libmopo_hip.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_sac.py tests/test_gpu_ref.py -q -x -p no:cacheprovider -k "sac or SAC" \
    --timeout 200 --timeout-method thread > gpurun_out/sac_tests_$v.log 2>&1
  rc=$?
  echo "== $v rc=$rc"; tail -1 gpurun_out/sac_tests_$v.log
  if [ $rc -eq 0 ]; then ok="$ok $v"; elif [ $rc -ne 1 ]; then cp /tmp/lib_keep_s.so mopo_amd/libmopo_hip.so; exit $rc; fi
done
AB="$ok" bash scripts/ab_sac.sh; rc=$?
cp /tmp/lib_keep_s.so mopo_amd/libmopo_hip.so
exit $rc
