#!/bin/bash
# SAC parity on each ab/<v>.so of $AB (default build first), a same-box A/B of the step time over them
# (plus $AB_EXTRA, timing only), then the phase stamps of ab/sac_stamps.so.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
cp mopo_amd/libmopo_hip.so /tmp/lib_keep.so
for v in $AB; do
  cp ab/$v.so mopo_amd/libmopo_hip.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_sac.py tests/test_gpu_ref.py -q -x -p no:cacheprovider -k "sac or SAC" \
    --timeout 200 --timeout-method thread > gpurun_out/sac_tests_$v.log 2>&1
  rc=$?
  echo "== $v parity rc=$rc: $(tail -1 gpurun_out/sac_tests_$v.log)"
  [ $rc -ne 0 ] && { cp /tmp/lib_keep.so mopo_amd/libmopo_hip.so; exit $rc; }
done
AB="$AB_EXTRA $AB" bash scripts/ab_sac.sh || { cp /tmp/lib_keep.so mopo_amd/libmopo_hip.so; exit 1; }
cp ab/sac_stamps.so mopo_amd/libmopo_hip.so
timeout -k 10 120 python scripts/sac_stamps.py > gpurun_out/sac_stamps.txt 2>&1
src=$?
cp /tmp/lib_keep.so mopo_amd/libmopo_hip.so
cat gpurun_out/sac_stamps.txt
exit $src
