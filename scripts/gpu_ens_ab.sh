#!/bin/bash
# Parity of kernel variants (each ab/<v>.so of $V swapped in for the ensemble / rollout GPU tests), then
# the A/B of $AB (scripts/ab.sh) over the variants that passed (and any $AB entry not in $V).
# usage: V="e_r2 a_r1" AB="e_r2 base" bash scripts/gpu_ens_ab.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
cp mopo_amd/libmopo_hip.so /tmp/lib_keep.so
failed=""
for v in $V; do
  cp ab/$v.so mopo_amd/libmopo_hip.so
  timeout -k 10 400 python -u -m pytest tests/test_gpu_ref.py tests/test_gpu_rollout.py -q -x -p no:cacheprovider \
    --timeout 200 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/ens_tests_$v.log 2>&1
  rc=$?
  echo "== $v"; tail -3 gpurun_out/ens_tests_$v.log
  # 1: a test failed (the variant is dropped); anything else (fault, abort, time limit): stop here
  if [ $rc -eq 1 ]; then failed="$failed $v"; elif [ $rc -ne 0 ]; then cp /tmp/lib_keep.so mopo_amd/libmopo_hip.so; exit $rc; fi
done
keep=""
for v in $AB; do
  case " $failed " in *" ${v%%:*} "*) echo "skip $v (parity failed)";; *) keep="$keep $v";; esac
done
rc=0
[ -n "$keep" ] && { AB="$keep" bash scripts/ab.sh; rc=$?; }
cp /tmp/lib_keep.so mopo_amd/libmopo_hip.so
exit $rc
