#!/bin/bash
# SAC checks (scripts/gpu_sac.sh), then an A/B of ensemble-kernel variants (scripts/ab.sh with $AB).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/gpu_sac.sh || exit $?
cp mopo_amd/libmopo_hip.so /tmp/lib_main.so
BENCH_ARGS="--no-alt-dtypes" bash scripts/ab.sh
rc=$?
cp /tmp/lib_main.so mopo_amd/libmopo_hip.so
exit $rc
