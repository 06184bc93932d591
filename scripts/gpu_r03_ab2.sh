#!/bin/bash
# variant parity, then the C2 A/B ($AB) and the C3 bf16 A/B ($AB3) (scripts/ab.sh)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
V="$V" AB="$AB" bash scripts/gpu_ens_ab.sh || exit $?
cp gpurun_out/ab.txt gpurun_out/ab_c2.txt
if [ -n "$AB3" ]; then
  cp mopo_amd/libmopo_hip.so /tmp/lib_keep2.so
  AB="$AB3" BENCH_ARGS="--config C3 --ensemble-dtype bf16" bash scripts/ab.sh; rc=$?
  cp /tmp/lib_keep2.so mopo_amd/libmopo_hip.so
  cp gpurun_out/ab.txt gpurun_out/ab_c3.txt
  exit $rc
fi
