#!/bin/bash
# One gpurun call: variant parity + A/B (scripts/gpu_ens_ab.sh: $V, $AB), then optionally the BNN.train
# kernel profile ($TRAINPROF=1, scripts/gpu_trainprof.sh) and the SAC trace ($SACPROF=1).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
if [ -n "$V$AB" ]; then bash scripts/gpu_ens_ab.sh || exit $?; fi
if [ -n "$TRAINPROF" ]; then bash scripts/gpu_trainprof.sh || exit $?; fi
exit 0
