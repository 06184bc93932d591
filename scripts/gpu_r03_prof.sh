#!/bin/bash
# One gpurun call: the rocprof kernel-trace stats and PMC passes of $STATS / $PMC (scripts/profile_r03.sh),
# then optional ensemble variant parity + A/B (scripts/gpu_ens_ab.sh: $V, $AB).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
if [ -n "$STATS$PMC" ]; then bash scripts/profile_r03.sh || exit $?; fi
[ -n "$PMC" ] && python -c "import json; d=json.load(open('gpurun_out/pmc_summary.json')); print(json.dumps(d)[:3000])"
if [ -n "$V$AB" ]; then bash scripts/gpu_ens_ab.sh || exit $?; fi
exit 0
