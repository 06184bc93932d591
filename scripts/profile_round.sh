#!/bin/bash
# One gpurun call: headline bench line, rocprofv3 kernel trace + stats of the headline workload (one
# stream, so every ensemble dispatch is the priced 50k-row launch), then the PMC passes (scripts/pmc.sh).
# Outputs under gpurun_out/; copy the ones to keep into profiles/<round>_*.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -5 gpurun_out/bench.err; exit 1; }
echo "bench ok"
cd /tmp && MOPO_ROLLOUT_SPLIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- \
  python "$R/bench.py" --no-cpu-baseline --no-c3 --no-alt-dtypes --train-epochs 0 > "$R/gpurun_out/prof_bench.json" 2> "$R/gpurun_out/prof.err" \
  || { tail -5 "$R/gpurun_out/prof.err"; exit 1; }
echo "rocprof ok"
cd "$R" && bash scripts/pmc.sh gpurun_out/pmc_summary.json
