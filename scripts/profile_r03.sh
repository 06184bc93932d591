#!/bin/bash
# Kernel-trace stats and PMC passes per workload, in one gpurun call.
#   STATS="C2:f16x3 C2:fp32 ..."  rocprofv3 --kernel-trace --stats of bench.py on each (one stream)
#   PMC="C2:f16x3 ..."            scripts/pmc.sh passes on each, merged into gpurun_out/pmc_summary.json
# Outputs under gpurun_out/; copy what to keep into profiles/r03_*.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
for W in $STATS; do
  cfg=${W%%:*}; dt=${W##*:}
  tag=${cfg}_${dt}
  (cd /tmp && MOPO_ROLLOUT_SPLIT=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$R/gpurun_out/stats_$tag" -o run -- python "$R/bench.py" --config $cfg --ensemble-dtype $dt --shards 8 --steps 10 \
      --warmup 3 --no-cpu-baseline --no-c3 --no-alt-dtypes --train-epochs 0 --sac-steps 400 \
      > "$R/gpurun_out/stats_$tag.json" 2> "$R/gpurun_out/stats_$tag.err") \
    || { echo "stats $tag failed"; tail -5 "$R/gpurun_out/stats_$tag.err"; exit 1; }
  echo "stats $tag ok"
done
for W in $PMC; do
  cfg=${W%%:*}; dt=${W##*:}
  bash scripts/pmc.sh gpurun_out/pmc_summary.json --config $cfg --ensemble-dtype $dt --shards 8 || exit 1
done
exit 0
