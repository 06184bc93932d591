#!/bin/bash
# rocprofv3 kernel stats of the BNN.train bench leg (row-block step).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/trainprof" -o run -- \
  python "$R/bench.py" --no-cpu-baseline --no-c3 --no-alt-dtypes --sac-steps 16 --steps 3 --warmup 1 --train-epochs 2 \
  > "$R/gpurun_out/trainprof.json" 2> "$R/gpurun_out/trainprof.err" || { tail -5 "$R/gpurun_out/trainprof.err"; exit 1; }
cd "$R" && f=$(find gpurun_out/trainprof -name '*kernel_stats.csv' | head -1) && head -20 "$f" | cut -c1-180
