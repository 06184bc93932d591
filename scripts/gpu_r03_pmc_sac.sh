#!/bin/bash
# PMC passes of $PMC (scripts/profile_r03.sh), then the SAC kernel trace (scripts/sac_trace.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/sacprof" -o run -- \
  python "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --sac-steps 300 --train-epochs 0 --no-c3 --no-alt-dtypes \
  > "$R/gpurun_out/sacprof.json" 2> "$R/gpurun_out/sacprof.err") || { tail -5 gpurun_out/sacprof.err; exit 1; }
python scripts/sac_trace.py gpurun_out/sacprof/run_kernel_trace.csv > gpurun_out/sac_trace.txt 2>&1
cat gpurun_out/sac_trace.txt | head -12
STATS="" PMC="$PMC" bash scripts/profile_r03.sh || exit $?
