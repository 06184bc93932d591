#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the ensemble launch for each build in $AB (abv/<name>.so), one PMC pass each.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp MOPO_ROLLOUT_SPLIT=1
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --sac-steps 16 --no-c3 --no-alt-dtypes --train-epochs 0 --prof-steps 1 ${BENCH_ARGS}"
for v in ${AB:-new old}; do
  cp abv/$v.so mopo_amd/libmopo_hip.so
  for C in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && timeout -k 10 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$R/gpurun_out/pmcab_${v}_$C" -o run -- python "$R/bench.py" $ARGS > "$R/gpurun_out/pmcab_${v}_$C.log" 2>&1) || { echo "pmc $v $C failed"; exit 1; }
    python - "$R/gpurun_out/pmcab_${v}_$C/run_counter_collection.csv" "$v" "$C" <<'PY'
import csv, sys, collections
tot = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    if 'bnn_fwd' in r['Kernel_Name']:
        tot[r['Dispatch_Id']] += float(r['Counter_Value'])
vals = list(tot.values())
print(sys.argv[2], sys.argv[3], 'dispatches', len(vals), 'avg KB', round(sum(vals) / max(len(vals), 1), 1))
PY
  done
done
