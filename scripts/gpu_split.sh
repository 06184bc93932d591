#!/bin/bash
# One gpurun call: split-bf16 ensemble parity tests, then short headline benches per ensemble dtype.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_rollout.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "${TESTK:-split or bf16x6}" > gpurun_out/pytest_split.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_split.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
for dt in ${DTYPES:-fp32 bf16x6 bf16x3}; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-c3 --train-epochs 0 --sac-steps 50 --ensemble-dtype $dt > gpurun_out/bench_$dt.json 2> gpurun_out/bench_$dt.err
  brc=$?
  if [ $brc -ne 0 ]; then tail -5 gpurun_out/bench_$dt.err; echo "bench rc=$brc"; exit $brc; fi
  python -c "import json; d=json.load(open('gpurun_out/bench_$dt.json')); print('$dt', d['value'], d['kernel_ms_avg'])"
done
