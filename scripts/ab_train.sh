#!/bin/bash
# A/B of BNN.train grad-steps/s over the libraries in $AB (ab/<so>.so), alternating runs on one box,
# after tests/test_gpu_train.py on each (a failing variant is skipped).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
cp mopo_amd/libmopo_hip.so /tmp/lib_keep_t.so
ok=""
for v in $AB; do
  cp ab/$v.so mopo_amd/libmopo_hip.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -q -x -p no:cacheprovider --timeout 200 \
    --timeout-method thread > gpurun_out/train_tests_$v.log 2>&1
  rc=$?
  echo "== $v tests rc=$rc"; tail -1 gpurun_out/train_tests_$v.log
  if [ $rc -eq 0 ]; then ok="$ok $v"; elif [ $rc -ne 1 ]; then cp /tmp/lib_keep_t.so mopo_amd/libmopo_hip.so; exit $rc; fi
done
: > gpurun_out/ab_train.txt
for i in 1 2 3; do
  for v in $ok; do
    cp ab/$v.so mopo_amd/libmopo_hip.so
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-c3 --no-alt-dtypes --sac-steps 16 --steps 3 --warmup 1 \
      --train-epochs 3 > gpurun_out/abt_cur.json 2> gpurun_out/abt_cur.err || { echo "bench $v failed"; tail -5 gpurun_out/abt_cur.err; break 2; }
    python -c "import json; d=json.load(open('gpurun_out/abt_cur.json')); t=d['model_train']; print('$v', round(t['value']), 'steps/s', round(t['ms_per_epoch'], 2), 'ms/epoch')" >> gpurun_out/ab_train.txt
  done
done
cp /tmp/lib_keep_t.so mopo_amd/libmopo_hip.so
cat gpurun_out/ab_train.txt
