#!/bin/bash
# BNN.train parity (tests/test_gpu_train.py) on the in-tree library, then the BNN.train bench leg with the
# row-block step (default), the 12-launch step (MOPO_TRAIN_ROWS=0), and 16x16 weight-gradient tiles (w16).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_mopo.py -q -x -p no:cacheprovider --timeout 200 \
  --timeout-method thread > gpurun_out/train_tests.log 2>&1
rc=$?
tail -15 gpurun_out/train_tests.log
[ $rc -ne 0 ] && exit $rc
for v in 1 0 w16; do
  if [ "$v" = w16 ]; then export MOPO_TRAIN_ROWS=1 MOPO_TRAIN_WGRAD_TILE=16; else export MOPO_TRAIN_ROWS=$v; unset MOPO_TRAIN_WGRAD_TILE; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-c3 --no-alt-dtypes --sac-steps 16 --steps 3 \
    --warmup 1 --train-epochs 3 > gpurun_out/b_train_$v.json 2> gpurun_out/b_train_$v.err || { tail -5 gpurun_out/b_train_$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/b_train_$v.json')); t=d.get('model_train') or {}; print('rows=$v', t.get('value'), t.get('ms_per_epoch'))"
done
