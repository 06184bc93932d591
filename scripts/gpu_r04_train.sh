#!/bin/bash
# BNN.train parity on the in-tree library (persistent weight-gradient launch by default), then the train
# bench leg alternating the env settings in $VARS (comma-joined per variant), then a kernel trace of the leg.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -q -x -p no:cacheprovider --timeout 200 \
  --timeout-method thread > gpurun_out/train_tests.log 2>&1
rc=$?
tail -3 gpurun_out/train_tests.log
[ $rc -ne 0 ] && exit $rc
: > gpurun_out/ab_train.txt
VARS=${VARS:-"MOPO_TRAIN_WG2=1 MOPO_TRAIN_WG2=0"}
for i in 1 2; do
  for v in $VARS; do
    env ${v//,/ } timeout -k 10 200 python bench.py --no-cpu-baseline --no-c3 --no-alt-dtypes --sac-steps 16 --steps 3 --warmup 1 \
      --train-epochs 3 > gpurun_out/abt_cur.json 2> gpurun_out/abt_cur.err || { echo "bench $v failed"; tail -5 gpurun_out/abt_cur.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/abt_cur.json')); t=d['model_train']; print('$v', round(t['value']), 'steps/s', round(t['ms_per_epoch'], 2), 'ms/epoch')" >> gpurun_out/ab_train.txt
  done
done
unset MOPO_TRAIN_WG2 MOPO_TRAIN_WG2_NWX
cat gpurun_out/ab_train.txt
rm -rf gpurun_out/trace_train
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_train -o tr -- python bench.py --no-cpu-baseline \
  --no-c3 --no-alt-dtypes --sac-steps 16 --steps 3 --warmup 1 --train-epochs 2 > gpurun_out/trace_train.json 2> gpurun_out/trace_train.err
r=$?
python scripts/trace_summary.py gpurun_out/trace_train
exit $r
