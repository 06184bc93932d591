#!/bin/bash
# One gpurun call: GPU parity tests, then a short bench (no CPU legs) and, with DIST=1, a
# two-rank gloo rehearsal of the multi-GPU bench path on the one GPU.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
brc=$?
cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
if [ $brc -ne 0 ]; then echo "bench rc=$brc"; exit $brc; fi
if [ -n "$DIST" ]; then
  MOPO_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --sac-steps 100 \
    > gpurun_out/bench_dist.json 2> gpurun_out/bench_dist.err
  drc=$?
  cat gpurun_out/bench_dist.json; tail -3 gpurun_out/bench_dist.err
  exit $drc
fi
