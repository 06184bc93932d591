#!/bin/bash
# bench.py's N>1 path rehearsed on one GPU: 2 ranks over gloo (RCCL needs a GPU per rank), C2 and C4.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for cfg in C2 C4; do
  MOPO_DIST_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 5 --warmup 2 --config $cfg \
    > gpurun_out/multi_$cfg.json 2> gpurun_out/multi_$cfg.err || { echo "N=2 $cfg failed"; tail -20 gpurun_out/multi_$cfg.err; exit 1; }
  echo "N=2 $cfg ok: $(cat gpurun_out/multi_$cfg.json | head -c 300)"
done
