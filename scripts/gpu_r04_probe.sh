#!/bin/bash
# XCD placement / L2 persistence probe, the BNN.train A/B ($VARS) and PMC passes over the train leg.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 60 ./scripts/micro/xcc_probe > gpurun_out/xcc_probe.txt 2>&1 || { cat gpurun_out/xcc_probe.txt; exit 1; }
cat gpurun_out/xcc_probe.txt
VARS="MOPO_TRAIN_WG2=1 MOPO_TRAIN_WG2_ORDER=1" bash scripts/gpu_r04_train.sh > gpurun_out/train_ab.log 2>&1 || { tail -20 gpurun_out/train_ab.log; exit 1; }
grep -E "passed|failed|steps/s" gpurun_out/train_ab.log
bash scripts/pmc_train.sh
