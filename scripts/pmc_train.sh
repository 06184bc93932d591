#!/bin/bash
# PMC passes over the BNN.train bench leg (one counter group per rocprofv3 run, --kernel-trace only besides
# --pmc): HBM bytes, MFMA busy, wait share, L2 hit/miss of train_rows_kernel and the weight-gradient launch.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --sac-steps 16 --no-c3 --no-alt-dtypes --train-epochs 1 --prof-steps 1"
cd /tmp
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES" "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_INSTS_MFMA"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_train/pmc$i" -o run -- python "$R/bench.py" $ARGS > "$R/gpurun_out/pmc_train_$i.log" 2>&1
  rc=$?
  echo "pass $i ($C) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$R/gpurun_out/pmc_train_$i.log"; exit $rc; fi
done
cd "$R" && python scripts/pmc_counters.py gpurun_out/pmc_train train_
