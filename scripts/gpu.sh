#!/bin/bash
# One gpurun call, any sequence of steps (each under its own time limit; the call stops at the first
# failing step):
#   tests       the whole -m gpu suite                                  -> gpurun_out/pytest_gpu.log
#   tests:EXPR  the -m gpu tests selected by -k EXPR                    -> gpurun_out/pytest_k.log
#   bench       the default bench line                                  -> gpurun_out/bench_full.json
#   profile     kernel traces + PMC passes of every leg (gpu_profile.sh) -> gpurun_out/prof_$TAG/
#   probe       XCD placement / L2 persistence probe (scripts/micro/xcc_probe)
#   ab          headline A/B over abv/<v>.so for v in $AB (scripts/ab.sh)
#   sac_ab      SAC parity on each abv/<v>.so of $AB, then the step-time A/B (scripts/ab_sac.sh)
#   train_ab    BNN.train parity, then the train leg under each env setting of $VARS
#   train_so_ab BNN.train parity on each abv/<v>.so of $AB, then the train leg alternating them
#   env_ab      bench (SAC + headline) alternating the env settings in $VARS (comma-joined per variant)
#   stamps      SAC phase stamps from abv/sac_stamps.so (scripts/sac_stamps.py)
#   train_stamps  BNN.train rows-launch phase stamps from abv/train_stamps.so (scripts/train_timeline.py)
# usage: bash scripts/gpu.sh tests bench ;  AB="new old" bash scripts/gpu.sh sac_ab
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PYT="python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread"
keep() { cp mopo_amd/libmopo_hip.so /tmp/lib_keep.so; }
restore() { cp /tmp/lib_keep.so mopo_amd/libmopo_hip.so; }
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 1100 $PYT tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
      tail -4 gpurun_out/pytest_gpu.log ;;
    tests:*)
      timeout -k 10 900 $PYT tests -m gpu -x -q -k "${step#tests:}" > gpurun_out/pytest_k.log 2>&1; rc=$?
      tail -4 gpurun_out/pytest_k.log ;;
    bench)
      timeout -k 10 400 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err; rc=$?
      [ $rc -eq 0 ] && python scripts/bench_brief.py gpurun_out/bench_full.json gpurun_out/bench_detail.json || tail -5 gpurun_out/bench_full.err ;;
    profile)
      bash scripts/gpu_profile.sh; rc=$? ;;
    probe)
      timeout -k 10 60 ./scripts/micro/xcc_probe > gpurun_out/xcc_probe.txt 2>&1; rc=$?
      cat gpurun_out/xcc_probe.txt ;;
    ab)
      keep; bash scripts/ab.sh; rc=$?; restore ;;
    sac_ab)
      keep; rc=0
      for v in $AB; do
        so=${v%%:*}; envs=""; [ "$so" != "$v" ] && envs=${v#*:}
        cp abv/$so.so mopo_amd/libmopo_hip.so
        env $envs timeout -k 10 300 $PYT tests/test_gpu_sac.py tests/test_gpu_ref.py -q -x -k "sac or SAC" > gpurun_out/sac_tests_$so.log 2>&1
        rc=$?; echo "== $v parity rc=$rc: $(tail -1 gpurun_out/sac_tests_$so.log)"
        [ $rc -ne 0 ] && break
      done
      [ $rc -eq 0 ] && { AB="$AB_EXTRA $AB" bash scripts/ab_sac.sh; rc=$?; }
      restore ;;
    train_ab)
      timeout -k 10 300 $PYT tests/test_gpu_train.py -q -x > gpurun_out/train_tests.log 2>&1; rc=$?
      tail -3 gpurun_out/train_tests.log
      if [ $rc -eq 0 ]; then
        : > gpurun_out/ab_train.txt
        for i in 1 2; do
          for v in ${VARS:-"MOPO_TRAIN_WG2=1 MOPO_TRAIN_WG2=0"}; do
            env ${v//,/ } timeout -k 10 200 python bench.py --no-cpu-baseline --no-c3 --no-alt-dtypes --sac-steps 16 --steps 3 \
              --warmup 1 --train-epochs ${TRAIN_EPOCHS:-3} > gpurun_out/abt_cur.json 2> gpurun_out/abt_cur.err || { rc=1; tail -5 gpurun_out/abt_cur.err; break 2; }
            python -c "import json; d=json.load(open('gpurun_out/abt_cur.json')); t=d['model_train']; print('$v', round(t['value']), 'steps/s', round(t['ms_per_epoch'], 2), 'ms/epoch')" >> gpurun_out/ab_train.txt
          done
        done
        cat gpurun_out/ab_train.txt
      fi ;;
    train_so_ab)
      # BNN.train parity on each abv/<v>.so of $AB, then the train leg alternating the builds
      # AB entries: <so> or <so>:ENV=VAL[,ENV=VAL]
      keep; rc=0; : > gpurun_out/ab_train.txt
      for v in $AB; do
        so=${v%%:*}; envs=""; [ "$so" != "$v" ] && envs=${v#*:}
        cp abv/$so.so mopo_amd/libmopo_hip.so
        env ${envs//,/ } timeout -k 10 300 $PYT tests/test_gpu_train.py -q -x -k "not variants" > gpurun_out/train_tests_$so.log 2>&1
        rc=$?; echo "== $v parity rc=$rc: $(tail -1 gpurun_out/train_tests_$so.log)"
        [ $rc -ne 0 ] && break
      done
      if [ $rc -eq 0 ]; then
        for i in 1 2 3; do
          for v in $AB; do
            so=${v%%:*}; envs=""; [ "$so" != "$v" ] && envs=${v#*:}
            cp abv/$so.so mopo_amd/libmopo_hip.so
            env ${envs//,/ } timeout -k 10 200 python bench.py --no-cpu-baseline --no-c3 --no-alt-dtypes --sac-steps 16 --steps 3 --warmup 1 \
              --train-epochs ${TRAIN_EPOCHS:-3} > gpurun_out/abt_cur.json 2> gpurun_out/abt_cur.err || { rc=1; tail -5 gpurun_out/abt_cur.err; break 2; }
            python -c "import json; d=json.load(open('gpurun_out/abt_cur.json')); t=d['model_train']; print('$v', round(t['value']), 'steps/s', round(t['ms_per_epoch'], 2), 'ms/epoch')" >> gpurun_out/ab_train.txt
          done
        done
        cat gpurun_out/ab_train.txt
      fi
      restore ;;
    env_ab)
      : > gpurun_out/env_ab.txt; rc=0
      for i in 1 2 3; do
        for v in ${VARS}; do
          env ${v//,/ } timeout -k 10 150 python bench.py --no-cpu-baseline --no-c3 --no-alt-dtypes --train-epochs 0 --steps 5 \
            --warmup 2 ${BENCH_ARGS} > gpurun_out/env_ab_cur.json 2> gpurun_out/env_ab_cur.err || { rc=1; tail -5 gpurun_out/env_ab_cur.err; break 2; }
          python -c "import json; d=json.load(open('gpurun_out/env_ab_cur.json')); print('$v', 'sac', round(d['sac']['us_per_step'], 2), 'us/step', 'rollout', round(d['value']/1e6, 2), 'M/s ens', round(d['kernel_ms_avg']['ensemble_fwd'], 4))" >> gpurun_out/env_ab.txt
        done
      done
      cat gpurun_out/env_ab.txt ;;
    stamps)
      keep; cp abv/sac_stamps.so mopo_amd/libmopo_hip.so; : > gpurun_out/sac_timeline.txt; rc=0
      for v in ${VARS:-MOPO_SAC_FUSE=1}; do
        echo "== $v" >> gpurun_out/sac_timeline.txt
        env ${v//,/ } timeout -k 10 120 python scripts/sac_timeline.py >> gpurun_out/sac_timeline.txt 2>&1 || { rc=1; break; }
      done
      restore; cat gpurun_out/sac_timeline.txt ;;
    train_stamps)
      # each stamps build of $SOS (default abv/train_stamps.so) under each env setting of $VARS
      keep; : > gpurun_out/train_timeline.txt; rc=0
      for so in ${SOS:-train_stamps}; do
        cp abv/$so.so mopo_amd/libmopo_hip.so
        for v in ${VARS:-MOPO_TRAIN_STAGE=1}; do
          echo "== $so $v" >> gpurun_out/train_timeline.txt
          env ${v//,/ } timeout -k 10 120 python scripts/train_timeline.py >> gpurun_out/train_timeline.txt 2>&1 || { rc=1; break 2; }
        done
      done
      restore; cat gpurun_out/train_timeline.txt ;;
    *) echo "unknown step $step"; rc=2 ;;
  esac
  echo "== step $step rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
