#!/bin/bash
# Same-box A/B of SAC step time over .so variants: abv/<name>.so for each name in $AB (alternating runs);
# an entry <name>:ENV=VAL runs that build with one environment setting.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/ab_sac.txt
for i in 1 2 3; do
  for v in ${AB:-pr_default pr_early}; do
    so=${v%%:*}; envs=""; [ "$so" != "$v" ] && envs=${v#*:}
    cp abv/$so.so mopo_amd/libmopo_hip.so
    env $envs timeout -k 10 120 python bench.py --no-cpu-baseline --no-c3 --no-alt-dtypes --train-epochs 0 --steps 3 --warmup 2 \
      > gpurun_out/ab_sac_cur.json 2> gpurun_out/ab_sac_cur.err || { echo "bench $v failed"; tail -5 gpurun_out/ab_sac_cur.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_sac_cur.json')); print('$v', round(d['sac']['us_per_step'], 2), 'us/step')" >> gpurun_out/ab_sac.txt
  done
done
cat gpurun_out/ab_sac.txt
