#!/bin/bash
# A/B of two builds of libmopo_hip.so on one box: abv/new.so vs abv/old.so (abv/, gitignored; removed after the A/B call),
# (or the variants named in $AB: abv/<so>.so, optionally <so>:ENV=VAL to run it with one env setting), alternating bench runs (headline rollout only) so box-to-box variation cancels.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/ab.txt
for i in 1 2 3; do
  for v in ${AB:-new old}; do
    so=${v%%:*}; envs=""; [ "$so" != "$v" ] && envs=${v#*:}
    cp abv/$so.so mopo_amd/libmopo_hip.so
    env $envs timeout -k 10 120 python bench.py --no-cpu-baseline --no-c3 --sac-steps 16 --train-epochs 0 --steps 20 ${BENCH_ARGS} \
      > gpurun_out/ab_cur.json 2> gpurun_out/ab_cur.err || { echo "bench $v failed"; tail -5 gpurun_out/ab_cur.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_cur.json')); print('$v', round(d['value']/1e6,2), 'M/s', 'ens', round(d['kernel_ms_avg']['ensemble_fwd'],4), 'actor', round(d['kernel_ms_avg']['actor'],4), 'start', round(d['kernel_ms_avg'].get('start',0),4), 'post', round(d['kernel_ms_avg'].get('fakeenv_post',0),4))" >> gpurun_out/ab.txt
  done
done
cat gpurun_out/ab.txt
