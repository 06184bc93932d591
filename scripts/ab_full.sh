#!/bin/bash
# Whole-bench A/B of library builds on one box: abv/<v>.so for v in $AB (default "base new"), alternating,
# $REPS rounds (default 2); every leg's value / frac, SAC us/step and BNN.train grad-steps/s per run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/ab_full.txt
cp mopo_amd/libmopo_hip.so /tmp/lib_keep_full.so
rc=0
for i in $(seq ${REPS:-2}); do
  for v in ${AB:-base new}; do
    cp abv/$v.so mopo_amd/libmopo_hip.so
    timeout -k 10 240 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/abf_cur.json 2> gpurun_out/abf_cur.err \
      || { echo "bench $v failed"; tail -5 gpurun_out/abf_cur.err; rc=1; break 2; }
    python - "$v" >> gpurun_out/ab_full.txt <<'EOF'
import json, sys
d = json.loads(open('gpurun_out/abf_cur.json').read().strip().splitlines()[-1])
legs = ' '.join('%s=%.4g/%s' % (k, v['value'], v['frac']) for k, v in d.get('legs', {}).items())
print('%-6s C2 %.4g frac %.4f ens %.4f | sac %.2f us | train %s | %s' % (
    sys.argv[1], d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['sac']['us_per_step'],
    d.get('model_train', {}).get('value'), legs))
EOF
  done
done
cp /tmp/lib_keep_full.so mopo_amd/libmopo_hip.so
cat gpurun_out/ab_full.txt
exit $rc
