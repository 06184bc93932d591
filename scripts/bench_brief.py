"""One-screen digest of a bench.py JSON line: python scripts/bench_brief.py gpurun_out/bench_full.json"""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('line bytes', len(json.dumps(d)))
if len(sys.argv) > 2:   # the detail file (bench_detail.json) has every leg in full
    d = json.load(open(sys.argv[2]))
r = d['roofline']
print('headline %.4g %s (%s) ms/step %.3f  ens %.4f ms frac %.3f traffic %s' % (
    d['value'], d['unit'], d['dtype'][:6], d['ms_per_step'], r['avg_launch_ms'], r['frac'], r.get('traffic')))
print('kernels', {k: round(v, 4) for k, v in d['kernel_ms_avg'].items()})
s = d.get('sac', {})
if s:
    print('sac %.2f us/step (frac %.3f)' % (s['us_per_step'], s['roofline']['frac'] if 'roofline' in s else s['frac']))
if 'model_train' in d:
    print('train %.0f grad-steps/s' % d['model_train']['value'])
for k, v in d.get('extra_configs', {}).items():
    rr = v.get('roofline', {})
    print('  %-18s %.4g  ens %s frac %s' % (k, v['value'], round(rr.get('avg_launch_ms', 0), 4), round(rr.get('frac', 0), 3)))
for k, v in d.get('headline_other_dtypes', {}).items():
    print('  alt %-14s %.4g  ens %.4f frac %.3f' % (k, v['value'], v['roofline']['avg_launch_ms'], v['roofline']['frac']))
for k, v in d.get('legs', {}).items():
    print('  leg %-18s %.4g  ens %s frac %s' % (k, v['value'], v['ms'], v['frac']))
for k in ('cpu_baseline', 'cpu_baseline_1core', 'cpu_baseline_sac', 'cpu_baseline_train'):
    if d.get(k):
        print('  %s %.4g %s' % (k, d[k]['value'], d[k]['unit']))
