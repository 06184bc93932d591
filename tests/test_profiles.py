"""The committed roofline evidence of the round bench.py prices from is self-consistent (CPU; reads profiles/ only):
  * each profiled leg's bench line (profiles/<round>_<leg>_prof_bench.json) prices the ensemble launch at an
    average that agrees within 5 % with rocprofv3's average for the full-batch launch of the same run
    (profiles/<round>_<leg>_trace.json, scripts/trace_summary.py: one row per kernel and grid size);
  * bench.py reads its PMC traffic from that round's summary, which holds every profiled workload.
<round> is the prefix of bench.PMC_SUMMARY, so the checks follow the summary bench.py uses."""
import glob
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _round():
    import bench
    return os.path.basename(bench.PMC_SUMMARY).split('_')[0]


def _legs():
    rnd = _round()
    return sorted(os.path.basename(f)[len(rnd) + 1:-len('_prof_bench.json')]
                  for f in glob.glob(os.path.join(ROOT, 'profiles', '%s_*_prof_bench.json' % rnd)))


def _load(name):
    return json.load(open(os.path.join(ROOT, 'profiles', name)))


def test_profiled_legs_present():
    assert {'C2_f16x3', 'C2_fp32'} <= set(_legs())


@pytest.mark.parametrize('leg', _legs())
def test_bench_launch_average_matches_rocprof(leg):
    rnd = _round()
    b = _load('%s_%s_prof_bench.json' % (rnd, leg))
    rows = [r for r in _load('%s_%s_trace.json' % (rnd, leg)) if 'bnn_fwd' in r['kernel']]
    full = max(rows, key=lambda r: r['grid_threads'])
    assert full['count'] >= 50
    ms = b['kernel_ms_avg']['ensemble_fwd']
    assert ms == pytest.approx(full['avg_us'] / 1e3, rel=0.05)
    if 'roofline' in b:
        assert b['roofline']['avg_launch_ms'] == pytest.approx(ms, rel=1e-3)


def test_pmc_summary_covers_profiled_workloads():
    import bench
    rnd = _round()
    w = json.load(open(bench.PMC_SUMMARY))['workloads']
    for leg in _legs():
        b = _load('%s_%s_prof_bench.json' % (rnd, leg))
        cfg, dt = leg.split('_')
        key = '%s B=%d h=%d dtype=%s' % (cfg, b['config']['rollout_batch_per_gpu'] if 'rollout_batch_per_gpu'
                                         in b['config'] else b['config']['global_batch'], b['config']['horizon'], dt)
        assert key in w, key
        ens = [k for k in w[key]['kernels'] if k.startswith('mopo::bnn_fwd')]
        assert ens and all(w[key]['kernels'][k]['hbm_bytes'] > 0 for k in ens)
    assert bench.sac_pmc_traffic() > 0
