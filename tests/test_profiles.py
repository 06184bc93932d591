"""The committed round-5 roofline evidence is self-consistent (CPU; reads profiles/ only):
  * each profiled leg's bench line (profiles/r05_<leg>_prof_bench.json) prices the ensemble launch at an
    average that agrees within 5 % with rocprofv3's average for the full-batch launch of the same run
    (profiles/r05_<leg>_trace.json, scripts/trace_summary.py: one row per kernel and grid size);
  * bench.py reads its PMC traffic from the round-5 summary, which holds every profiled workload."""
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LEGS = ['C2_f16x3', 'C2_fp32', 'C3_bf16', 'C5_fp32', 'C5_f16x3', 'C5_bf16', 'N2_f16x3']


def _load(name):
    return json.load(open(os.path.join(ROOT, 'profiles', name)))


@pytest.mark.parametrize('leg', LEGS)
def test_bench_launch_average_matches_rocprof(leg):
    b = _load('r05_%s_prof_bench.json' % leg)
    rows = [r for r in _load('r05_%s_trace.json' % leg) if 'bnn_fwd' in r['kernel']]
    full = max(rows, key=lambda r: r['grid_threads'])
    assert full['count'] >= 50
    ms = b['kernel_ms_avg']['ensemble_fwd']
    assert ms == pytest.approx(full['avg_us'] / 1e3, rel=0.05)
    if 'roofline' in b:
        assert b['roofline']['avg_launch_ms'] == ms


def test_pmc_summary_covers_profiled_workloads():
    import bench
    assert os.path.basename(bench.PMC_SUMMARY) == 'r05_pmc_summary.json'
    w = json.load(open(bench.PMC_SUMMARY))['workloads']
    for leg in LEGS:
        b = _load('r05_%s_prof_bench.json' % leg)
        cfg, dt = leg.split('_')
        key = '%s B=%d h=%d dtype=%s' % (cfg, b['config']['rollout_batch_per_gpu'] if 'rollout_batch_per_gpu'
                                         in b['config'] else b['config']['global_batch'], b['config']['horizon'], dt)
        assert key in w, key
        ens = [k for k in w[key]['kernels'] if k.startswith('mopo::bnn_fwd')]
        assert ens and all(w[key]['kernels'][k]['hbm_bytes'] > 0 for k in ens)
    assert bench.sac_pmc_traffic() > 0
