"""CPU: the bench line's contract -- its headline dtype is the one the product runs, and its roofline
traffic comes from the committed PMC summary of the same workload (bench.py pmc_traffic)."""
import sys


def test_headline_dtype_is_the_product_default(monkeypatch):
    import inspect

    import bench
    from mopo_amd.bnn import DEFAULT_ENSEMBLE_DTYPE
    from mopo_amd.mopo import MOPO
    monkeypatch.setattr(sys, 'argv', ['bench.py'])
    args = bench.parse()
    assert args.ensemble_dtype == DEFAULT_ENSEMBLE_DTYPE
    # MOPO builds its ensemble with DEFAULT_ENSEMBLE_DTYPE unless ensemble_dtype is passed
    assert inspect.signature(MOPO.__init__).parameters['ensemble_dtype'].default is None
    assert 'DEFAULT_ENSEMBLE_DTYPE' in inspect.getsource(MOPO.__init__)


def test_committed_pmc_summary_prices_the_measured_workloads(monkeypatch):
    import bench
    for argv, lo in ((['bench.py'], 19.6e6), (['bench.py', '--ensemble-dtype', 'fp32'], 19.6e6),
                     (['bench.py', '--config', 'N2'], 31.7e6)):
        monkeypatch.setattr(sys, 'argv', argv)
        args = bench.parse()
        t = bench.pmc_traffic(args)
        assert t is not None and t > 0, 'profiles PMC summary has no pass for %s' % bench.workload_key(args)
        # HBM bytes per ensemble launch: at least the algorithmic bytes, far below 1 GB
        alg = bench.ensemble_bytes(args.batch, bench.CONFIGS[args.config], args.ensemble_dtype)
        assert alg >= lo * 0.9 and alg * 0.9 <= t < 1e9, (bench.workload_key(args), alg, t)


def test_cpu_baseline_median_of_five_after_warmup():
    """every CPU-baseline figure is the median of >= 5 timed runs after 1 warm-up."""
    import bench
    calls = []

    def fn():
        calls.append(1)
        return 10, 0.5 + 0.1 * len(calls)
    med, runs, units, secs = bench.median_runs(fn)
    assert len(calls) == 1 + bench.CPU_RUNS and len(runs) == bench.CPU_RUNS >= 5
    assert med == sorted(runs)[len(runs) // 2] and units == 10 * bench.CPU_RUNS
    run = bench.cpu_rollout_leg(64, 2, 'walker2d', 5.0, env_rows=500)   # the oracle rollout leg, tiny
    n, dt = run()
    assert 0 < n <= 128 and dt > 0


def test_roofline_names_the_dispatched_ensemble_kernel():
    """The roofline's kernel is the one csrc/bnn.hip launch_bnn_fwd dispatches at the config's width: the LDS ring
    at H <= 256 (bf16x6: P = 3, f16x3: P = 2), the column-half f16h kernel for f16x3 at H = 400, the split bf16
    kernel for bf16x6 at H = 400; the executed-flop fraction counts every MFMA product."""
    import bench
    ms, rows = 0.5, 50000
    r = bench.roofline_of('bf16x6', rows, ms, bench.FLOP_BNN_ROW, 200)
    assert r['kernel'].startswith('bnn_fwd_ring_kernel<P=3>')
    assert abs(r['frac'] - 6 * rows * bench.FLOP_BNN_ROW / (ms * 1e-3) / 1e12 / bench.BF16_PEAK_TFLOPS) < 1e-12
    assert bench.roofline_of('f16x3', rows, ms, bench.FLOP_BNN_ROW, 200)['kernel'].startswith('bnn_fwd_ring_kernel<P=2>')
    assert bench.roofline_of('f16x3', rows, ms, bench.FLOP_BNN_ROW, 400)['kernel'].startswith('bnn_fwd_f16h_kernel')
    assert bench.roofline_of('bf16x6', rows, ms, bench.FLOP_BNN_ROW, 400)['kernel'].startswith('bnn_fwd_bf16_kernel<P=3>')
    assert bench.roofline_of('fp32', rows, ms)['kernel'].startswith('bnn_fwd_kernel')
