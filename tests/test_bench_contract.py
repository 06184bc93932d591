"""CPU: the bench line's roofline traffic comes from the committed PMC summary of the same workload and
kernel (bench.py pmc_traffic); a kernel renamed by a template change must not silently null it."""
import sys


def test_committed_pmc_summary_prices_the_default_workload(monkeypatch):
    import bench
    monkeypatch.setattr(sys, 'argv', ['bench.py'])
    args = bench.parse()
    t = bench.pmc_traffic(args)
    assert t is not None and t > 0, 'profiles PMC summary does not match %s / %s' % (
        bench.workload_key(args), bench.ENSEMBLE_KERNEL[args.ensemble_dtype])
    # HBM bytes per 50k-row ensemble launch: at least the algorithmic 19.6 MB, far below 1 GB
    assert 19.6e6 <= t < 1e9
