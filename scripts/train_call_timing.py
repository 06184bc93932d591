"""Where one BNN.train call's time goes outside its epochs (bench.py's train-leg workload).

Times a plain call, then one with every trainer / BNN library call bracketed by device syncs, and
prints per-entry-point totals plus the host time between them.  Usage: python scripts/train_call_timing.py [epochs]
"""
import os
import sys
import time
from collections import defaultdict

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mopo_amd import _lib as L  # noqa: E402
from mopo_amd.bnn import construct_model  # noqa: E402

O, A, E, ELITES, H, N = 17, 6, 7, 5, 200, 101000


def main():
    epochs = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    rs = np.random.RandomState(5)
    X = rs.normal(size=(N, O + A)).astype(np.float32)
    Y = rs.normal(size=(N, O + 1)).astype(np.float32)
    m = construct_model(obs_dim=O, act_dim=A, hidden_dim=H, num_networks=E, num_elites=ELITES,
                        separate_mean_var=True, seed=1)
    x, y = torch.from_numpy(X).cuda(), torch.from_numpy(Y).cuda()
    np.random.seed(0)
    m.train(x, y, batch_size=256, max_epochs=1, holdout_ratio=0.2, permuted=True)
    for ep in (1, epochs):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m.train(x, y, batch_size=256, max_epochs=ep, holdout_ratio=0.2, permuted=True)
        torch.cuda.synchronize()
        print('plain call, %d epochs: %.2f ms' % (ep, (time.perf_counter() - t0) * 1e3))

    lib = L.lib()
    acc = defaultdict(float)
    names = [n for n in dir(lib) if n.startswith('mopo_bnn')]
    orig = {}
    for n in names:
        f = getattr(lib, n)
        orig[n] = f

        def wrap(*a, _f=f, _n=n):
            torch.cuda.synchronize()
            t = time.perf_counter()
            r = _f(*a)
            torch.cuda.synchronize()
            acc[_n] += time.perf_counter() - t
            return r
        setattr(lib, n, wrap)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    m.train(x, y, batch_size=256, max_epochs=epochs, holdout_ratio=0.2, permuted=True)
    torch.cuda.synchronize()
    tot = time.perf_counter() - t0
    for n, f in orig.items():
        setattr(lib, n, f)
    print('synced call, %d epochs: %.2f ms' % (epochs, tot * 1e3))
    for n, v in sorted(acc.items(), key=lambda kv: -kv[1]):
        print('  %-36s %8.3f ms' % (n, v * 1e3))
    print('  %-36s %8.3f ms' % ('(host, between library calls)', (tot - sum(acc.values())) * 1e3))


if __name__ == '__main__':
    main()
