"""Host time to enqueue one BNN.train epoch (mopo_bnn_train_epoch: 49 graph launches + the partial step) vs
its device time, at bench.py's train-leg size.  A host-bound epoch leaves the GPU waiting for launches."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mopo_amd import _lib as L  # noqa: E402
from mopo_amd.bnn import construct_model  # noqa: E402

O, A, E, H, N = 17, 6, 7, 200, 100000


def main():
    rs = np.random.RandomState(5)
    x = torch.from_numpy(rs.normal(size=(N, O + A)).astype(np.float32)).cuda()
    y = torch.from_numpy(rs.normal(size=(N, O + 1)).astype(np.float32)).cuda()
    m = construct_model(obs_dim=O, act_dim=A, hidden_dim=H, num_networks=E, num_elites=5, separate_mean_var=True, seed=1)
    t = m._trainer(256, 1000)
    m._train_params(t, m.get_params())
    L.check(L.lib().mopo_bnn_train_fit_scaler(t, L.ptr(x), N, None))
    idxs = torch.from_numpy(rs.randint(N, size=E * N).astype(np.int32)).cuda()
    for rep in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        L.check(L.lib().mopo_bnn_train_epoch(t, L.ptr(x), L.ptr(y), L.ptr(idxs), N, 256, None))
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print('epoch %d: host enqueue %.2f ms, enqueue + device %.2f ms' % (rep, (t1 - t0) * 1e3, (t2 - t0) * 1e3))
    # two epochs back to back: the second's enqueue overlaps the first's execution
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(2):
        L.check(L.lib().mopo_bnn_train_epoch(t, L.ptr(x), L.ptr(y), L.ptr(idxs), N, 256, None))
    torch.cuda.synchronize()
    print('two epochs back to back: %.2f ms' % ((time.perf_counter() - t0) * 1e3))


if __name__ == '__main__':
    main()
