"""Timeline of one BNN.train minibatch step's rows launch (train_rows_kernel) from the per-workgroup stamps
of a MOPO_TRAIN_STAMPS=1 build: the p50 / max of each phase stamp, us after the step's first workgroup start.
The epoch holds whole minibatches only, so the stamps are a graph-replayed full step's.
usage: python scripts/train_timeline.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from mopo_amd import _lib as L
    from mopo_amd.bnn import construct_model
    O, A, E, H = 17, 6, 7, 200
    N = 256 * 64 + 1000                       # 64 full minibatches after the 1000-row holdout
    rs = np.random.RandomState(0)
    X = rs.normal(size=(N, O + A)).astype(np.float32)
    Y = rs.normal(size=(N, O + 1)).astype(np.float32)
    m = construct_model(obs_dim=O, act_dim=A, hidden_dim=H, num_networks=E, num_elites=5, separate_mean_var=True,
                        seed=1)
    x, y = torch.from_numpy(X).cuda(), torch.from_numpy(Y).cuda()
    np.random.seed(0)
    m.train(x, y, batch_size=256, max_epochs=2, holdout_ratio=0.2, permuted=True)   # holdout min(0.2 N, 1000) = 1000
    torch.cuda.synchronize()
    buf = np.zeros(2048 * 8, np.uint64)
    L.check(L.lib().mopo_bnn_train_debug_stamps(buf.ctypes.data, buf.size))
    st = buf.reshape(2048, 8).astype(np.int64)
    nrb = 16
    nrw = 8 * nrb * ((E + 7) // 8)
    nblk = int(np.nonzero(st[:, 0])[0].max()) + 1
    t0 = st[:nblk, 0][st[:nblk, 0] > 0].min()
    us = lambda v: (v - t0) * 0.01
    rows = [b for b in range(nrw) if (b & 7) + 8 * ((b >> 3) // nrb) < E]
    def show(name, idx, cols, labels):
        for c, lab in zip(cols, labels):
            v = np.array([us(st[b, c]) for b in idx if st[b, c] > 0])
            if len(v):
                print('%-8s %-22s p50 %7.2f  min %7.2f  max %7.2f  (n=%d)' % (name, lab, np.median(v), v.min(), v.max(), len(v)))
    print('rows launch, %d row blocks, us' % len(rows))
    show('rows', rows, range(8), ['start', 'gather done', 'layer 0', 'hidden + heads', 'loss + dY',
                                  'bwd l4', 'bwd l3, l2', 'bwd l1 (end)'])

if __name__ == '__main__':
    main()
