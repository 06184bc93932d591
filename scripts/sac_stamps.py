"""Per-workgroup phase timestamps of the SAC row-block launches (diagnostic build: MOPO_SAC_STAMPS=1,
scripts/build_sac_variant.sh).  Runs SAC steps on synthetic pools, reads the last step's stamps and
prints, per launch (F1, F2, B1): workgroup start spread and the median / p90 / max phase durations.
Stamps: 0 start, 1 operands issued (+ head / dq prologue), 2 slabs in LDS, 3 MFMA done, 4 end (100 MHz).
usage: python scripts/sac_stamps.py [steps]"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from mopo_amd import _lib as L
    from mopo_amd.replay_pool import SimpleReplayPool
    from mopo_amd.sac import SAC
    O, A, H = 17, 6, 256
    rs = np.random.RandomState(0)
    pools = []
    for n in (5000, 20000):
        p = SimpleReplayPool(obs_dim=O, act_dim=A, max_size=n)
        p.add_samples({'observations': rs.normal(size=(n, O)), 'actions': rs.uniform(-1, 1, (n, A)),
                       'next_observations': rs.normal(size=(n, O)), 'rewards': rs.normal(size=(n, 1)),
                       'terminals': np.zeros((n, 1), bool)})
        pools.append(p)
    sac = SAC(O, A, H, batch_size=256, real_ratio=0.05, target_entropy=-3)
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    for rep in range(3):
        sac._do_training(rep * steps, pools[0], pools[1], n_steps=steps, seed=5)
        torch.cuda.synchronize()
    buf = np.zeros(4 * 1024 * 8, np.uint64)
    L.check(L.lib().mopo_sac_debug_stamps(sac._h, buf.ctypes.data, buf.size))
    st = buf.reshape(4, 1024, 8).astype(np.int64)
    nb1 = int((buf.reshape(4, 1024, 8)[2, :, 0] > 0).sum())   # B1: ncq1 x 16 row blocks x 4 (z)
    z1 = nb1 // 4                                              # blocks per z slice
    nblk = [256, 256, nb1]
    t_first = min(int(st[k, :nblk[k], 0].min()) for k in range(3))
    for k in (3,):            # the grouped-GEMM launch: blocks with a stamp (gather blocks: 0 and 4 only)
        nb = int((st[k, :, 0] > 0).sum())
        print('   loss-tail block (block 0): %.2f us long' % ((st[k, 0, 4] - st[k, 0, 0]) * 0.01))
        s = st[k, 1:nb]
        t0 = s[:, 0].min()
        us = lambda x: x * 0.01
        name = 'B2 every weight gradient + Adam + gather'
        print('%s: %d blocks, launch span %.2f us (first start at +%.2f us); start spread p50 %.2f max %.2f' % (
            name, nb, us(s[:, 4].max() - t0), us(t0 - t_first), us(np.median(s[:, 0] - t0)), us((s[:, 0] - t0).max())))
        g = s[:, 1] != 0
        for i, (a_, b_, ph) in enumerate(((0, 1, 'operands to LDS'), (1, 2, 'MFMA'), (2, 4, 'epilogue (+Adam)'))):
            d = us(s[g, b_] - s[g, a_])
            print('   %-18s p50 %5.2f  p90 %5.2f  max %5.2f us' % (ph, np.median(d), np.quantile(d, 0.9), d.max()))
    for k, name in enumerate(('F1 fwd (pi, Q(s,a))', 'F2 fwd (head + Q(s,pi), targets)', 'B1 dh1 + dq + loss tail')):
        off = z1 if k == 2 else 0   # B1: z = 0 holds the step control (block 0) and the gather blocks
        s = st[k, off:(3 * z1 if k == 2 else nblk[k]), :5]   # B1: the two (s, a) critic instances (z = 1, 2)
        us = lambda x: x * 0.01   # 100 MHz ticks -> us
        t0 = s[:, 0].min()
        print('%s: launch span %.2f us (first start at +%.2f us); start spread p50 %.2f max %.2f' % (
            name, us(s[:, 4].max() - t0), us(t0 - t_first), us(np.median(s[:, 0] - t0)), us((s[:, 0] - t0).max())))
        for i, ph in enumerate(('operands+prologue', 'slab to LDS', 'MFMA', 'epilogue')):
            d = us(s[:, i + 1] - s[:, i])
            print('   %-18s p50 %5.2f  p90 %5.2f  max %5.2f us' % (ph, np.median(d), np.quantile(d, 0.9), d.max()))
        if k == 2:
            print('   step-control block: start +%.2f us, %.2f us long' % (us(st[2, 0, 0] - t0), us(st[2, 0, 4] - st[2, 0, 0])))
            gb = st[2, 1:z1, :5]
            gb = gb[gb[:, 0] > 0]
            if len(gb):
                print('   gather blocks (%d): end +%.2f .. +%.2f us' % (len(gb), us(gb[:, 4].min() - t0), us(gb[:, 4].max() - t0)))
            prb = st[2, 3 * z1:4 * z1, :5]    # the policy-row blocks (z = 3)
            print('   policy-row blocks: start +%.2f..+%.2f us, end +%.2f..+%.2f us (launch end +%.2f)' % (
                us(prb[:, 0].min() - t0), us(prb[:, 0].max() - t0), us(prb[:, 4].min() - t0), us(prb[:, 4].max() - t0),
                us(max(prb[:, 4].max(), s[:, 4].max(), st[2, 0, 4]) - t0)))
            for i, ph in enumerate(('operands issued', 'head bwd done at', 'dh2p done at', 'end at')):
                d = us(prb[:, i + 1] - t0)
                print('      %-16s +%5.2f .. +%5.2f us (p50 +%5.2f)' % (ph, d.min(), d.max(), np.median(d)))


if __name__ == '__main__':
    main()
