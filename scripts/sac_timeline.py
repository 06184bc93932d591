"""Timeline of one SAC step from the per-workgroup stamps of a MOPO_SAC_STAMPS=1 build (both the separate
F2 / B1 launches and the fused F2 + B1 launch): per workgroup group, start and end (p50 / max, us after the
step's first F1 start), and for the fused B1 blocks when their prefetch was issued and their wait ended.
Stamp slots: 0 F1, 1 F2 (or the fused F2 + B1), 2 B1, 3 B2.  usage: python scripts/sac_timeline.py"""
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
    for rep in range(3):
        sac._do_training(rep * 64, pools[0], pools[1], n_steps=64, seed=5)
        torch.cuda.synchronize()
    buf = np.zeros(4 * 1024 * 8, np.uint64)
    L.check(L.lib().mopo_sac_debug_stamps(sac._h, buf.ctypes.data, buf.size))
    st = buf.reshape(4, 1024, 8).astype(np.int64)
    t0 = st[0, :256, 0].min()
    us = lambda x: (x - t0) * 0.01
    fused = (st[1, 256:512, 0] > 0).any() or (st[0, 256:768, 0] > 0).any()
    groups = [('F1', st[0, :256])]
    if (st[0, 256:768, 0] > 0).any():     # F1 + F2 + B1 in one launch: all in slot 0
        groups = [('F1 (fused)', st[0, :256]), ('F2 (fused)', st[0, 256:512]), ('B1 step/gather (fused)', st[0, 512:576]),
                  ('B1 critic dh1 (fused)', st[0, 576:704]), ('B1 policy rows (fused)', st[0, 704:768])]
    elif fused:
        groups += [('F2 (fused)', st[1, :256]), ('B1 step/gather (fused)', st[1, 256:320]),
                   ('B1 critic dh1 (fused)', st[1, 320:448]), ('B1 policy rows (fused)', st[1, 448:512])]
    else:
        groups += [('F2', st[1, :256]), ('B1 step/gather', st[2, :64]), ('B1 critic dh1', st[2, 64:192]),
                   ('B1 policy rows', st[2, 192:256])]
    if os.environ.get('MOPO_SAC_FUSE') == '3':   # the whole step in slot 0: B2 blocks from 768 on
        groups += [('B2 loss tail (fused)', st[0, 768:769]), ('B2 tiles (fused)', st[0, 769:1024])]
    else:
        nb = int((st[3, :, 0] > 0).sum())
        groups += [('B2 loss tail', st[3, :1]), ('B2 tiles', st[3, 1:nb])]
    print('SAC step timeline (%s), us after the first F1 start' % (os.environ.get('MOPO_SAC_FUSE', 'default fusion')))
    for name, g in groups:
        g = g[g[:, 0] > 0]
        if not len(g):
            continue
        line = '%-26s start p50 %6.2f max %6.2f | end p50 %6.2f max %6.2f' % (
            name, np.median(us(g[:, 0])), us(g[:, 0]).max(), np.median(us(g[:, 4])), us(g[:, 4]).max())
        if fused and 'fused' in name and (g[:, 5] > 0).any():
            line += ' | prefetch issued p50 %6.2f, wait done p50 %6.2f max %6.2f' % (
                np.median(us(g[:, 5])), np.median(us(g[:, 6])), us(g[:, 6]).max())
        print(line)


if __name__ == '__main__':
    main()
