"""Diagnostic: device SAC (perf-mode streams) vs the f64 oracle after n steps, for several n."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from oracle import replay_pool as opool, rng as orng, sac as osac
from mopo_amd.replay_pool import SimpleReplayPool
from mopo_amd.sac import SAC
O, A, seed = 17, 6, 0x5eed
rs = np.random.RandomState(3)
pools = []
for rows in (3000, 5000):
    s = {'observations': rs.normal(size=(rows, O)).astype(np.float32), 'actions': rs.uniform(-1, 1, (rows, A)).astype(np.float32),
         'next_observations': rs.normal(size=(rows, O)).astype(np.float32), 'rewards': rs.normal(size=(rows, 1)).astype(np.float32),
         'terminals': rs.uniform(size=(rows, 1)) < 0.05}
    p = SimpleReplayPool(obs_dim=O, act_dim=A, max_size=rows); p.add_samples(s)
    q = opool.Pool(O, A, rows); q.add_samples(s)
    pools.append((p, q))
for nsteps in (1, 2, 10, 50, 200):
    sac = SAC(O, A, 256, batch_size=256, real_ratio=0.05, target_entropy=-3, seed=seed)
    p0, la0 = sac.get_params()
    flat0 = p0.cpu().numpy().astype(np.float64)
    P0, off = [], 0
    for sh in osac.param_shapes(O, A, 256):
        P0.append(flat0[off:off + int(np.prod(sh))].reshape(sh)); off += int(np.prod(sh))
    sac._do_training(0, pools[0][0], pools[1][0], n_steps=nsteps, seed=seed)
    torch.cuda.synchronize()
    st = osac.SACState(P0, log_alpha=float(la0.item()))
    for k in range(nsteps):
        idx = orng.sac_batch_indices(256, 12, 3000, 5000, seed, k)
        e, m = pools[0][1].batch_by_indices(idx[:12]), pools[1][1].batch_by_indices(idx[12:])
        b = {f: np.concatenate([e[f], m[f]]).astype(np.float64) for f in e}
        lg = osac.sac_step(st, b, orng.sac_noise(256, A, seed, k, 0).astype(np.float64),
                           orng.sac_noise(256, A, seed, k, 1).astype(np.float64), target_entropy=-3.0)
    dl = sac.logs()
    flat = lambda xs: np.concatenate([np.asarray(x, np.float64).ravel() for x in xs])
    ref = np.append(flat(st.params), st.log_alpha)
    dev = sac.state_dict()['params'].cpu().numpy().astype(np.float64)
    err = np.abs(dev - ref) / (1 + np.abs(ref))
    i = int(err.argmax())
    print('steps %3d: params max %.3g (idx %d: dev %.6g ref %.6g p50 %.3g p99 %.3g); q1 loss dev %.6g ref %.6g; pi loss dev %.6g ref %.6g' % (
        nsteps, err.max(), i, dev[i], ref[i], np.median(err), np.quantile(err, 0.99), dl['Q/q1_loss'], lg['Q/q1_loss'],
        dl['policy_loss'], lg['pi_loss']), flush=True)
