"""GPU: the overlapped multi-rank rollout path (per-step staging blocks, async all-gather,
mopo_pool_add_blocks) reproduces a single-process rollout over the concatenated shards bit-exactly.

Two ranks share the one GPU of the test box over gloo (the driver's 8-GPU runs use RCCL); with
uid_offset = rank * B each rank's rows are rows [rB, (r+1)B) of the single-process rollout (Philox
streams are keyed by the global row id), and the pool order is step-major, then rank-major."""
import os
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
O, A, HZ = 17, 6, 3


def _setup():
    import torch
    from mopo_amd.bnn import construct_model
    from mopo_amd.rollout import init_sac_params
    rs = np.random.RandomState(0)
    env = torch.from_numpy(rs.normal(size=(5000, O)).astype(np.float32)).cuda()
    m = construct_model(obs_dim=O, act_dim=A, hidden_dim=200, num_networks=7, num_elites=5, separate_mean_var=True,
                        seed=1)
    m.set_elites([0, 1, 2, 3, 4])
    pi = torch.from_numpy(init_sac_params(O, A, 256, seed=2)).cuda()
    return m, env, pi


def _fields(pool):
    n = pool.size
    return {k: v[:n].cpu().numpy() for k, v in pool.fields.items()}


def _worker(rank, world, port, out, B, backend='gloo'):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY='0')
    torch.cuda.set_device(0)
    dist.init_process_group(backend, rank=rank, world_size=world)
    from mopo_amd.distributed import DistributedRollout
    from mopo_amd.replay_pool import SimpleReplayPool
    m, env, pi = _setup()
    pool = SimpleReplayPool(obs_dim=O, act_dim=A, max_size=10 * B * world)
    dr = DistributedRollout(m, B, HZ, O, A)
    for ep in range(2):  # two rollouts: the second appends after the first (ptr advanced on the device)
        counts = dr.run(env, pi, pool, 0, 1.0, [0, 1, 2, 3, 4], seed=88, epoch=ep)
    torch.cuda.synchronize()
    extra = {}
    if backend == 'nccl':
        # the other collectives of the sharded loop, through RCCL: the ensemble's packed device image, the
        # SAC state, numpy's global stream and the model-training metrics (rank 0 is the source)
        from mopo_amd.distributed import broadcast_metrics, broadcast_model, broadcast_numpy_rng, broadcast_sac
        from mopo_amd.sac import SAC
        before = m.export_packed().cpu().numpy()
        broadcast_model(m)
        extra['model_same'] = np.array(np.array_equal(before, m.export_packed().cpu().numpy()))
        sac = SAC(O, A, 256, batch_size=64)
        p0 = sac.get_params()[0].cpu().numpy()
        broadcast_sac(sac)
        extra['sac_same'] = np.array(np.array_equal(p0, sac.get_params()[0].cpu().numpy()))
        np.random.seed(123)
        st = np.random.get_state()[1].copy()
        broadcast_numpy_rng()
        extra['rng_same'] = np.array(np.array_equal(st, np.random.get_state()[1]))
        extra['metrics_same'] = np.array(broadcast_metrics({'val_loss': 0.25}) == {'val_loss': 0.25})
        extra['backend'] = np.array(dist.get_backend())
    if rank == 0:
        np.savez(out, counts=counts.cpu().numpy(), **_fields(pool), **extra)
    dist.barrier()
    dist.destroy_process_group()


def test_rccl_rank_runs_the_sharded_rollout_and_broadcasts():
    """The RCCL branch on hardware: one rank with backend 'nccl' (RCCL) runs the overlapped rollout (its
    per-step all-gathers through RCCL) into a pool identical to a single-process rollout, and every
    broadcast of the sharded training loop (model image, SAC state, numpy stream, metrics) round-trips.
    (The test box has one GPU and RCCL takes one GPU per rank; the 2-rank data path is covered over gloo
    above and multi-GPU by the driver's scaling runs.)"""
    import torch
    import torch.multiprocessing as mp
    from mopo_amd.replay_pool import SimpleReplayPool
    from mopo_amd.rollout import ModelRollout
    B = 4500
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, 'r0.npz')
        mp.start_processes(_worker, args=(1, 29500 + os.getpid() % 1000, out, B, 'nccl'), nprocs=1, join=True,
                           start_method='spawn')
        got = dict(np.load(out))
    assert str(got['backend']) == 'nccl'
    for k in ('model_same', 'sac_same', 'rng_same', 'metrics_same'):
        assert bool(got[k]), k
    m, env, pi = _setup()
    pool = SimpleReplayPool(obs_dim=O, act_dim=A, max_size=10 * B)
    ro = ModelRollout(m, B, HZ)
    for ep in range(2):
        steps = ro.run(env, pi, pool, B, HZ, 0, 1.0, [0, 1, 2, 3, 4], seed=88, epoch=ep)
    torch.cuda.synchronize()
    ref = _fields(pool)
    np.testing.assert_array_equal(got['counts'], steps.cpu().numpy())
    for k in ref:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)


@pytest.mark.parametrize('B', [700, 4500])  # 4500 rows per rank: the split (two-stream) staged rollout
def test_overlapped_allgather_matches_single_process(B):
    import torch
    import torch.multiprocessing as mp
    from mopo_amd.replay_pool import SimpleReplayPool
    from mopo_amd.rollout import ModelRollout
    world = 2
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, 'r0.npz')
        mp.start_processes(_worker, args=(world, 29600 + os.getpid() % 1000 + B % 7, out, B), nprocs=world, join=True,
                           start_method='spawn')
        got = dict(np.load(out))
    m, env, pi = _setup()
    pool = SimpleReplayPool(obs_dim=O, act_dim=A, max_size=10 * B * world)
    ro = ModelRollout(m, world * B, HZ)
    for ep in range(2):
        steps = ro.run(env, pi, pool, world * B, HZ, 0, 1.0, [0, 1, 2, 3, 4], seed=88, epoch=ep)
    torch.cuda.synchronize()
    ref = _fields(pool)
    np.testing.assert_array_equal(got['counts'], steps.cpu().numpy())
    for k in ref:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)


# ---- the training loop itself sharded: MOPO.train with torch.distributed initialised ---------------
def _mopo(data_path, B):
    from mopo_amd.config import get_params
    from mopo_amd.loader import restore_pool
    from mopo_amd.mopo import from_config
    from mopo_amd.replay_pool import SimpleReplayPool
    from mopo_amd.static import static_fns
    pool = SimpleReplayPool(obs_dim=O, act_dim=A, max_size=int(1e5))
    restore_pool(pool, data_path)
    np.random.seed(0)   # numpy's global stream drives the model training loop (bnn.py:369-503)
    return from_config(get_params('examples.config.d4rl.halfcheetah_mixed'), pool, static_fns['halfcheetah'],
                       rollout_batch_size=B, epoch_length=40, model_train_freq=40)


def _state(algo):
    p, la = algo._sac.get_params()
    mp_ = algo._model_pool
    return dict(sac=p.cpu().numpy(), log_alpha=np.float32(la.item()), target=algo._sac.get_target().cpu().numpy(),
                bnn=algo._model.export_packed().cpu().numpy(), elites=np.array(algo._model._model_inds),
                # every rank's host model state (import_packed used to leave it stale / None)
                bnn_mats=algo._model.flat_params(), bnn_holdout=np.asarray(algo._model._holdout_losses),
                bnn_scaler_mu=np.asarray(algo._model.scaler.cached_mu),
                **{'pool_' + k: v[:mp_.size].cpu().numpy() for k, v in mp_.fields.items()})


def _mopo_worker(rank, world, port, data_path, out, B):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY='0')
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    algo = _mopo(data_path, B)
    assert algo._world == world
    diags = list(algo.train(2))
    torch.cuda.synchronize()
    st = _state(algo)
    st['mean_rollout_length'] = np.array([d['model/mean_rollout_length'] for d in diags])
    np.savez(out % rank, **st)
    dist.barrier()
    dist.destroy_process_group()


def test_mopo_train_sharded_matches_single_process(tmp_path):
    """Two ranks (gloo on the one GPU; RCCL on a real node) run MOPO.train(2) with the rollout rows
    sharded: rank 0 alone trains the ensemble and broadcasts its packed device image; both ranks end
    with identical model pools, SAC states and ensembles (packed images, elites), and those equal a
    single-process MOPO.train(2) of the same config bit for bit."""
    import torch
    import torch.multiprocessing as mp
    rs = np.random.RandomState(0)
    n = 3000
    obs = rs.normal(size=(n, O)).astype(np.float32)
    data = str(tmp_path / 'd.npz')
    np.savez(data, observations=obs, actions=rs.uniform(-1, 1, (n, A)).astype(np.float32),
             next_observations=obs + 0.1 * rs.normal(size=(n, O)).astype(np.float32),
             rewards=rs.normal(size=n).astype(np.float32), terminals=np.zeros(n, bool))
    B, world = 2400, 2
    out = str(tmp_path / 'r%d.npz')
    mp.start_processes(_mopo_worker, args=(world, 29700 + os.getpid() % 1000, data, out, B), nprocs=world, join=True,
                       start_method='spawn')
    r0, r1 = dict(np.load(out % 0)), dict(np.load(out % 1))
    for k in r0:
        np.testing.assert_array_equal(r0[k], r1[k], err_msg='ranks differ: ' + k)
    algo = _mopo(data, B)
    diags = list(algo.train(2))
    torch.cuda.synchronize()
    single = _state(algo)
    np.testing.assert_array_equal(r0['mean_rollout_length'], [d['model/mean_rollout_length'] for d in diags])
    bad = {k: float(np.max(np.abs(r0[k].astype(np.float64) - single[k]))) for k in single
           if not np.array_equal(r0[k], single[k])}
    assert not bad, 'sharded != single process: %s' % bad
