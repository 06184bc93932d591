"""CPU (gloo, world_size 2): the multi-GPU rollout's collective leg -- all-gather of staged
transitions + per-step counts and reassembly in the single-GPU global order."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

O, A, H, B = 17, 6, 3, 5


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def staging_for(rank):
    """Rank-local staging: step i rows carry (rank, step, row) in their observation columns."""
    n = H * B
    f = {'observations': torch.zeros(n, O), 'actions': torch.full((n, A), float(rank)),
         'rewards': torch.zeros(n, 1), 'terminals': torch.zeros(n, 1, dtype=torch.bool),
         'next_observations': torch.zeros(n, O)}
    for i in range(H):
        for r in range(B):
            f['observations'][i * B + r, 0] = rank
            f['observations'][i * B + r, 1] = i
            f['observations'][i * B + r, 2] = r
            f['rewards'][i * B + r, 0] = 100 * rank + 10 * i + r
            f['terminals'][i * B + r, 0] = (r + i + rank) % 3 == 0
    steps = torch.tensor([B, B - rank, 2 + rank][:H], dtype=torch.int64)   # ragged live counts
    return f, steps


def _worker(rank, world, port, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from mopo_amd.distributed import allgather_transitions, unpack_rows
    f, steps = staging_for(rank)
    rows, counts = allgather_transitions(f, steps, H, B, O, A)
    out = unpack_rows(rows, O, A)
    q.put((rank, {k: v.numpy() for k, v in out.items()}, counts.numpy()))
    dist.destroy_process_group()


def test_allgather_global_order_world2():
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=60) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda t: t[0])
    # expected: step-major, then rank-major, live rows only, in row order
    exp_rows = []
    for i in range(H):
        for r in range(world):
            f, steps = staging_for(r)
            for j in range(int(steps[i])):
                exp_rows.append((r, i, j, float(f['rewards'][i * B + j, 0]), bool(f['terminals'][i * B + j, 0])))
    for rank, out, counts in res:
        got = [(int(o[0]), int(o[1]), int(o[2]), float(rw[0]), bool(t[0]))
               for o, rw, t in zip(out['observations'], out['rewards'], out['terminals'])]
        assert got == exp_rows
        np.testing.assert_array_equal(counts, np.stack([staging_for(r)[1].numpy() for r in range(world)]))
        assert (out['actions'][:, 0] == out['observations'][:, 0]).all()   # rows moved whole
    # both ranks hold identical pools
    for k in res[0][1]:
        np.testing.assert_array_equal(res[0][1][k], res[1][1][k])


def _rng_worker(rank, world, port, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from mopo_amd.distributed import broadcast_metrics, broadcast_numpy_rng
    np.random.seed(100 + rank)                  # the ranks' global streams differ ...
    if rank == 0:                               # ... and only rank 0 runs the model-training phase
        np.random.permutation(1000)
        np.random.normal(size=3)                # leaves a cached gaussian (has_gauss = 1)
    broadcast_numpy_rng()
    m = broadcast_metrics({'val_loss': 0.25, 'epochs': 7.0} if rank == 0 else None)
    q.put((rank, np.random.normal(size=5), np.random.randint(0, 1 << 30, 4), m))
    dist.destroy_process_group()


def test_numpy_stream_and_metrics_follow_rank0_world2():
    """MOPO.train on several ranks trains the ensemble on rank 0 only (mopo_amd/mopo.py); rank 0's numpy
    legacy stream (MT19937 key, position, cached gaussian) and training metrics are then broadcast, so
    every rank continues exactly where a single process would."""
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rng_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r[0], r[1:]) for r in [q.get(timeout=60) for _ in range(world)])
    for p in procs:
        p.join(timeout=60)
    np.random.seed(100)
    np.random.permutation(1000)
    np.random.normal(size=3)
    ref = (np.random.normal(size=5), np.random.randint(0, 1 << 30, 4))
    for r in range(world):
        np.testing.assert_array_equal(res[r][0], ref[0])
        np.testing.assert_array_equal(res[r][1], ref[1])
        assert res[r][2] == {'val_loss': 0.25, 'epochs': 7.0}


def _slow_src_worker(rank, world, port, q):
    """Rank 0 'trains' for longer than the default group's timeout; the others wait on wait_group."""
    import datetime
    import time
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world, timeout=datetime.timedelta(seconds=3))
    from mopo_amd.distributed import wait_for_src, wait_group
    g = wait_group()
    if rank == 0:
        time.sleep(6)                     # longer than the default group's 3 s timeout
    wait_for_src(g)
    t = torch.tensor([7.0 if rank == 0 else 0.0])
    dist.broadcast(t, 0)                  # the default group's collective, after the wait
    q.put((rank, float(t[0])))
    dist.destroy_process_group()


def test_slow_training_rank_does_not_time_out_waiters():
    """while rank 0 alone trains the ensemble (no time bound), the other ranks must not sit in a
    default-group collective (RCCL's watchdog would abort the job): MOPO.train waits on a long-timeout
    gloo group first (mopo_amd/distributed.py wait_group / wait_for_src)."""
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_slow_src_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == {0: 7.0, 1: 7.0}
