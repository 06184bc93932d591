"""Multi-GPU rollout: shard rollout rows over ranks, RCCL all-gather into replicated device pools.

One process per GPU (torchrun), ``torch.distributed`` backend ``nccl`` (= RCCL over xGMI).  Rank r
rolls out its own ``B`` rows with ``uid_offset = r*B`` (disjoint Philox sub-streams).  The device
path (``DistributedRollout``) stages each horizon step into its own 165-byte-per-row block and
all-gathers it asynchronously while the next step computes; every rank then appends all
transitions in the global order of a single-GPU rollout over the concatenated shards (step-major,
then rank-major) to its own pool (``mopo_pool_add_blocks``), so the pools stay identical across
ranks (SAC samples from them locally).  ``pack_rows`` / ``assemble_global`` /
``allgather_transitions`` are the host-orchestrated form of the same order (CPU gloo tests).
No reference counterpart (the reference is single-process); see SURVEY §8(e).
"""
import numpy as np
import torch


def pack_rows(fields, n, O, A):
    """[n, 2*O + A + 2] f32: obs | act | rew | term | next_obs (the SimpleReplayPool fields)."""
    return torch.cat([fields['observations'][:n], fields['actions'][:n], fields['rewards'][:n],
                      fields['terminals'][:n].float(), fields['next_observations'][:n]], 1)


def unpack_rows(rows, O, A):
    return {'observations': rows[:, :O], 'actions': rows[:, O:O + A], 'rewards': rows[:, O + A:O + A + 1],
            'terminals': rows[:, O + A + 1:O + A + 2] > 0.5, 'next_observations': rows[:, O + A + 2:]}


def assemble_global(gathered, counts, horizon, B):
    """gathered [world, horizon*B, W] (rank-local step-major staging), counts [world, horizon]
    -> rows in global order: for each step, rank 0's live rows, then rank 1's, ..."""
    world = gathered.shape[0]
    g = gathered.view(world, horizon, B, -1)
    cnt = counts.cpu().tolist()
    parts = [g[r, i, :int(cnt[r][i])] for i in range(horizon) for r in range(world)]
    return torch.cat(parts, 0) if parts else gathered.new_zeros((0, gathered.shape[-1]))


def allgather_transitions(staging_fields, steps, horizon, B, O, A, group=None):
    """Collective leg: returns (rows in global order [sum(counts), W], counts [world, horizon])."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    packed = pack_rows(staging_fields, horizon * B, O, A).contiguous()
    # concatenated (world*n, W) output: the form both RCCL and gloo accept
    gathered = torch.empty((world * packed.shape[0], packed.shape[1]), dtype=packed.dtype, device=packed.device)
    dist.all_gather_into_tensor(gathered, packed, group=group)
    counts = torch.empty((world * horizon,), dtype=torch.int64, device=steps.device)
    dist.all_gather_into_tensor(counts, steps.contiguous().to(torch.int64), group=group)
    counts = counts.view(world, horizon)
    return assemble_global(gathered.view(world, packed.shape[0], -1), counts, horizon, B), counts


def staged_block_desc(block, B, O, A):
    """PoolDesc over one staged block (uint8 tensor of mopo_pool_staged_block_bytes): obs | act | rew |
    next_obs | term (the layout mopo_pool_add_blocks reads)."""
    from . import _lib as L
    base = L.ptr(block)
    obs = base
    act = obs + 4 * B * O
    rew = act + 4 * B * A
    nobs = rew + 4 * B
    term = nobs + 4 * B * O
    return L.PoolDesc(d_obs=obs, d_act=act, d_rew=rew, d_term=term, d_next_obs=nobs, d_state=None, max_size=B)


class DistributedRollout:
    """Per-rank rollout + all-gather into this rank's replicated ``SimpleReplayPool``.

    Each horizon step is staged into its own block and all-gathered asynchronously (RCCL runs on its
    own stream) while the next step computes; the per-step counts are gathered once at the end and
    ``mopo_pool_add_blocks`` appends every rank's rows in global order (step-major, then rank) with
    device-side offsets -- no host synchronisation, no packing or re-ordering copies."""

    def __init__(self, model, batch_per_rank, horizon, obs_dim, act_dim, group=None, device=None):
        import torch
        import torch.distributed as dist
        from . import _lib as L
        from .rollout import ModelRollout
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.group = group
        self.B, self.horizon, self.O, self.A = int(batch_per_rank), int(horizon), obs_dim, act_dim
        self.ro = ModelRollout(model, self.B, self.horizon)
        self.blk = int(L.lib().mopo_pool_staged_block_bytes(obs_dim, act_dim, self.B))
        dev = device or torch.device('cuda', torch.cuda.current_device())
        self.staging = torch.empty((self.horizon, self.blk), dtype=torch.uint8, device=dev)
        self.gathered = torch.empty((self.horizon, self.world * self.blk), dtype=torch.uint8, device=dev)
        self.counts = torch.empty((self.world * self.horizon,), dtype=torch.int64, device=dev)

    def run(self, env_obs, pi_params, pool, term_kind, penalty_coeff, elites, seed=0, epoch=0, pi_hidden=256,
            **modes):
        """``modes``: the FakeEnv / rollout modes of ModelRollout.run (penalty_learned_var, deterministic,
        rollout_random, actor_dtype).  Returns the global rows per step (sum over ranks)."""
        import ctypes as C
        import torch.distributed as dist
        from . import _lib as L
        works = []

        def step_desc(i):
            return staged_block_desc(self.staging[i], self.B, self.O, self.A)

        def step_hook(i, steps):
            works.append(dist.all_gather_into_tensor(self.gathered[i], self.staging[i], group=self.group,
                                                     async_op=True))

        steps = self.ro.run(env_obs, pi_params, None, self.B, self.horizon, term_kind, penalty_coeff, elites,
                            seed=seed, epoch=epoch, pi_hidden=pi_hidden, staged=True, uid_offset=self.rank * self.B,
                            step_desc=step_desc, step_hook=step_hook, **modes)
        works.append(dist.all_gather_into_tensor(self.counts, steps.contiguous(), group=self.group, async_op=True))
        for w in works:
            w.wait()
        # blocks in memory order (step i, rank r) -> b = i * world + r; counts gathered as [rank][step]
        cb = self.counts.view(self.world, self.horizon).t().contiguous()
        desc = pool.desc()
        L.check(L.lib().mopo_pool_add_blocks(C.byref(desc), self.O, self.A, L.ptr(self.gathered), self.blk,
                                             self.horizon * self.world, self.B, L.ptr(cb), None))
        self._keep = cb
        return self.counts.view(self.world, self.horizon).sum(0)


# ---------------------------------------------------------------------------------------------------
# State sync for the multi-GPU training loop (MOPO with torch.distributed initialised).  Rank 0 is
# authoritative: it trains the ensemble and broadcasts its packed device image once (+ elites, ~4 MB at
# E=7, H=200), and before every rollout it broadcasts the whole SAC state (parameters, targets, Adam
# moments: ~3.5 MB at 256-256), so every rank rolls out its shard with the same policy and model
# (SURVEY 8(e)), and the replicated learners stay identical even if some float reduction on the device
# were not bit-reproducible.

WAIT_TIMEOUT_S = 30 * 24 * 3600   # rank 0's model training has no time bound (max_model_t=None)


def wait_group():
    """A CPU (gloo) process group with a month-long timeout, for the ranks that wait while rank 0 alone
    trains the ensemble: a collective of the default group (RCCL, 10-minute watchdog by default) would
    abort the job when training outlasts that timeout.  Collective: every rank calls it, in the same
    order (``MOPO.__init__``)."""
    import datetime
    import torch.distributed as dist
    return dist.new_group(backend='gloo', timeout=datetime.timedelta(seconds=WAIT_TIMEOUT_S))


def wait_for_src(group):
    """Every rank blocks here until all ranks arrive -- the training rank after its training, the others
    at once -- on ``group`` (``wait_group``), so the default group's next collective starts only when
    every rank is ready for it."""
    import torch.distributed as dist
    dist.barrier(group=group)


def world_info(group=None):
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def broadcast_model(model, src=0, group=None):
    """The ensemble from ``src`` to every rank as its packed device image (weights in the kernels'
    fragment layout, biases, scaler, log-var bounds, f16x3 scales: mopo_bnn_packed_copy) -- one
    device-to-device broadcast, no repack -- plus the elite indices, the holdout losses and the .mat
    arrays (so every rank's host state -- ``get_params``, ``scaler``, ``save``, ``train`` -- describes
    the same model)."""
    import torch.distributed as dist
    rank = dist.get_rank(group)
    dev = torch.device('cuda', torch.cuda.current_device())
    buf = model.export_packed() if rank == src else torch.empty(model.packed_nbytes(), dtype=torch.uint8,
                                                                  device=dev)
    el = torch.tensor(list(model._model_inds), dtype=torch.int64, device=dev)
    ne = torch.tensor([el.numel()], dtype=torch.int64, device=dev)
    dist.broadcast(ne, src, group=group)
    if rank != src:
        el = torch.empty(int(ne.item()), dtype=torch.int64, device=dev)
    n_flat = sum(z.size for z in model._mat_shapes())
    if rank == src:
        hl = getattr(model, '_holdout_losses', None)
        has = np.array([0.0 if hl is None else 1.0])   # a has-holdout flag: None stays None on every rank
        hl = np.zeros(model.num_nets) if hl is None else np.asarray(hl, np.float64)
        host = torch.from_numpy(np.concatenate([model.flat_params().astype(np.float64), hl, has])).to(dev)
    else:
        host = torch.empty(n_flat + model.num_nets + 1, dtype=torch.float64, device=dev)
    dist.broadcast(buf, src, group=group)
    dist.broadcast(el, src, group=group)
    dist.broadcast(host, src, group=group)
    if rank != src:
        h = host.cpu().numpy()
        hl = h[n_flat:n_flat + model.num_nets] if h[-1] != 0 else None
        model.import_packed(buf, mats=model.unflatten_params(h[:n_flat]), holdout_losses=hl)
        model.set_elites(el.cpu().tolist())
    torch.cuda.current_stream().synchronize()


def broadcast_numpy_rng(src=0, group=None):
    """numpy's legacy global RandomState (MT19937 key, position, cached gaussian) from ``src``, so every
    rank continues the single-process stream after a phase only ``src`` ran."""
    import numpy as np
    import torch.distributed as dist
    _, key, pos, has_gauss, gauss = np.random.get_state()
    t = torch.zeros(624 + 3, dtype=torch.float64)
    t[:624] = torch.from_numpy(key.astype(np.float64))
    t[624], t[625], t[626] = pos, has_gauss, gauss
    if dist.get_backend(group) == 'nccl':
        t = t.cuda()
    dist.broadcast(t, src, group=group)
    t = t.cpu().numpy()
    np.random.set_state(('MT19937', t[:624].astype(np.uint32), int(t[624]), int(t[625]), float(t[626])))


def broadcast_metrics(metrics, src=0, group=None):
    """``src``'s model-training metrics dict (float values) to every rank."""
    import torch.distributed as dist
    obj = [metrics]
    dist.broadcast_object_list(obj, src, group=group)
    return dict(obj[0])


def broadcast_sac(sac, src=0, group=None):
    """The SAC state (params + log_alpha, targets, Adam m / v) from ``src`` to every rank."""
    import torch.distributed as dist
    n = sac._n_dev     # the raw device buffers (padded layout of a [H1, H2] network)
    parts = [(0, n + 1), (1, n), (2, n + 1), (3, n + 1)]
    buf = torch.cat([sac._copy(w, c) for w, c in parts])
    dist.broadcast(buf, src, group=group)
    off = 0
    for w, c in parts:
        sac._copy(w, c, buf[off:off + c].contiguous(), to_handle=True)
        off += c
