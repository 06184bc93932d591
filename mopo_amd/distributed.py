"""Multi-GPU rollout: shard rollout rows over ranks, RCCL all-gather into replicated device pools.

One process per GPU (torchrun), ``torch.distributed`` backend ``nccl`` (= RCCL over xGMI).  Rank r
rolls out its own ``B`` rows with ``uid_offset = r*B`` (disjoint Philox sub-streams), staged
step-major (``mopo_rollout_run_staged``); one ``all_gather_into_tensor`` moves the packed 165-byte
rows and one moves the per-step counts; every rank then appends all transitions in the global
order of a single-GPU rollout over the concatenated shards (step-major, then rank-major) to its
own pool, so the pools stay identical across ranks (SAC samples from them locally).
No reference counterpart (the reference is single-process); see SURVEY §8(e).
"""
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


class DistributedRollout:
    """Per-rank rollout + all-gather into this rank's replicated ``SimpleReplayPool``."""

    def __init__(self, model, batch_per_rank, horizon, obs_dim, act_dim, group=None):
        import torch.distributed as dist
        from .replay_pool import SimpleReplayPool
        from .rollout import ModelRollout
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.group = group
        self.B, self.horizon, self.O, self.A = int(batch_per_rank), int(horizon), obs_dim, act_dim
        self.ro = ModelRollout(model, self.B, self.horizon)
        self.staging = SimpleReplayPool(obs_dim=obs_dim, act_dim=act_dim, max_size=self.B * self.horizon)

    def run(self, env_obs, pi_params, pool, term_kind, penalty_coeff, elites, seed=0, epoch=0, pi_hidden=256):
        steps = self.ro.run(env_obs, pi_params, self.staging, self.B, self.horizon, term_kind, penalty_coeff, elites,
                            seed=seed, epoch=epoch, pi_hidden=pi_hidden, staged=True,
                            uid_offset=self.rank * self.B)
        rows, counts = allgather_transitions(self.staging.fields, steps, self.horizon, self.B, self.O, self.A,
                                             self.group)
        pool.add_samples(unpack_rows(rows, self.O, self.A))
        return counts.sum(0)
