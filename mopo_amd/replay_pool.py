"""Device-resident SimpleReplayPool.

Mirrors ``SimpleReplayPool`` / ``FlexibleReplayPool`` (softlearning/replay_pools/
simple_replay_pool.py:37-106, flexible_replay_pool.py:9-182): same field names, dtypes and
ring semantics, ``add_samples``, ``random_indices``/``random_batch``, ``batch_by_indices``,
``return_all_samples``, ``size``, ``_max_size``, ``_pointer``.  Fields are torch CUDA tensors in
HBM (SoA); pointer and size live on the device (int64[2]) so fused rollouts append without a host
round trip -- read ``size``/``_pointer`` and the device copy is synchronised lazily.
"""
import numpy as np

from . import _lib as L

FIELDS = ('observations', 'actions', 'rewards', 'terminals', 'next_observations')


class SimpleReplayPool:
    def __init__(self, observation_space=None, action_space=None, max_size=int(1e6), obs_dim=None, act_dim=None,
                 device='cuda'):
        import torch
        self._observation_space, self._action_space = observation_space, action_space
        if obs_dim is None:
            obs_dim = int(np.prod(_space_shape(observation_space)))
        if act_dim is None:
            act_dim = int(np.prod(_space_shape(action_space)))
        self.obs_dim, self.act_dim = obs_dim, act_dim
        self._max_size = int(max_size)
        m = self._max_size
        f32 = dict(dtype=torch.float32, device=device)
        self.fields = {
            'observations': torch.zeros((m, obs_dim), **f32),
            'actions': torch.zeros((m, act_dim), **f32),
            'rewards': torch.zeros((m, 1), **f32),
            'terminals': torch.zeros((m, 1), dtype=torch.bool, device=device),
            'next_observations': torch.zeros((m, obs_dim), **f32),
        }
        self._state = torch.zeros(2, dtype=torch.int64, device=device)   # {pointer, size}

    # -- descriptor for the C ABI --------------------------------------------------------------------
    def desc(self):
        f = self.fields
        return L.PoolDesc(d_obs=L.ptr(f['observations']), d_act=L.ptr(f['actions']), d_rew=L.ptr(f['rewards']),
                          d_term=L.ptr(f['terminals']), d_next_obs=L.ptr(f['next_observations']),
                          d_state=L.ptr(self._state), max_size=self._max_size)

    @property
    def size(self):
        return int(self._state[1].item())

    @property
    def _pointer(self):
        return int(self._state[0].item())

    @property
    def _size(self):
        return self.size

    @property
    def field_names(self):
        return list(FIELDS)

    def add_samples(self, samples, stream=None):
        """flexible_replay_pool.py:57-83 (numpy or torch inputs; cast to the field dtypes)."""
        import torch
        n = int(samples['observations'].shape[0])
        if n == 0:
            return
        dev = self._state.device

        def t(x, dt):
            x = torch.as_tensor(np.asarray(x) if not torch.is_tensor(x) else x)
            return x.to(dev, dt).contiguous()

        if n > self._max_size:  # only the last max_size rows survive a wrapping write
            samples = {k: v[n - self._max_size:] for k, v in samples.items()}
            # rows overwritten within one call: write the leading part first to keep the pointer math
            self._state[0] = (self._state[0] + (n - self._max_size)) % self._max_size
            self._state[1] = torch.clamp(self._state[1] + (n - self._max_size), max=self._max_size)
            n = self._max_size
        obs = t(samples['observations'], torch.float32)
        act = t(samples['actions'], torch.float32)
        rew = t(samples['rewards'], torch.float32).reshape(n)
        term = t(samples['terminals'], torch.bool).reshape(n).view(torch.uint8)
        nobs = t(samples['next_observations'], torch.float32)
        d = self.desc()
        L.check(L.lib().mopo_pool_add(d, self.obs_dim, self.act_dim, L.ptr(obs), L.ptr(act), L.ptr(rew),
                                      L.ptr(term), L.ptr(nobs), n, L.stream_ptr(stream)))

    def random_indices(self, batch_size):
        """flexible_replay_pool.py:85-87 (numpy legacy stream, as the reference)."""
        size = self.size
        if size == 0:
            return np.arange(0, 0)
        return np.random.randint(0, size, batch_size)

    def batch_by_indices(self, indices, as_numpy=False):
        import torch
        idx = torch.as_tensor(np.asarray(indices) if not torch.is_tensor(indices) else indices)
        idx = idx.to(self._state.device, torch.int64)
        out = {k: v[idx] for k, v in self.fields.items()}
        if as_numpy:
            out = {k: v.cpu().numpy() for k, v in out.items()}
        return out

    def random_batch(self, batch_size, as_numpy=False, **kwargs):
        return self.batch_by_indices(self.random_indices(batch_size), as_numpy=as_numpy)

    def return_all_samples(self, as_numpy=False):
        s = self.size
        out = {k: v[:s] for k, v in self.fields.items()}
        if as_numpy:
            out = {k: v.cpu().numpy() for k, v in out.items()}
        return out

    def terminate_episode(self):
        pass


def _space_shape(space):
    if space is None:
        raise ValueError('pass obs_dim/act_dim or a space')
    if hasattr(space, 'spaces'):  # gym Dict of Boxes (simple_replay_pool.py:42-46)
        return (sum(int(np.prod(s.shape)) for s in space.spaces.values()),)
    return space.shape
