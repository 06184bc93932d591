"""SAC update of MOPO on the MI355X: ``_do_training`` + ``_update_target`` in one device step.

Mirrors the reference surface:
  * MOPO's in-graph SAC (mopo/algorithms/mopo.py:204-466): pi (256-256 relu, squashed Gaussian),
    twin Q (256-256 relu), targets, learned alpha with target_entropy, four TF1 Adams, Polyak.
  * ``_training_batch`` (mopo.py:801-821): int(batch*real_ratio) env rows + the rest model rows.
  * ``_do_training(iteration, batch)`` -> logs with the fetch names of mopo.py:453-463, and
    ``_update_target`` (mopo.py:852-853), folded into the same device step.
  * the ``SAC`` class API of softlearning/algorithms/sac.py:26-47, 340-349 (``_do_training``,
    ``_update_target``, ``get_diagnostics``, ``_training_batch``).
Everything runs in csrc/sac.hip; perf-mode steps replay one captured hipGraph.
"""
import ctypes as C
from collections import OrderedDict

import numpy as np

from . import _lib as L
from .rollout import init_sac_params

LOG_KEYS = ['Q/q1_loss', 'sac_Q/q2_loss', 'sac_Q/q1', 'sac_Q/q2', 'sac_pi/alpha', 'sac_pi/pi_entropy',
            'sac_pi/logp_pi', 'sac_pi/pi_global_norm', 'sac_Q/q_global_norm', 'policy_loss']


class SAC:
    def __init__(self, obs_dim, act_dim, hidden=256, batch_size=256, real_ratio=0.05, lr=3e-4, discount=0.99,
                 tau=5e-3, reward_scale=1.0, target_entropy='auto', params=None, log_alpha=0.0, seed=2,
                 reparameterize=True, use_graph=True):
        if not reparameterize:
            raise NotImplementedError('MOPO only implements the reparameterized policy loss (mopo.py:370-374)')
        self.obs_dim, self.act_dim, self.hidden = obs_dim, act_dim, hidden
        self.batch_size = int(batch_size)
        self._real_ratio = real_ratio
        self.n_env = int(self.batch_size * real_ratio)                       # mopo.py:803
        self._target_entropy = -float(act_dim) if target_entropy == 'auto' else float(target_entropy)
        self._discount, self._tau, self._reward_scale, self._lr = discount, tau, reward_scale, lr
        flat = init_sac_params(obs_dim, act_dim, hidden, seed=seed) if params is None else \
            np.ascontiguousarray(params, np.float32)
        n = L.lib().mopo_sac_param_count(obs_dim, act_dim, hidden)
        if flat.size != n:
            raise ValueError('expected %d parameters, got %d' % (n, flat.size))
        h = C.c_void_p()
        L.check(L.lib().mopo_sac_create(C.byref(h), obs_dim, act_dim, hidden, self.batch_size, self.n_env,
                                        flat.ctypes.data, float(log_alpha), float(lr), float(discount), float(tau),
                                        float(reward_scale), float(self._target_entropy)))
        self._h = h
        self.n_params = n
        L.check(L.lib().mopo_sac_set_graph(h, int(bool(use_graph))))
        bufs = [C.c_void_p() for _ in range(6)]
        npar = C.c_int64()
        L.check(L.lib().mopo_sac_buffers(h, *[C.byref(b) for b in bufs], C.byref(npar)))
        self._ptrs = dict(zip(['params', 'target', 'm', 'v', 'grads', 'logs'], [b.value for b in bufs]))
        self._num_train_steps = 0

    def __del__(self):
        h = getattr(self, '_h', None)
        if h is not None and h.value:
            L.lib().mopo_sac_destroy(h)
            self._h = None

    @property
    def policy_params_ptr(self):
        """Device pointer of the live policy parameters (pi block at offset 0) for rollouts."""
        return self._ptrs['params']

    def _copy(self, which, count, tensor=None, to_handle=False, stream=None):
        import torch
        if tensor is None:
            tensor = torch.empty(count, dtype=torch.float32, device='cuda')
        L.check(L.lib().mopo_sac_copy(self._h, which, int(to_handle), L.ptr(tensor), count, L.stream_ptr(stream)))
        return tensor

    def get_params(self):
        """(flat params [n_params], log_alpha) as torch CUDA tensors (copies)."""
        t = self._copy(0, self.n_params + 1)
        return t[:-1], t[-1]

    def get_target(self):
        return self._copy(1, self.n_params)

    def get_grads(self):
        t = self._copy(4, self.n_params + 1)
        return t[:-1], t[-1]

    def get_adam(self):
        return self._copy(2, self.n_params + 1), self._copy(3, self.n_params + 1)

    def set_params(self, flat, log_alpha=None):
        import torch
        t = torch.as_tensor(np.asarray(flat, np.float32) if not torch.is_tensor(flat) else flat).cuda().float()
        la = float(self.get_params()[1].item()) if log_alpha is None else float(log_alpha)
        t = torch.cat([t.reshape(-1), torch.tensor([la], device=t.device)])
        self._copy(0, self.n_params + 1, t, to_handle=True)

    def logs(self):
        """Fetches of the last step (mopo.py:453-463 names, plus policy_loss); synchronises."""
        v = self._copy(5, len(LOG_KEYS)).cpu().numpy()
        d = OrderedDict((k, float(x)) for k, x in zip(LOG_KEYS, v))
        d['sac_pi/std'] = d['sac_pi/logp_pi']   # the reference logs logp_pi under this key (mopo.py:463)
        return d

    def _do_training(self, iteration, env_pool, model_pool, n_steps=1, seed=0, idx=None, eps_s=None, eps_n=None,
                     stream=None):
        """``n_steps`` x (_training_batch + _do_training + _update_target) on the device.  With
        injected ``idx`` ([batch] rows: first n_env index the env pool) and policy noise, one step."""
        import torch
        keep = []

        def dp(x, dt):
            if x is None:
                return None
            t = torch.as_tensor(x).to('cuda', dt).contiguous()
            keep.append(t)
            return L.ptr(t)

        L.check(L.lib().mopo_sac_step(self._h, env_pool.desc(), model_pool.desc(), int(n_steps),
                                      int(seed) & (2 ** 64 - 1), dp(idx, torch.int64), dp(eps_s, torch.float32),
                                      dp(eps_n, torch.float32), L.stream_ptr(stream)))
        self._keepalive = keep
        self._num_train_steps += n_steps

    def _training_batch(self, env_pool, model_pool, batch_size=None, as_numpy=False):
        """mopo.py:801-821 as a host-visible batch (the device step assembles the same batch itself):
        int(batch_size * real_ratio) env rows, the rest model rows, env-first per shared field."""
        import torch
        batch_size = int(batch_size or self.batch_size)
        env_n = int(batch_size * self._real_ratio)
        model_n = batch_size - env_n
        env_batch = env_pool.random_batch(env_n, as_numpy=as_numpy)
        if model_n <= 0:
            return env_batch
        model_batch = model_pool.random_batch(model_n, as_numpy=as_numpy)
        keys = set(env_batch) & set(model_batch)
        cat = np.concatenate if as_numpy else torch.cat
        return {k: cat((env_batch[k], model_batch[k]), 0) for k in keys}

    def _update_target(self):
        """Folded into every device step (target_update_interval=1, mopo.py:843-845)."""

    def get_diagnostics(self):
        lg = self.logs()
        return OrderedDict({'Q_loss': (lg['Q/q1_loss'] + lg['sac_Q/q2_loss']) / 2, 'alpha': lg['sac_pi/alpha']})
