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
from .rollout import device_hidden, hidden_pair, init_sac_params, sac_pad_index, sac_param_shapes

LOG_KEYS = ['Q/q1_loss', 'sac_Q/q2_loss', 'sac_Q/q1', 'sac_Q/q2', 'sac_pi/alpha', 'sac_pi/pi_entropy',
            'sac_pi/logp_pi', 'sac_pi/pi_global_norm', 'sac_Q/q_global_norm', 'policy_loss']


def _space_dim(space):
    shp = getattr(space, 'shape', None)
    if shp is None or len(shp) != 1:
        raise ValueError('expected a flat Box space with a 1-D shape, got %r' % (space,))
    return int(shp[0])


class SAC:
    """Two constructor forms:

    * ``SAC(obs_dim, act_dim, hidden=256, ...)`` -- the dims directly (``hidden`` an int H for [H, H], or the
      two widths [H1, H2] of mopo.py:275-280's ``hidden_sizes``);
    * ``SAC(training_environment, evaluation_environment, policy, Qs, pool, plotter=None,
      tf_summaries=False, lr=3e-4, reward_scale=1.0, target_entropy='auto', discount=0.99, tau=5e-3,
      target_update_interval=1, action_prior='uniform', reparameterize=False, store_extra_policy_info=False,
      save_full_state=False, **kwargs)`` -- softlearning/algorithms/sac.py:26-47: the dims come from the
      environment's spaces, the hidden width from the policy / Qs (``hidden_layer_sizes`` or
      ``hidden_sizes``, default 256 x 2); ``pool`` becomes the default env pool of ``_do_training``.
    """

    def __init__(self, obs_dim, act_dim=None, *args, **kwargs):
        if not isinstance(obs_dim, (int, np.integer)):
            self._init_softlearning(obs_dim, act_dim, *args, **kwargs)
        else:
            self._init(obs_dim, act_dim, *args, **kwargs)

    def _init_softlearning(self, training_environment, evaluation_environment, policy=None, Qs=(), pool=None,
                           plotter=None, tf_summaries=False, lr=3e-4, reward_scale=1.0, target_entropy='auto',
                           discount=0.99, tau=5e-3, target_update_interval=1, action_prior='uniform',
                           reparameterize=False, store_extra_policy_info=False, save_full_state=False,
                           batch_size=256, real_ratio=1.0, **kwargs):
        if action_prior not in ('uniform', 'normal'):
            raise NotImplementedError("action_prior must be 'uniform' or 'normal' (sac.py:285-289)")
        if store_extra_policy_info:
            raise NotImplementedError('store_extra_policy_info')
        env = training_environment
        obs_space = getattr(env, 'active_observation_shape', None)
        obs_dim = int(obs_space[0]) if obs_space is not None else _space_dim(env.observation_space)
        act_dim = _space_dim(env.action_space)
        hs = None
        for src in (policy, *(Qs or ())):
            hs = hs or getattr(src, 'hidden_layer_sizes', None) or getattr(src, '_hidden_layer_sizes', None) or \
                getattr(src, 'hidden_sizes', None)
        hs = hidden_pair(list(hs or [256, 256]))
        self._training_environment, self._evaluation_environment = training_environment, evaluation_environment
        self._policy, self._Qs, self._pool, self._plotter = policy, Qs, pool, plotter
        self._init(obs_dim, act_dim, hidden=hs, batch_size=batch_size, real_ratio=real_ratio, lr=lr,
                   discount=discount, tau=tau, reward_scale=reward_scale, target_entropy=target_entropy,
                   reparameterize=reparameterize, target_update_interval=target_update_interval,
                   action_prior=action_prior, **kwargs)

    def _init(self, obs_dim, act_dim, hidden=256, batch_size=256, real_ratio=0.05, lr=3e-4, discount=0.99,
              tau=5e-3, reward_scale=1.0, target_entropy='auto', params=None, log_alpha=0.0, seed=2,
              reparameterize=True, use_graph=True, target_update_interval=1, action_prior='uniform'):
        if not reparameterize:
            raise NotImplementedError('only the reparameterized policy loss is implemented (mopo.py:370-374; '
                                      'every config sets reparameterize=True, examples/config/d4rl/base.py)')
        # a [H1, H2] network runs on the device as the square device_hidden() one with the narrower
        # layer zero-padded (exact: rollout.device_hidden); every accessor speaks the [H1, H2] layout
        self.hidden_sizes = hidden_pair(hidden)
        self.obs_dim, self.act_dim, self.hidden = obs_dim, act_dim, device_hidden(hidden)
        self._pad = sac_pad_index(obs_dim, act_dim, self.hidden_sizes)
        self._pad_t = None
        self._pool = getattr(self, '_pool', None)
        self.batch_size = int(batch_size)
        self._real_ratio = real_ratio
        self.n_env = int(self.batch_size * real_ratio)                       # mopo.py:803
        self._target_entropy = -float(act_dim) if target_entropy == 'auto' else float(target_entropy)
        self._discount, self._tau, self._reward_scale, self._lr = discount, tau, reward_scale, lr
        self._seed = int(seed)
        if int(target_update_interval) < 1:
            raise ValueError('target_update_interval must be >= 1')
        self._target_update_interval = int(target_update_interval)
        self._schedule = (0, 1, 1)       # the device's target schedule (mopo_sac_set_target_schedule)
        flat = init_sac_params(obs_dim, act_dim, self.hidden_sizes, seed=seed) if params is None else \
            np.ascontiguousarray(params, np.float32).ravel()
        n = sum(int(np.prod(s)) for s in sac_param_shapes(obs_dim, act_dim, self.hidden_sizes))
        if flat.size != n:
            raise ValueError('expected %d parameters, got %d' % (n, flat.size))
        self._n_dev = L.lib().mopo_sac_param_count(obs_dim, act_dim, self.hidden)
        if self._pad is not None:
            dev_flat = np.zeros(self._n_dev, np.float32)
            dev_flat[self._pad] = flat
            flat = dev_flat
        h = C.c_void_p()
        L.check(L.lib().mopo_sac_create(C.byref(h), obs_dim, act_dim, self.hidden, self.batch_size, self.n_env,
                                        flat.ctypes.data, float(log_alpha), float(lr), float(discount), float(tau),
                                        float(reward_scale), float(self._target_entropy)))
        self._h = h
        self.n_params = n
        L.check(L.lib().mopo_sac_set_graph(h, int(bool(use_graph))))
        if action_prior not in ('uniform', 'normal'):
            raise NotImplementedError("action_prior must be 'uniform' or 'normal' (sac.py:285-289)")
        self._action_prior = action_prior
        L.check(L.lib().mopo_sac_set_action_prior(h, int(action_prior == 'normal')))
        bufs = [C.c_void_p() for _ in range(6)]
        npar = C.c_int64()
        L.check(L.lib().mopo_sac_buffers(h, *[C.byref(b) for b in bufs], C.byref(npar)))
        self._ptrs = dict(zip(['params', 'target', 'm', 'v', 'grads', 'logs'], [b.value for b in bufs]))
        self._num_train_steps = 0

    def __del__(self):
        h = getattr(self, '_h', None)
        if h is not None and h.value and L is not None and L.lib is not None:   # not at interpreter teardown
            L.lib().mopo_sac_destroy(h)
            self._h = None

    @property
    def policy_params_ptr(self):
        """Device pointer of the live policy parameters (pi block at offset 0, the device_hidden layout)
        for rollouts (run them with pi_hidden = self.hidden)."""
        return self._ptrs['params']

    def _copy(self, which, count, tensor=None, to_handle=False, stream=None):
        """Raw copy of a device buffer (the device layout: self._n_dev parameters)."""
        import torch
        if tensor is None:
            tensor = torch.empty(count, dtype=torch.float32, device='cuda')
        L.check(L.lib().mopo_sac_copy(self._h, which, int(to_handle), L.ptr(tensor), count, L.stream_ptr(stream)))
        return tensor

    def _index(self):
        import torch
        if self._pad_t is None:
            self._pad_t = torch.from_numpy(self._pad).cuda()
        return self._pad_t

    def _get(self, which, extra):
        """Buffer ``which`` in the [H1, H2] layout (+ ``extra`` trailing elements: log_alpha)."""
        import torch
        t = self._copy(which, self._n_dev + extra)
        if self._pad is None:
            return t
        return torch.cat([t[self._index()], t[self._n_dev:]])

    def _put(self, which, t, extra):
        """Buffer ``which`` from the [H1, H2] layout; the padding stays 0."""
        import torch
        t = t.reshape(-1).float().contiguous()
        if self._pad is not None:
            d = torch.zeros(self._n_dev + extra, dtype=torch.float32, device=t.device)
            d[self._index()] = t[:self.n_params]
            d[self._n_dev:] = t[self.n_params:]
            t = d
        self._copy(which, self._n_dev + extra, t, to_handle=True)

    def get_params(self):
        """(flat params [n_params], log_alpha) as torch CUDA tensors (copies)."""
        t = self._get(0, 1)
        return t[:-1], t[-1]

    def get_target(self):
        return self._get(1, 0)

    def get_grads(self):
        t = self._get(4, 1)
        return t[:-1], t[-1]

    def get_adam(self):
        return self._get(2, 1), self._get(3, 1)

    def set_params(self, flat, log_alpha=None):
        import torch
        t = torch.as_tensor(np.asarray(flat, np.float32) if not torch.is_tensor(flat) else flat).cuda().float()
        la = float(self.get_params()[1].item()) if log_alpha is None else float(log_alpha)
        t = torch.cat([t.reshape(-1), torch.tensor([la], device=t.device)])
        self._put(0, t, 1)

    def logs(self):
        """Fetches of the last step (mopo.py:453-463 names, plus policy_loss); synchronises."""
        v = self._copy(5, len(LOG_KEYS)).cpu().numpy()
        self.check()
        d = OrderedDict((k, float(x)) for k, x in zip(LOG_KEYS, v))
        d['sac_pi/std'] = d['sac_pi/logp_pi']   # the reference logs logp_pi under this key (mopo.py:463)
        return d

    def check(self):
        """Raises if a fused step's bounded hand-off wait gave up since the last check (the device then held
        every parameter / Adam / target update instead of applying one from stale operands); synchronises."""
        flag = C.c_int(0)
        L.check(L.lib().mopo_sac_check(self._h, C.byref(flag)))

    def _do_training(self, iteration, env_pool=None, model_pool=None, n_steps=1, seed=0, idx=None, eps_s=None,
                     eps_n=None, stream=None, n_train_repeat=1):
        """``n_steps`` x (_training_batch + _do_training + _update_target) on the device.  With
        injected ``idx`` ([batch] rows: first n_env index the env pool) and policy noise, one step.
        ``iteration`` is the timestep of the first step (each timestep runs ``n_train_repeat`` steps,
        mopo.py:780-799); the targets move on the steps whose timestep % target_update_interval == 0
        (mopo.py:843-845).
        ``_do_training(iteration, batch)`` with a batch dict (sac.py:340-349 / mopo.py:834-850): one step
        on exactly those rows (host or device arrays, ``batch_size`` rows)."""
        import torch
        if isinstance(env_pool, dict):
            return self._do_training_batch(iteration, env_pool, eps_s=eps_s, eps_n=eps_n, stream=stream)
        if env_pool is None:
            env_pool = self._pool
        if model_pool is None:
            model_pool = env_pool
        keep = []

        def dp(x, dt):
            if x is None:
                return None
            t = torch.as_tensor(x).to('cuda', dt).contiguous()
            keep.append(t)
            return L.ptr(t)

        sched = (self._num_train_steps - int(iteration) * int(n_train_repeat), int(n_train_repeat),
                 self._target_update_interval)
        if self._target_update_interval == 1:
            sched = (0, 1, 1)            # every step; the schedule's base is irrelevant
        if sched != self._schedule:
            L.check(L.lib().mopo_sac_set_target_schedule(self._h, *sched, L.stream_ptr(stream)))
            self._schedule = sched
        L.check(L.lib().mopo_sac_step(self._h, env_pool.desc(), model_pool.desc(), int(n_steps),
                                      int(seed) & (2 ** 64 - 1), dp(idx, torch.int64), dp(eps_s, torch.float32),
                                      dp(eps_n, torch.float32), L.stream_ptr(stream)))
        self._keepalive = keep
        self._num_train_steps += n_steps

    def _do_training_batch(self, iteration, batch, eps_s=None, eps_n=None, stream=None):
        """One step on the given batch: its rows are staged in two scratch pools (env part first,
        mopo.py:815-816 order) and drawn back by index, so the device step sees exactly this batch."""
        import torch
        from .replay_pool import SimpleReplayPool
        n = int(np.asarray(batch['observations']).shape[0] if not torch.is_tensor(batch['observations'])
                else batch['observations'].shape[0])
        if n != self.batch_size:
            raise ValueError('batch has %d rows, the step was built for %d' % (n, self.batch_size))
        cut = self.n_env
        pools = []
        for lo, hi in ((0, cut), (cut, n)):
            p = SimpleReplayPool(obs_dim=self.obs_dim, act_dim=self.act_dim, max_size=max(hi - lo, 1))
            p.add_samples({k: v[lo:hi] for k, v in batch.items() if k in p.fields})
            pools.append(p)
        idx = np.concatenate([np.arange(cut), np.arange(n - cut)]).astype(np.int64)
        if eps_s is None or eps_n is None:
            # the reference draws these in-graph (tf.random_normal, mopo.py:306); a private stream keyed by
            # (seed, iteration) keeps numpy's global stream -- which drives BNN.train -- untouched
            rs = np.random.RandomState([self._seed & 0xffffffff, int(iteration) & 0xffffffff])
            eps_s = rs.normal(size=(n, self.act_dim)) if eps_s is None else eps_s
            eps_n = rs.normal(size=(n, self.act_dim)) if eps_n is None else eps_n
        self._do_training(iteration, pools[0], pools[1], idx=idx, seed=iteration, eps_s=eps_s, eps_n=eps_n,
                          stream=stream)
        return self.logs()

    def state_dict(self):
        """Device copies of everything a step reads (the saveables of sac.py:418-427 and the targets), in
        the [H1, H2] layout."""
        return {'params': self._get(0, 1), 'target': self._get(1, 0), 'adam_m': self._get(2, 1),
                'adam_v': self._get(3, 1)}

    def load_state_dict(self, state):
        for w, (k, x) in enumerate((('params', 1), ('target', 0), ('adam_m', 1), ('adam_v', 1))):
            self._put(w, state[k], x)

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
        """Folded into the device step: Polyak on the steps of the target schedule (mopo.py:843-845)."""

    def get_diagnostics(self, *args, **kwargs):
        """mopo.py:900-905 keys (the arguments of sac.py's get_diagnostics are accepted and unused)."""
        lg = self.logs()
        return OrderedDict({'Q_loss': (lg['Q/q1_loss'] + lg['sac_Q/q2_loss']) / 2, 'alpha': lg['sac_pi/alpha']})
