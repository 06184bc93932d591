"""MOPO outer loop on the MI355X path (host mirror of ``mopo.algorithms.mopo.MOPO``).

Reference: mopo/algorithms/mopo.py — ``__init__`` (46-201), ``_train`` (490-648),
``_set_rollout_length`` (675-687), ``_reallocate_model_pool`` (689-711), ``_rollout_model``
(723-765), ``_do_training_repeats`` (780-799), ``_training_batch`` (801-821), ``_do_training``
(834-850), ``get_diagnostics`` (876-918).

Differences that are deliberate: the rollout and the SAC steps run on the device
(csrc/rollout.hip, csrc/sac.hip); the epoch's 1000 SAC steps are issued as one replayed hipGraph
batch (the reference runs them one ``session.run`` at a time, with the same batch rule per step);
Evaluation rollouts (``_evaluation_paths`` / ``_evaluate_rollouts``, mopo.py:575-629) run when an
``evaluation_environment`` (gym API) is passed -- MuJoCo is not in this image, so the caller supplies
it; without one the ``evaluation/*`` and ``perf/*`` keys are absent.  The dynamics model is trained once before the epoch loop
(mopo.py:526-531): one epoch when it was loaded from ``model_load_dir``, else to early stopping,
on the device (``_train_model`` formats the env pool on the device in the holdout-permutation order).
"""
import time
from collections import OrderedDict

import numpy as np

from .bnn import DEFAULT_ENSEMBLE_DTYPE, construct_model, default_ensemble_dtype
from .fake_env import FakeEnv
from .replay_pool import SimpleReplayPool
from .rollout import ModelRollout
from .sac import SAC


class MOPO:
    def __init__(self, pool, static_fns, obs_dim, act_dim, lr=3e-4, reward_scale=1.0, target_entropy='auto',
                 discount=0.99, tau=5e-3, target_update_interval=1, model_train_freq=250, num_networks=7,
                 num_elites=5, model_retain_epochs=20, rollout_batch_size=100e3, real_ratio=0.1, rollout_length=1,
                 hidden_dim=200, separate_mean_var=False, penalty_coeff=0., penalty_learned_var=False,
                 model_name=None, model_load_dir=None, deterministic=False, network_kwargs=None, epoch_length=1000,
                 n_epochs=1000, n_train_repeat=1, batch_size=256, seed=88, reparameterize=True, max_model_t=None,
                 rollout_random=False, evaluation_environment=None, eval_n_episodes=10, eval_deterministic=True,
                 max_path_length=1000, ensemble_dtype=None, actor_dtype=None, **kwargs):
        """``ensemble_dtype``: the ensemble forward's arithmetic (``mopo_amd.bnn.DTYPES``), default
        ``DEFAULT_ENSEMBLE_DTYPE`` ('bf16x6': the f32 operands split exactly into 3 bf16 parts, 6 bf16
        MFMA products, f32 accumulate; 'fp32' above H = 256: ``bnn.default_ensemble_dtype``); 'fp32' runs
        exact-f32 MFMA, 'f16x3' ~22-bit operands.  ``actor_dtype``: the rollout policy forward ('fp32' /
        'bf16x6' / 'f16x3'; default the ensemble's for fp32 and bf16x6, else f16x3:
        ``rollout.default_actor_dtype``)."""
        if kwargs.get('action_prior', 'uniform') != 'uniform':   # mopo.py:364 asserts the uniform prior
            raise AssertionError("MOPO's policy loss supports action_prior='uniform' only (mopo.py:364)")
        self._pool = pool                                   # device SimpleReplayPool of env data
        self._static_fns = static_fns
        self._obs_dim, self._act_dim = obs_dim, act_dim
        self._model = construct_model(obs_dim=obs_dim, act_dim=act_dim, hidden_dim=hidden_dim,
                                      num_networks=num_networks, num_elites=num_elites,
                                      separate_mean_var=separate_mean_var, name=model_name,
                                      load_dir=model_load_dir, deterministic=deterministic,
                                      dtype=ensemble_dtype or default_ensemble_dtype(hidden_dim), seed=seed)   # the run seed (simple_run/main.py:180 set_seed) fixes the init
        self.fake_env = FakeEnv(self._model, static_fns, penalty_coeff=penalty_coeff,
                                penalty_learned_var=penalty_learned_var)
        self._rollout_schedule = [20, 100, rollout_length, rollout_length]                 # mopo.py:137
        self._model_retain_epochs = model_retain_epochs
        self._model_train_freq = model_train_freq
        self._rollout_batch_size = int(rollout_batch_size)
        self._deterministic = deterministic
        self._rollout_random = rollout_random
        self._actor_dtype = actor_dtype
        self._real_ratio = real_ratio
        self._epoch_length, self._n_epochs, self._n_train_repeat = epoch_length, n_epochs, n_train_repeat
        self._epoch = 0
        self._num_train_steps = 0
        self._seed = seed
        hs = list((network_kwargs or {}).get('hidden_sizes', [256, 256]))   # mopo.py:275-280, base.py:60-66
        self._sac = SAC(obs_dim, act_dim, hidden=hs, batch_size=batch_size, real_ratio=real_ratio, lr=lr,
                        discount=discount, tau=tau, reward_scale=reward_scale, target_entropy=target_entropy,
                        seed=seed, reparameterize=reparameterize, target_update_interval=target_update_interval)
        self._pi_hidden = self._sac.hidden   # the device width the rollout actor runs (rollout.device_hidden)
        self._rollout = None
        self._rollout_length = rollout_length
        # multi-GPU (torch.distributed initialised, one process per GPU): the rollout rows are sharded
        # over the ranks and all-gathered into every rank's model pool; SAC runs replicated
        from .distributed import wait_group, world_info
        self._rank, self._world = world_info()
        # the ranks that wait while rank 0 trains the ensemble wait on this long-timeout CPU group
        self._wait_group = wait_group() if self._world > 1 else None
        if self._rollout_batch_size % self._world:
            raise ValueError('rollout_batch_size must be a multiple of the world size')
        self._max_model_t = max_model_t
        self._evaluation_environment = evaluation_environment
        self._eval_n_episodes, self._eval_deterministic = eval_n_episodes, eval_deterministic
        self._max_path_length = max_path_length
        from .evaluation import ref_scores
        self.min_ret, self.max_ret = ref_scores(model_name)                              # mopo.py:115-123
        self._model_train_metrics = None

    # -- mopo.py:675-687
    def _set_rollout_length(self):
        min_epoch, max_epoch, min_length, max_length = self._rollout_schedule
        if self._epoch <= min_epoch:
            y = min_length
        else:
            dx = min((self._epoch - min_epoch) / (max_epoch - min_epoch), 1)
            y = dx * (max_length - min_length) + min_length
        self._rollout_length = int(y)

    # -- mopo.py:689-711
    def _reallocate_model_pool(self):
        rollouts_per_epoch = self._rollout_batch_size * self._epoch_length / self._model_train_freq
        model_steps_per_epoch = int(self._rollout_length * rollouts_per_epoch)
        new_pool_size = self._model_retain_epochs * model_steps_per_epoch
        if not hasattr(self, '_model_pool'):
            self._model_pool = SimpleReplayPool(obs_dim=self._obs_dim, act_dim=self._act_dim, max_size=new_pool_size)
        elif self._model_pool._max_size != new_pool_size:
            samples = self._model_pool.return_all_samples()
            new_pool = SimpleReplayPool(obs_dim=self._obs_dim, act_dim=self._act_dim, max_size=new_pool_size)
            new_pool.add_samples(samples)
            assert self._model_pool.size == new_pool.size
            self._model_pool = new_pool

    # -- mopo.py:713-721 + constructor.py:46-57
    def _train_model(self, **kwargs):
        import ctypes as C
        import torch
        from . import _lib as L
        N, O, A = self._pool.size, self._obs_dim, self._act_dim
        # bnn.py:392 draws np.random.permutation first; drawing it here keeps the stream order and
        # lets the format kernel write the rows already permuted (holdout first)
        perm = torch.from_numpy(np.random.permutation(N)).cuda()
        x = torch.empty((N, O + A), dtype=torch.float32, device='cuda')
        y = torch.empty((N, O + 1), dtype=torch.float32, device='cuda')
        L.check(L.lib().mopo_bnn_format_samples(C.byref(self._pool.desc()), O, A, L.ptr(perm), N, L.ptr(x),
                                                L.ptr(y), None))
        return self._model.train(x, y, permuted=True, **kwargs)

    # -- mopo.py:723-765 (device-resident, perf-mode RNG); ``deterministic`` as mopo.py:558-559 passes it
    def _rollout_model(self, rollout_batch_size, deterministic=None, rollout_key=None, **kwargs):
        key = self._epoch if rollout_key is None else rollout_key
        modes = dict(penalty_learned_var=self.fake_env.penalty_learned_var,
                     deterministic=self._deterministic if deterministic is None else deterministic,
                     rollout_random=self._rollout_random)
        env_obs = self._pool.fields['observations'][:self._pool.size]
        if self._world > 1:
            return self._rollout_model_sharded(rollout_batch_size, env_obs, modes, key)
        if self._rollout is None or self._rollout.max_batch < rollout_batch_size or \
                self._rollout.max_horizon < self._rollout_length:
            self._rollout = ModelRollout(self._model, rollout_batch_size, max(self._rollout_length, 1))
        steps = self._rollout.run(env_obs, self._sac.policy_params_ptr, self._model_pool, rollout_batch_size,
                                  self._rollout_length, self.fake_env.term_kind, self.fake_env.penalty_coeff,
                                  self._model._model_inds, seed=self._seed, epoch=key,
                                  pi_hidden=self._pi_hidden, actor_dtype=self._actor_dtype, **modes)
        added = int(steps.sum().item())
        return {'mean_rollout_length': added / rollout_batch_size}

    def _rollout_model_sharded(self, rollout_batch_size, env_obs, modes, key):
        """Rank r rolls out rows [r B/N, (r + 1) B/N) of the batch (Philox streams keyed by the global
        row id, so the N shards are exactly the single-GPU rollout's rows) after rank 0's model and SAC
        state are broadcast; every rank's model pool receives all transitions in the single-GPU order."""
        from .distributed import DistributedRollout, broadcast_sac
        # the ensemble is fixed after _train_model (broadcast once, in train()); the replicated learners
        # are re-synchronised from rank 0 before every rollout as a guard against any drift
        broadcast_sac(self._sac)
        b = rollout_batch_size // self._world
        h = max(self._rollout_length, 1)
        if self._rollout is None or self._rollout.B != b or self._rollout.horizon != h:
            self._rollout = DistributedRollout(self._model, b, h, self._obs_dim, self._act_dim)
        steps = self._rollout.run(env_obs, self._sac.policy_params_ptr, self._model_pool, self.fake_env.term_kind,
                                  self.fake_env.penalty_coeff, self._model._model_inds, seed=self._seed,
                                  epoch=key, pi_hidden=self._pi_hidden, actor_dtype=self._actor_dtype,
                                  **modes)
        added = int(steps.sum().item())
        return {'mean_rollout_length': added / rollout_batch_size}

    # -- mopo.py:780-799 + 834-853: n steps of (_training_batch, _do_training, _update_target); the first
    #    is timestep `first_timestep` of the epoch, each timestep n_train_repeat steps
    def _do_training_repeats(self, n_steps, first_timestep=0):
        # real_ratio = 1.0: no model pool (mopo.py:554 skips the rollouts); every row comes from the env pool
        self._sac._do_training(first_timestep, self._pool, getattr(self, '_model_pool', None), n_steps=n_steps,
                               seed=self._seed + 7919 * self._epoch, n_train_repeat=self._n_train_repeat)
        self._num_train_steps += n_steps
        return self._sac.logs()

    def _train_epoch(self):
        """One epoch of mopo.py:536-573: a model rollout at every ``model_train_freq``-th timestep
        (mopo.py:554-563; all D4RL configs: one, at timestep 0), and between rollouts the SAC steps of
        those timesteps (``n_train_repeat`` per timestep, mopo.py:780-799).  The k-th rollout of epoch e
        draws its Philox streams under the key e * rollouts_per_epoch + k (= e for one rollout per epoch)."""
        import torch
        f = self._model_train_freq
        per_epoch = -(-self._epoch_length // f)
        metrics, logs = {}, {}
        t_roll = t_train = 0.0
        for k, ts in enumerate(range(0, self._epoch_length, f)):
            t0 = time.perf_counter()
            if self._real_ratio < 1.0:                                                  # mopo.py:554
                self._set_rollout_length()
                self._reallocate_model_pool()
                metrics.update(self._rollout_model(self._rollout_batch_size,
                                                   rollout_key=self._epoch * per_epoch + k))
                torch.cuda.synchronize()
            t1 = time.perf_counter()
            logs = self._do_training_repeats(min(f, self._epoch_length - ts) * self._n_train_repeat, first_timestep=ts)
            t_roll, t_train = t_roll + t1 - t0, t_train + time.perf_counter() - t1
        t2 = time.perf_counter()
        evaluation = self._evaluate()
        t3 = time.perf_counter()
        diag = OrderedDict()
        diag.update(('evaluation/' + k, evaluation[k]) for k in sorted(evaluation))
        diag.update(('model/' + k, v) for k, v in metrics.items())
        diag.update(('training/' + k, v) for k, v in logs.items())
        diag.update({'Q_loss': (logs['Q/q1_loss'] + logs['sac_Q/q2_loss']) / 2, 'alpha': logs['sac_pi/alpha'],
                     'epoch': self._epoch, 'train-steps': self._num_train_steps,
                     'times/epoch_rollout_model': t_roll, 'times/train': t_train,
                     'times/evaluation_paths': t3 - t2})
        if evaluation:
            from .evaluation import perf_metrics
            diag.update(perf_metrics(evaluation, self.min_ret, self.max_ret))
        return diag

    # -- mopo.py:575-584: the current policy (deterministic: tanh(mu)) in the evaluation environment
    def _evaluate(self):
        from .evaluation import DevicePolicy, evaluate_rollouts, evaluation_paths
        if self._evaluation_environment is None:
            return {}
        policy = DevicePolicy(self._sac.policy_params_ptr, self._obs_dim, self._act_dim, self._pi_hidden,
                              deterministic=self._eval_deterministic)
        paths = evaluation_paths(self._evaluation_environment, policy, self._eval_n_episodes, self._max_path_length)
        return evaluate_rollouts(paths, self._evaluation_environment) if paths else {}

    def train(self, n_epochs=None):
        """Generator of per-epoch diagnostics (mopo.py:650-651)."""
        if self._model_train_metrics is None:                                            # mopo.py:526-531
            t0 = time.perf_counter()
            max_epochs = 1 if self._model.model_loaded else None
            if self._rank == 0:   # multi-GPU: rank 0 trains, the others receive its packed weights below
                self._model_train_metrics = self._train_model(batch_size=256, max_epochs=max_epochs,
                                                              holdout_ratio=0.2, max_t=self._max_model_t)
            if self._world > 1:
                from .distributed import broadcast_model, broadcast_numpy_rng, broadcast_metrics, wait_for_src
                wait_for_src(self._wait_group)   # no RCCL collective is pending while rank 0 trains
                broadcast_model(self._model)
                broadcast_numpy_rng()       # the training loop drew from numpy's global stream on rank 0 only
                self._model_train_metrics = broadcast_metrics(self._model_train_metrics)
            self._model_train_metrics['train_time'] = time.perf_counter() - t0
        for self._epoch in range(self._epoch, n_epochs or self._n_epochs):
            d = self._train_epoch()
            d.update(('model/' + k, v) for k, v in self._model_train_metrics.items())
            yield d

    def get_diagnostics(self):
        return self._sac.get_diagnostics()


def from_config(params, pool, static_fns, model_load_dir=None, **overrides):
    """Build MOPO from ``mopo_amd.config.get_params(...)`` (examples/config/d4rl dicts)."""
    from .config import DIMS
    kw = dict(params['kwargs'])
    kw.update(overrides)
    obs_dim, act_dim = DIMS[params['domain']]
    kw.setdefault('model_load_dir', model_load_dir)
    return MOPO(pool, static_fns, obs_dim, act_dim, **kw)
