"""Oracle: MOPO._rollout_model horizon loop.  TEST INFRASTRUCTURE ONLY.

Follows (reference xionghuichen/mopo):
  * ``MOPO._rollout_model``          mopo/algorithms/mopo.py:723-765
  * start states ``sampler.random_batch`` -> ``pool.random_batch``  softlearning/samplers/simple_sampler.py:103-108
  * ``get_action_meta`` (policy noise is TF's; injected here)       mopo/algorithms/mopo.py:468-485
  * ``_set_rollout_length`` schedule                               mopo/algorithms/mopo.py:675-684
  * ``_reallocate_model_pool`` sizing + sample carry-over          mopo/algorithms/mopo.py:689-711

RNG order per rollout (numpy legacy global state): randint(size, B) start rows; then per
step normal(E, B_i, D) and choice(elites, B_i).  Policy noise eps_act[i] ([B_i, A]) is injected.
"""
import numpy as np

from . import fake_env as ofe
from . import sac as osac


def model_pool_size(rollout_batch_size, epoch_length, model_train_freq, rollout_length, retain_epochs):
    """mopo.py:693-695"""
    rollouts_per_epoch = rollout_batch_size * epoch_length / model_train_freq
    model_steps_per_epoch = int(rollout_length * rollouts_per_epoch)
    return retain_epochs * model_steps_per_epoch


def rollout_length(epoch, schedule):
    """mopo.py:675-684: linear ramp from min_length (epoch <= min_epoch) to max_length (epoch >= max_epoch),
    truncated to int."""
    min_epoch, max_epoch, min_length, max_length = schedule
    if epoch <= min_epoch:
        y = min_length
    else:
        y = min((epoch - min_epoch) / (max_epoch - min_epoch), 1) * (max_length - min_length) + min_length
    return int(y)


def reallocate(pool, obs_dim, act_dim, rollout_batch_size, epoch_length, model_train_freq, rollout_length,
               retain_epochs):
    """mopo.py:689-711 on an oracle ``Pool`` (None: first allocation).  Returns the pool to use: the
    same object when the size is unchanged, else a new pool holding ``return_all_samples()``."""
    from .replay_pool import Pool
    size = model_pool_size(rollout_batch_size, epoch_length, model_train_freq, rollout_length, retain_epochs)
    if pool is None:
        return Pool(obs_dim, act_dim, size)
    if pool._max_size == size:
        return pool
    new = Pool(obs_dim, act_dim, size)
    new.add_samples(pool.return_all_samples())
    assert new.size == pool.size
    return new


def rollout(env_pool, model_pool, bnn_params, elites, pi_params, B, horizon, termination_fn,
            penalty_coeff, penalty_learned_var=True, eps_act=None, start_idx=None,
            noise=None, model_inds=None):
    """Returns dict(mean_rollout_length, steps_added list).  ``eps_act[i]`` may be a callable
    taking B_i.  ``noise``/``model_inds`` (lists per step) may inject the FakeEnv streams."""
    if start_idx is None:
        start_idx = env_pool.random_indices(B)                      # flexible_replay_pool.py:85-87
    obs = env_pool.batch_by_indices(start_idx)['observations']      # mopo.py:727-728
    steps_added = []
    for i in range(horizon):                                        # mopo.py:730
        Bi = len(obs)
        e = eps_act[i] if not callable(eps_act) else eps_act(Bi)
        act, _ = osac.actor_act(pi_params, obs.astype(np.float32).astype(np.float64), e)
        act = act.astype(np.float32)                                # TF session returns f32
        nz = None if noise is None else noise[i]
        mi = None if model_inds is None else model_inds[i]
        next_obs, rew, term, info = ofe.step(bnn_params, elites, obs, act, termination_fn,
                                             penalty_coeff=penalty_coeff,
                                             penalty_learned_var=penalty_learned_var,
                                             noise=nz, model_inds=mi)  # mopo.py:747
        steps_added.append(len(obs))                                # mopo.py:748
        model_pool.add_samples({'observations': obs, 'actions': act, 'next_observations': next_obs,
                                'rewards': rew, 'terminals': term})  # mopo.py:750-751
        nonterm = ~term.squeeze(-1)                                 # mopo.py:753
        if nonterm.sum() == 0:
            break
        obs = next_obs[nonterm]                                     # mopo.py:758
    return {'mean_rollout_length': sum(steps_added) / B, 'steps_added': steps_added}
