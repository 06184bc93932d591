"""Oracle: FakeEnv.step + termination functions, numpy restatement.  TEST INFRASTRUCTURE ONLY.

Follows (reference xionghuichen/mopo):
  * ``FakeEnv.step``           mopo/models/fake_env.py:37-131
  * ``FakeEnv._get_logprob``   mopo/models/fake_env.py:20-35
  * ``BNN.random_inds``        mopo/models/bnn.py:342-344
  * termination functions      mopo/static/halfcheetah.py:6-11, walker2d.py:6-17, hopper.py:6-18,
                               ant.py:6-17, antangle.py:6-17, humanoid.py:7-15 and the never-done
                               halfcheetahjump/vel/veljump, point2denv, point2dwallenv, pendulum

Pinned against golden vectors from the reference's own ``FakeEnv.step`` and
``mopo/static`` (tests/golden/make_golden.py).
"""
import numpy as np

from . import bnn as obnn


# ---- termination functions (mopo/static/*.py) ---------------------------------------------
def term_halfcheetah(obs, act, next_obs):
    # halfcheetah.py:6-11  -> never done
    return np.zeros((len(obs), 1), dtype=bool)


def term_walker2d(obs, act, next_obs):
    # walker2d.py:6-17
    h, a = next_obs[:, 0], next_obs[:, 1]
    not_done = (h > 0.8) * (h < 2.0) * (a > -1.0) * (a < 1.0)
    return (~not_done)[:, None]


def term_hopper(obs, act, next_obs):
    # hopper.py:6-18; note np.abs(bool_array) at hopper.py:12 is the bool array itself
    h, a = next_obs[:, 0], next_obs[:, 1]
    not_done = (np.isfinite(next_obs).all(axis=-1)
                * (next_obs[:, 1:] < 100).all(axis=-1)
                * (h > .7) * (np.abs(a) < .2))
    return (~not_done)[:, None]


def term_ant(obs, act, next_obs):
    # ant.py:6-17 (antangle.py is the same rule)
    x = next_obs[:, 0]
    not_done = np.isfinite(next_obs).all(axis=-1) * (x >= 0.2) * (x <= 1.0)
    return (~not_done)[:, None]


def term_humanoid(obs, act, next_obs):
    # humanoid.py:7-15; bool + bool is logical or
    z = next_obs[:, 0]
    return ((z < 1.0) | (z > 2.0))[:, None]


TERMINATION = {'halfcheetah': term_halfcheetah, 'walker2d': term_walker2d, 'hopper': term_hopper,
               'ant': term_ant, 'antangle': term_ant, 'humanoid': term_humanoid}
for _d in ('halfcheetahjump', 'halfcheetahvel', 'halfcheetahveljump', 'point2denv', 'point2dwallenv'):
    TERMINATION[_d] = term_halfcheetah
# pendulum.py:9 returns np.zeros((n, 1)) (float); its truth value is the never-done rule
TERMINATION['pendulum'] = term_halfcheetah


def get_logprob(x, means, variances):
    """fake_env.py:20-35 (naive exp-then-log; may underflow to -inf like the reference)."""
    k = x.shape[-1]
    log_prob = -1 / 2 * (k * np.log(2 * np.pi) + np.log(variances).sum(-1)
                         + (np.power(x - means, 2) / variances).sum(-1))
    with np.errstate(divide='ignore'):
        prob = np.exp(log_prob).sum(0)
        log_prob = np.log(prob)
    stds = np.std(means, 0).mean(-1)
    return log_prob, stds


def step(params, elites, obs, act, termination_fn, penalty_coeff=0.0, penalty_learned_var=False,
         deterministic=False, noise=None, model_inds=None, predicted=None):
    """FakeEnv.step (fake_env.py:37-131) with the ensemble forward of ``oracle.bnn``.

    RNG order follows the reference: ``np.random.normal(size=[E,B,D])`` (fake_env.py:72)
    then ``np.random.choice(elites, B)`` (bnn.py:343).  Either stream may be injected.
    Returns next_obs, penalized_rewards, terminals, info (same keys as fake_env.py:129-130).
    ``predicted=(mean, var)`` replaces the forward (e.g. the reference graph's own f32 outputs).
    """
    return_single = obs.ndim == 1
    if return_single:
        obs, act = obs[None], act[None]
    inputs = np.concatenate((obs, act), axis=-1)                       # fake_env.py:46
    if predicted is None:
        means, variances = obnn.forward(params, inputs)                # fake_env.py:50-64 (chunking is row-independent)
    else:
        means, variances = (np.array(a, np.float32) for a in predicted)
    means[:, :, 1:] += obs                                             # fake_env.py:66 (in-place, stays f32)
    stds = np.sqrt(variances)                                          # fake_env.py:67
    E, B, _ = means.shape
    if deterministic:
        samples_all = means                                            # fake_env.py:69-70
    else:
        if noise is None:
            noise = np.random.normal(size=means.shape)                 # fake_env.py:72
        samples_all = means + noise * stds                             # -> float64
    if not deterministic:
        if model_inds is None:
            model_inds = np.random.choice(elites, size=B)              # bnn.py:343
        bidx = np.arange(0, B)
        samples = samples_all[model_inds, bidx]                        # fake_env.py:79-81
        model_means = means[model_inds, bidx]
        model_stds = stds[model_inds, bidx]
    else:
        samples = np.mean(samples_all, axis=0)                         # fake_env.py:84-86
        model_means = np.mean(means, axis=0)
        model_stds = np.mean(stds, axis=0)
    log_prob, dev = get_logprob(samples, means, variances)             # fake_env.py:88
    rewards, next_obs = samples[:, :1], samples[:, 1:]                 # fake_env.py:90
    terminals = termination_fn(obs, act, next_obs)                     # fake_env.py:91
    return_means = np.concatenate((model_means[:, :1], terminals, model_means[:, 1:]), axis=-1)
    return_stds = np.concatenate((model_stds[:, :1], np.zeros((B, 1)), model_stds[:, 1:]), axis=-1)
    if penalty_coeff != 0:
        if not penalty_learned_var:                                    # fake_env.py:98-108
            ens_obs = means[:, :, 1:]
            diffs = ens_obs - np.mean(ens_obs, axis=0)
            penalty = np.max(np.linalg.norm(diffs, axis=2), axis=0)
        else:                                                          # fake_env.py:110
            penalty = np.amax(np.linalg.norm(stds, axis=2), axis=0)
        penalty = np.expand_dims(penalty, 1)
        unpenalized = rewards
        penalized = rewards - penalty_coeff * penalty                  # fake_env.py:115
    else:
        penalty, unpenalized, penalized = None, rewards, rewards
    if return_single:
        next_obs, return_means, return_stds = next_obs[0], return_means[0], return_stds[0]
        unpenalized, penalized, terminals = unpenalized[0], penalized[0], terminals[0]
    info = {'mean': return_means, 'std': return_stds, 'log_prob': log_prob, 'dev': dev,
            'unpenalized_rewards': unpenalized, 'penalty': penalty, 'penalized_rewards': penalized,
            'model_inds': model_inds}
    return next_obs, penalized, terminals, info
