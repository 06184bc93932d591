"""Evaluation rollouts in a real environment and the normalized return (host loop around the device policy).

Reference: ``RLAlgorithm._evaluation_paths`` / ``_evaluate_rollouts`` (softlearning/algorithms/
rl_algorithm.py:258-304), ``rollout`` / ``rollouts`` (softlearning/samplers/utils.py:36-92), MOPO's
deterministic evaluation policy and ``perf/*`` keys (mopo/algorithms/mopo.py:577-629), the D4RL env
name and reference scores (mopo.py:115-123, d4rl.infos).  The environment is any object with the gym
API (``reset() -> obs``, ``step(action) -> (obs, reward, done, info)``): MuJoCo is not in this image,
so the caller supplies it.  Actions come from the device actor (``mopo_actor_forward_dtype``): the
deterministic branch of get_action_meta, tanh(mu) (mopo.py:481-482).
"""
from collections import OrderedDict

import numpy as np

from . import _lib as L

# d4rl/infos.py REF_MIN_SCORE / REF_MAX_SCORE of the MuJoCo v0 tasks the configs name (random-policy and
# expert returns per domain; d4rl is not installed here, so the published constants are restated)
_DOMAIN_REF = {'halfcheetah': (-280.178953, 12135.0), 'hopper': (-20.272305, 3234.3),
               'walker2d': (1.629008, 4592.3)}
_DATASETS = ('random', 'medium', 'expert', 'medium-replay', 'medium-expert')
REF_MIN_SCORE = {'%s-%s-v0' % (d, s): v[0] for d, v in _DOMAIN_REF.items() for s in _DATASETS}
REF_MAX_SCORE = {'%s-%s-v0' % (d, s): v[1] for d, v in _DOMAIN_REF.items() for s in _DATASETS}


def env_name_of(model_name):
    """mopo.py:115-118: '<task>_smv_1_0' -> '<task>-v0'."""
    return (model_name[:-8] if '_smv' in model_name else model_name[:-4]) + '-v0'


def ref_scores(model_name):
    """(min_ret, max_ret) of mopo.py:119-123 (0, 0 when the task is not a D4RL one)."""
    n = env_name_of(model_name or '')
    return (REF_MIN_SCORE[n], REF_MAX_SCORE[n]) if n in REF_MIN_SCORE else (0.0, 0.0)


class DevicePolicy:
    """The current policy on the device: ``actions(obs[B, O]) -> [B, A]`` (deterministic: tanh(mu))."""

    def __init__(self, pi_params, obs_dim, act_dim, hidden=256, deterministic=True, dtype=0):
        self.P, self.O, self.A, self.H = pi_params, obs_dim, act_dim, hidden
        self.deterministic, self.dtype = deterministic, dtype
        self._step = 0

    def actions(self, obs):
        import torch
        o = torch.as_tensor(np.ascontiguousarray(obs, np.float32)).cuda()
        if o.dim() == 1:
            o = o[None]
        B = int(o.shape[0])
        act = torch.empty((B, self.A), dtype=torch.float32, device=o.device)
        mu = torch.empty_like(act)
        ptr = self.P if isinstance(self.P, int) else L.ptr(self.P)
        self._step += 1
        L.check(L.lib().mopo_actor_forward_dtype(ptr, self.O, self.A, self.H, L.ptr(o), 0, B, None, 2024,
                                                 self._step, L.ptr(act), L.ptr(mu), self.dtype, L.stream_ptr()))
        return (mu if self.deterministic else act).cpu().numpy()


def rollout(env, policy, path_length, break_on_terminal=True):
    """One episode (samplers/utils.py:36-80): observations, actions, rewards, terminals, next_observations."""
    obs = env.reset()
    path = {k: [] for k in ('observations', 'actions', 'rewards', 'terminals', 'next_observations')}
    infos = []
    for t in range(path_length):
        a = policy.actions(np.asarray(obs)[None])[0]
        nobs, r, done, info = env.step(a)
        for k, v in zip(path, (obs, a, [r], [done], nobs)):
            path[k].append(np.asarray(v))
        infos.append(info)
        obs = nobs
        if done and break_on_terminal:
            break
    out = {k: np.stack(v) for k, v in path.items()}
    out['infos'] = infos
    return out


def evaluation_paths(env, policy, n_episodes, path_length):
    """_evaluation_paths (rl_algorithm.py:258-279): ``n_episodes`` rollouts, none if n_episodes < 1."""
    return [rollout(env, policy, path_length) for _ in range(n_episodes)] if n_episodes >= 1 else []


def evaluate_rollouts(paths, env=None):
    """_evaluate_rollouts (rl_algorithm.py:281-304)."""
    total = [float(np.sum(p['rewards'])) for p in paths]
    lengths = [len(p['rewards']) for p in paths]
    d = OrderedDict((('return-average', np.mean(total)), ('return-min', np.min(total)),
                     ('return-max', np.max(total)), ('return-std', np.std(total)),
                     ('episode-length-avg', np.mean(lengths)), ('episode-length-min', np.min(lengths)),
                     ('episode-length-max', np.max(lengths)), ('episode-length-std', np.std(lengths))))
    if env is not None and hasattr(env, 'get_path_infos'):
        for k, v in env.get_path_infos(paths).items():
            d['env_infos/{}'.format(k)] = v
    return d


def perf_metrics(evaluation, min_ret, max_ret):
    """mopo.py:623-629: perf/AverageReturn, perf/AverageLength, perf/NormalizedReturn (D4RL tasks)."""
    out = OrderedDict([('perf/AverageReturn', evaluation['return-average']),
                       ('perf/AverageLength', evaluation['episode-length-avg'])])
    if min_ret != max_ret:
        out['perf/NormalizedReturn'] = (out['perf/AverageReturn'] - min_ret) / (max_ret - min_ret)
    return out
