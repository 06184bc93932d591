"""Env-pool ingress (``mopo.off_policy.loader``).

``restore_pool_d4rl`` (mopo/off_policy/loader.py:23-29) calls ``d4rl.qlearning_dataset`` and adds
``observations, actions, next_observations, rewards[:,None], terminals[:,None]`` to the pool.
d4rl/gym/h5py are not installed and there is no network, so this reads the same arrays from a
local ``.npz`` (the qlearning_dataset layout); ``format_samples_for_training``
(mopo/models/constructor.py:46-57) is provided for the (later-round) ensemble training.
"""
import numpy as np

KEYS = ('observations', 'actions', 'next_observations', 'rewards', 'terminals')


def load_qlearning_npz(path):
    z = np.load(path, allow_pickle=False)
    missing = [k for k in KEYS if k not in z]
    if missing:
        raise KeyError('%s lacks %s (qlearning_dataset layout expected)' % (path, missing))
    data = {k: z[k] for k in KEYS}
    if data['rewards'].ndim == 1:
        data['rewards'] = data['rewards'][:, None]       # loader.py:27
    if data['terminals'].ndim == 1:
        data['terminals'] = data['terminals'][:, None]   # loader.py:28
    return data


def restore_pool(pool, path, max_size=None):
    """loader.py:8-20 for a local file; returns the number of rows added."""
    data = load_qlearning_npz(path)
    pool.add_samples(data)
    return len(data['observations'])


def format_samples_for_training(samples):
    """constructor.py:46-57: inputs (obs, act) -> targets (rew, next_obs - obs)."""
    obs, act = samples['observations'], samples['actions']
    delta = samples['next_observations'] - obs
    return np.concatenate((obs, act), axis=-1), np.concatenate((samples['rewards'], delta), axis=-1)
