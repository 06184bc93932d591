"""Oracle: SimpleReplayPool / FlexibleReplayPool SoA ring buffer.  TEST INFRASTRUCTURE ONLY.

Follows (reference xionghuichen/mopo):
  * field dtypes/shapes        softlearning/replay_pools/simple_replay_pool.py:48-70
  * ring write + advance       softlearning/replay_pools/flexible_replay_pool.py:45-48, 57-83
  * random_indices (randint)   flexible_replay_pool.py:85-87
  * batch_by_indices           flexible_replay_pool.py:121-135
  * return_all_samples         flexible_replay_pool.py:157-161
Pinned against golden traces of the reference FlexibleReplayPool (tests/golden).
"""
import numpy as np

FIELDS = ('actions', 'rewards', 'terminals', 'observations', 'next_observations')


class Pool:
    def __init__(self, obs_dim, act_dim, max_size):
        self._max_size = int(max_size)
        m = self._max_size
        self.fields = {
            'actions': np.zeros((m, act_dim), np.float32),
            'rewards': np.zeros((m, 1), np.float32),
            'terminals': np.zeros((m, 1), bool),
            'observations': np.zeros((m, obs_dim), np.float32),
            'next_observations': np.zeros((m, obs_dim), np.float32),
        }
        self._pointer = 0
        self._size = 0

    @property
    def size(self):
        return self._size

    def add_samples(self, samples):
        n = samples[next(iter(samples))].shape[0]
        index = np.arange(self._pointer, self._pointer + n) % self._max_size
        for k in FIELDS:
            self.fields[k][index] = samples[k]
        self._pointer = (self._pointer + n) % self._max_size
        self._size = min(self._size + n, self._max_size)

    def random_indices(self, batch_size):
        if self._size == 0:
            return np.arange(0, 0)
        return np.random.randint(0, self._size, batch_size)

    def batch_by_indices(self, indices):
        return {k: self.fields[k][indices] for k in FIELDS}

    def random_batch(self, batch_size):
        return self.batch_by_indices(self.random_indices(batch_size))

    def return_all_samples(self):
        return {k: self.fields[k][:self._size] for k in FIELDS}
