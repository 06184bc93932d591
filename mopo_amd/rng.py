"""numpy legacy RandomState replica (C++, csrc/mt19937.cpp) with state exchange.

``LegacyRandomState`` reproduces np.random.RandomState draws bit-exactly (normal, randint,
random_sample); ``sync_from_numpy``/``sync_to_numpy`` move the global np.random state in and out
so large parity-mode streams can be produced natively while the caller's np.random stream advances
exactly as the reference's would (fake_env.py:72, bnn.py:343, flexible_replay_pool.py:87).
"""
import ctypes as C

import numpy as np

from . import _lib as L


class LegacyRandomState:
    def __init__(self, seed=0):
        h = C.c_void_p()
        L.check(L.lib().mopo_mt_create(C.byref(h), int(seed) & 0xffffffff))
        self._h = h

    def __del__(self):
        h = getattr(self, '_h', None)
        if h is not None and h.value:
            L.lib().mopo_mt_destroy(h)
            self._h = None

    def seed(self, s):
        L.check(L.lib().mopo_mt_seed(self._h, int(s) & 0xffffffff))

    def normal(self, size):
        n = int(np.prod(size))
        out = np.empty(n, np.float64)
        L.check(L.lib().mopo_mt_normal(self._h, out.ctypes.data, n))
        return out.reshape(size)

    def random_sample(self, size, out=None):
        """``out``: an optional C-contiguous float64 array (e.g. a pinned host tensor's numpy view) the
        draws are written into."""
        n = int(np.prod(size))
        out = np.empty(n, np.float64) if out is None else _check_out(out, n, np.float64)
        L.check(L.lib().mopo_mt_random_sample(self._h, out.ctypes.data, n))
        return out.reshape(size)

    def randint(self, low, high, size, out=None):
        """np.random.randint(low, high, size); ``out`` may be int64 or int32 (the same draws)."""
        n = int(np.prod(size))
        if out is not None and out.dtype == np.int32:
            out = _check_out(out, n, np.int32)
            L.check(L.lib().mopo_mt_randint_i32(self._h, out.ctypes.data, n, int(low), int(high)))
            return out.reshape(size)
        out = np.empty(n, np.int64) if out is None else _check_out(out, n, np.int64)
        L.check(L.lib().mopo_mt_randint(self._h, out.ctypes.data, n, int(low), int(high)))
        return out.reshape(size)

    def choice(self, a, size):
        a = np.asarray(a)
        return a[self.randint(0, len(a), size)]

    def get_state(self):
        key = np.empty(624, np.uint32)
        pos, hg, g = C.c_int(), C.c_int(), C.c_double()
        L.check(L.lib().mopo_mt_get_state(self._h, key.ctypes.data, C.byref(pos), C.byref(hg), C.byref(g)))
        return ('MT19937', key, pos.value, hg.value, g.value)

    def set_state(self, st):
        key = np.ascontiguousarray(st[1], np.uint32)
        L.check(L.lib().mopo_mt_set_state(self._h, key.ctypes.data, int(st[2]), int(st[3]), float(st[4])))

    def sync_from_numpy(self):
        self.set_state(np.random.get_state())

    def sync_to_numpy(self):
        np.random.set_state(self.get_state())


def _check_out(out, n, dtype):
    if out.dtype != dtype or out.size != n or not out.flags['C_CONTIGUOUS'] or not out.flags['WRITEABLE']:
        raise ValueError('out must be a writeable C-contiguous %s array of %d elements' % (np.dtype(dtype).name, n))
    return out
