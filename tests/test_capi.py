"""CPU: the C-ABI library loads, exports every symbol include/mopo_hip.h declares, and its host-only
pieces (numpy legacy RNG replica, parameter counting) behave.  No GPU compute calls here."""
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, 'include', 'mopo_hip.h')).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(mopo_[a-z0-9_]+)\s*\(', src)))


def test_library_exports_all_declared_symbols():
    from mopo_amd import _lib
    L = _lib.lib()
    syms = declared_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(L, s), s
        assert s in _lib.SIGNATURES, 'binding missing for ' + s


def test_param_count_matches_reference_shapes():
    from mopo_amd import _lib
    from mopo_amd.rollout import sac_param_shapes
    n = sum(int(np.prod(s)) for s in sac_param_shapes(17, 6, 256))
    assert _lib.lib().mopo_sac_param_count(17, 6, 256) == n == 73484 + 2 * 72193


@pytest.mark.parametrize('seed', [0, 1, 88, 2 ** 32 - 1])
def test_mt19937_normal_bit_exact(seed):
    from mopo_amd.rng import LegacyRandomState
    r = LegacyRandomState(seed)
    np.random.seed(seed)
    a = np.random.normal(size=1001)          # odd count: exercises the cached second gaussian
    b = np.random.normal(size=(7, 3, 18))
    np.testing.assert_array_equal(r.normal(1001), a)
    np.testing.assert_array_equal(r.normal((7, 3, 18)), b)


@pytest.mark.parametrize('high', [1, 5, 7, 100, 101000, 1000000, 2 ** 31 + 5])
def test_mt19937_randint_choice_bit_exact(high):
    from mopo_amd.rng import LegacyRandomState
    r = LegacyRandomState(123)
    np.random.seed(123)
    np.testing.assert_array_equal(r.randint(0, high, 5000), np.random.randint(0, high, 5000))
    el = [3, 0, 6, 1, 5]
    np.testing.assert_array_equal(r.choice(el, 777), np.random.choice(el, size=777))
    np.testing.assert_array_equal(r.random_sample(99), np.random.random_sample(99))


def test_mt19937_state_exchange_with_numpy():
    from mopo_amd.rng import LegacyRandomState
    np.random.seed(5)
    np.random.normal(size=3)  # leaves a cached gaussian
    r = LegacyRandomState(0)
    r.sync_from_numpy()
    exp = np.random.normal(size=10)
    np.testing.assert_array_equal(r.normal(10), exp)
    r.sync_to_numpy()
    st_np = np.random.get_state()
    st_r = r.get_state()
    np.testing.assert_array_equal(st_np[1], st_r[1])
    assert st_np[2:] == st_r[2:]


def test_error_reporting():
    import ctypes as C
    from mopo_amd import _lib
    L = _lib.lib()
    h = C.c_void_p()
    assert L.mopo_bnn_create(C.byref(h), 0, 17, 6, 200, 1, 0) == -1
    assert b'num_networks' in L.mopo_last_error()
