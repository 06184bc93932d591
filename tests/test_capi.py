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


@pytest.mark.parametrize('skip', [0, 1, 623])
def test_mt19937_block_draws_bit_exact_and_leave_numpy_state(skip):
    """The block-wise randint / random_sample (BNN.train's bootstrap indices and shuffle keys,
    bnn.py:385-387, 402) at that call's size, starting at any stream position (a random_sample pair
    straddling a reload included): same values and the same generator state afterwards as numpy."""
    from mopo_amd.rng import LegacyRandomState
    r = LegacyRandomState(0)
    n = 5003
    for draw in ('randint32', 'randint64', 'uniform'):
        np.random.seed(7)
        np.random.randint(0, 2 ** 32 - 1, size=skip, dtype=np.uint64)  # one 32-bit draw each
        r.sync_from_numpy()
        if draw == 'uniform':
            exp = np.random.uniform(size=[7, n])
            got = r.random_sample([7, n], out=np.empty(7 * n))
        else:
            exp = np.random.randint(n, size=[7, n])
            dt = np.int32 if draw == 'randint32' else np.int64
            got = r.randint(0, n, [7, n], out=np.empty(7 * n, dt))
        np.testing.assert_array_equal(got, exp)
        st_np, st_r = np.random.get_state(), r.get_state()
        np.testing.assert_array_equal(st_np[1], st_r[1])
        assert st_np[2:] == st_r[2:]
    with pytest.raises(ValueError):
        r.randint(0, 5, [4], out=np.empty(3, np.int32))


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


@pytest.mark.parametrize('E,O,A,H', [(7, 17, 6, 200), (7, 11, 3, 200), (5, 17, 6, 256), (16, 17, 6, 32), (1, 3, 1, 8)])
def test_train_weight_gradient_tile_lists(E, O, A, H):
    """The training step's weight-gradient tiles (bnn_train.hip make_wlist, host only): every (layer,
    member, tile row, tile column) of the 5 layers exactly once over the 8 XCD lists, the lists within one
    tile of an even share, and -- except the overflow past that share -- member e's tiles on list e mod 8."""
    from mopo_amd import _lib
    L = _lib.lib()
    fn = L.mopo_bnn_train_tile_lists
    per = fn(E, O, A, H, None, 0)
    assert per > 0
    out = np.empty(8 * per + 8, np.int32)
    assert fn(E, O, A, H, out.ctypes.data, out.size) == per
    cnt = out[8 * per:]
    IN, D = O + A, O + 1
    dims = [(IN, H), (H, H), (H, H), (H, H), (H, 2 * D)]
    want = {(l, e, tm, tn) for e in range(E) for l, (K, N) in enumerate(dims)
            for tm in range(-(-K // 32)) for tn in range(-(-N // 32))}
    got, home = [], 0
    for x in range(8):
        lst = out[x * per:x * per + cnt[x]]
        assert np.all(out[x * per + cnt[x]:(x + 1) * per] == -1)
        for v in lst:
            t = (v & 7, (v >> 3) & 15, (v >> 7) & 31, (v >> 12) & 31)
            got.append(t)
            home += t[1] % 8 == x
    assert len(got) == len(set(got)) and set(got) == want
    assert cnt.max() - cnt.min() <= 1
    target = -(-len(want) // 8)
    per_member = len(want) // E
    # tiles kept at home: all of them when the members fill the XCDs evenly, at least the even share otherwise
    assert home >= min(len(want), sum(min(per_member * len(range(x, E, 8)), target) for x in range(8)))
    with pytest.raises(Exception):
        _lib.check(fn(E, O, A, H, out.ctypes.data, 3))
