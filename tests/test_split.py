"""CPU: the bf16x6 operand split (mlp_tile.h split_bf16 / split_bf16_pair) restated in numpy and held to its
exactness claim -- three round-to-nearest-even bf16 parts reproduce every f32 x with 2^-100 <= |x| < 2^127
bit for bit (x0 + x1 + x2 == x), |x1| <= 2^-8 |x|, |x2| <= 2^-16 |x|, so the three products the ensemble kernels
drop (x1 w2, x2 w1, x2 w2) total at most (2^-23 + 2^-32) |x w| -- over sampled and extreme exponents and
significands, including the round-half-even ties."""
import numpy as np
import pytest


def bf16_rn(x):
    """v_cvt_pk_bf16_f32 on finite f32: round to nearest, ties to even, on the upper 16 bits."""
    u = np.asarray(x, np.float32).view(np.uint32).astype(np.uint64)
    r = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return r.astype(np.uint32).view(np.float32)


def split3(x):
    x = np.asarray(x, np.float32)
    p0 = bf16_rn(x)
    r1 = (x - p0).astype(np.float32)
    p1 = bf16_rn(r1)
    r2 = (r1 - p1).astype(np.float32)
    p2 = bf16_rn(r2)
    return p0, p1, p2, r1, r2


def samples():
    rs = np.random.RandomState(0)
    exps = np.arange(-100, 127)
    mants = np.concatenate([rs.randint(0, 1 << 23, size=200), [0, 1, 0x7FFFFF, 0x400000, 0x7F8000, 0x008000, 0x00FFFF,
                                                               0x7F7FFF, 0x0080FF, 0x3FFFFF, 0x7FFF80, 0x000080]])
    # every exponent with every mantissa pattern; the ties (bit 15 set, bits below zero) round to even
    e = (exps + 127).astype(np.uint32)[:, None]
    m = mants.astype(np.uint32)[None, :]
    u = (e << 23) | m
    x = u.ravel().view(np.float32)
    return np.concatenate([x, -x, np.float32([0.0])])


def test_split_is_exact_in_range():
    x = samples()
    p0, p1, p2, r1, r2 = split3(x)
    # each residual is an exact f32 subtraction
    assert np.all(r1.astype(np.float64) == x.astype(np.float64) - p0.astype(np.float64))
    assert np.all(r2.astype(np.float64) == r1.astype(np.float64) - p1.astype(np.float64))
    # the parts reproduce x bit for bit
    s = p0.astype(np.float64) + p1.astype(np.float64) + p2.astype(np.float64)
    bad = s != x.astype(np.float64)
    assert not bad.any(), x[bad][:8]
    assert np.all(p2 == r2)
    ax = np.abs(x.astype(np.float64))
    assert np.all(np.abs(p1) <= 2.0 ** -8 * ax)
    assert np.all(np.abs(p2) <= 2.0 ** -16 * ax)
    # every part is a bf16 value (low 16 bits zero) and normal or zero
    for p in (p0, p1, p2):
        u = p.view(np.uint32)
        assert np.all(u & 0xFFFF == 0)
        assert np.all((np.abs(p) >= 2.0 ** -126) | (p == 0))


@pytest.mark.parametrize('seed', [1, 2])
def test_dropped_products_bound(seed):
    """The 6-product form sum_{p+q<3} x_p w_q differs from the exact f64 product x w by at most
    (2^-23 + 2^-32) |x w| (x1 w2 + x2 w1 + x2 w2 are dropped; every kept bf16 x bf16 product is exact in f32)."""
    rs = np.random.RandomState(seed)
    n = 200000
    x = (rs.normal(size=n) * np.exp2(rs.randint(-40, 40, n))).astype(np.float32)
    w = (rs.normal(size=n) * np.exp2(rs.randint(-20, 20, n))).astype(np.float32)
    xp, wp = split3(x)[:3], split3(w)[:3]
    kept = sum(xp[p].astype(np.float64) * wp[q].astype(np.float64) for p in range(3) for q in range(3) if p + q < 3)
    exact = x.astype(np.float64) * w.astype(np.float64)
    err = np.abs(kept - exact)
    assert np.all(err <= (2.0 ** -23 + 2.0 ** -32) * np.abs(exact))
    # and each kept product is exact in f32 (8 x 8 significand bits)
    for p in range(3):
        for q in range(3 - p):
            pr = xp[p].astype(np.float64) * wp[q].astype(np.float64)
            assert np.all(pr.astype(np.float32).astype(np.float64) == pr)

