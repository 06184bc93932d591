"""CPU: non-square policy / Q hidden_sizes [H1, H2] (mopo.py:275-280, 311-325) run on the device as the
square device_hidden() network with the narrower layer zero-padded (mopo_amd/rollout.py).  These tests pin
the index map and show in the f64 oracle that the embedding is exact over SAC steps: the padded network's
losses, parameters, targets and Adam moments equal the [H1, H2] network's, and its padding stays 0."""
import numpy as np
import pytest

from oracle import sac as osac


def _pad(O, A, hs):
    from mopo_amd.rollout import device_hidden, sac_pad_index, sac_param_shapes
    return device_hidden(hs), sac_pad_index(O, A, hs), sac_param_shapes(O, A, hs)


def test_pad_index_maps_each_tensor_corner():
    from mopo_amd.rollout import sac_param_shapes
    O, A, hs = 17, 6, (256, 128)
    hd, idx, shapes = _pad(O, A, hs)
    assert hd == 256 and idx.size == sum(int(np.prod(s)) for s in shapes)
    assert len(np.unique(idx)) == idx.size
    dshapes = sac_param_shapes(O, A, hd)
    dev = np.zeros(sum(int(np.prod(s)) for s in dshapes))
    logical = np.arange(1, idx.size + 1, dtype=np.float64)
    dev[idx] = logical
    off_l = off_d = 0
    for ls, ds in zip(shapes, dshapes):
        dt = dev[off_d:off_d + int(np.prod(ds))].reshape(ds)
        lt = logical[off_l:off_l + int(np.prod(ls))].reshape(ls)
        corner = dt[tuple(slice(0, n) for n in ls)]
        np.testing.assert_array_equal(corner, lt)
        assert dt.sum() == lt.sum()          # nothing outside the corner
        off_l += int(np.prod(ls))
        off_d += int(np.prod(ds))
    from mopo_amd.rollout import device_hidden, sac_pad_index
    assert device_hidden(200) == 208 and device_hidden((48, 200)) == 208 and device_hidden([256, 256]) == 256
    assert sac_pad_index(O, A, 256) is None and sac_pad_index(O, A, (256, 256)) is None
    with pytest.raises(NotImplementedError):
        device_hidden((256, 256, 256))


@pytest.mark.parametrize('hs', [(256, 128), (48, 200)])
def test_zero_padding_is_exact_in_the_oracle(hs):
    O, A, n = 11, 3, 64
    rs = np.random.RandomState(3)
    hd, idx, shapes = _pad(O, A, hs)
    P = [p + 0.02 * rs.normal(size=p.shape) for p in osac.init_params(O, A, hs, seed=4)]
    flat = np.concatenate([p.ravel() for p in P])
    dshapes = osac.param_shapes(O, A, hd)
    dflat = np.zeros(sum(int(np.prod(s)) for s in dshapes))
    dflat[idx] = flat
    D, off = [], 0
    for s in dshapes:
        D.append(dflat[off:off + int(np.prod(s))].reshape(s))
        off += int(np.prod(s))
    a, b = osac.SACState(P, log_alpha=0.1), osac.SACState(D, log_alpha=0.1)
    for k in range(6):
        batch = {'observations': rs.normal(size=(n, O)), 'actions': rs.uniform(-1, 1, (n, A)),
                 'next_observations': rs.normal(size=(n, O)), 'rewards': rs.normal(size=(n, 1)),
                 'terminals': rs.uniform(size=(n, 1)) < 0.1}
        e1, e2 = rs.normal(size=(n, A)), rs.normal(size=(n, A))
        la = osac.sac_step(a, batch, e1, e2)
        lb = osac.sac_step(b, batch, e1, e2)
        for key in la:
            np.testing.assert_allclose(lb[key], la[key], rtol=1e-12, atol=1e-14, err_msg=key)
    fl = lambda xs: np.concatenate([np.asarray(x).ravel() for x in xs])
    pad = np.ones(dflat.size, bool)
    pad[idx] = False
    for name, xa, xb in (('params', a.params, b.params), ('target', a.target, b.target),
                         ('m', a.opt_pi.m + a.opt_q1.m + a.opt_q2.m, b.opt_pi.m + b.opt_q1.m + b.opt_q2.m),
                         ('v', a.opt_pi.v + a.opt_q1.v + a.opt_q2.v, b.opt_pi.v + b.opt_q1.v + b.opt_q2.v)):
        fb = fl(xb)
        np.testing.assert_allclose(fb[idx], fl(xa), rtol=1e-12, atol=1e-14, err_msg=name)
        assert np.all(fb[pad] == 0), name
