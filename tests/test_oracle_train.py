"""CPU checks of the ensemble-training oracle (oracle/bnn_train.py): the hand-derived gradient
against central differences of the training loss, and the train() loop's control flow."""
import numpy as np
import pytest

from oracle import bnn as obnn
from oracle import bnn_train as ot


def _tiny(E=2, O=3, A=1, H=6, seed=0, smv=True):
    p = obnn.init_params(E, O, A, hidden=H, seed=seed, bias_std=0.1, smv=smv)
    p['max_logvar'] = p['max_logvar'] * 0 + 0.3
    p['min_logvar'] = p['min_logvar'] * 0 - 2.0
    return {k: (v.astype(np.float64) if isinstance(v, np.ndarray) else
                [x.astype(np.float64) for x in v] if isinstance(v, list) else v) for k, v in p.items()}


@pytest.mark.parametrize('smv', [True, False])
def test_loss_gradient_matches_finite_differences(smv):
    rs = np.random.RandomState(1)
    p = _tiny(smv=smv)
    E, IN, D = 2, 4, 4
    X = rs.normal(size=(E, 5, IN))
    Y = rs.normal(size=(E, 5, D))
    loss, g = ot.loss_and_grads(p, X, Y)
    vals = ot.optvars(p)
    eps = 1e-6
    for vi, (v, gv) in enumerate(zip(vals, g)):
        assert gv.shape == v.shape
        flat = v.reshape(-1)
        for j in rs.choice(flat.size, size=min(6, flat.size), replace=False):
            vp = [x.copy() for x in vals]
            vm = [x.copy() for x in vals]
            vp[vi].reshape(-1)[j] += eps
            vm[vi].reshape(-1)[j] -= eps
            lp, _ = ot.loss_and_grads(ot.set_optvars(p, vp), X, Y)
            lm, _ = ot.loss_and_grads(ot.set_optvars(p, vm), X, Y)
            fd = (lp - lm) / (2 * eps)
            assert abs(fd - gv.reshape(-1)[j]) <= 1e-6 * (1 + abs(fd)), (vi, j, fd, gv.reshape(-1)[j])


def test_loss_value_matches_direct_expression():
    rs = np.random.RandomState(2)
    p = _tiny()
    X = rs.normal(size=(2, 7, 4))
    Y = rs.normal(size=(2, 7, 4))
    loss, _ = ot.loss_and_grads(p, X, Y)
    _, mean, lv = ot.forward3d(p, X)
    direct = np.sum(np.mean(np.mean((mean - Y) ** 2 * np.exp(-lv), -1), -1) + np.mean(np.mean(lv, -1), -1))
    direct += sum(w * 0.5 * np.sum(W ** 2) for w, W in zip(ot.WD, p['W'])) + ot.WD_VAR * 0.5 * np.sum(p['Wv'] ** 2)
    direct += 0.01 * np.sum(p['max_logvar']) - 0.01 * np.sum(p['min_logvar'])
    assert loss == pytest.approx(direct, rel=1e-12)


def test_mse_loss_is_the_plain_mean_square():
    rs = np.random.RandomState(3)
    p = _tiny()
    X = rs.normal(size=(2, 6, 4))
    Y = rs.normal(size=(2, 6, 4))
    m = ot.mse_losses(p, X, Y)
    _, mean, _ = ot.forward3d(p, X)
    np.testing.assert_allclose(m, ((mean - Y) ** 2).mean((1, 2)), rtol=1e-12)


def test_train_loop_early_stops_and_picks_elites():
    rs = np.random.RandomState(4)
    E, O, A = 3, 3, 1
    p = _tiny(E=E)
    N = 60
    X = rs.normal(size=(N, O + A)).astype(np.float32)
    Y = np.concatenate([X[:, :1] * 0.5, X[:, :O] * 0.1], 1).astype(np.float32)
    np.random.seed(0)
    q, elites, hl, epochs, updates = ot.train(p, X, Y, num_elites=2, batch_size=16, holdout_ratio=0.2,
                                              max_epochs=30, max_epochs_since_update=2)
    assert len(elites) == 2 and set(elites) <= set(range(E))
    assert list(np.argsort(hl)[:2]) == elites
    assert 1 <= epochs <= 30 and updates == epochs * int(np.ceil((N - 12) / 16))
    # the same seed reproduces the same run (the reference's global-stream call order)
    np.random.seed(0)
    q2, elites2, hl2, _, _ = ot.train(p, X, Y, num_elites=2, batch_size=16, holdout_ratio=0.2, max_epochs=30,
                                      max_epochs_since_update=2)
    assert elites2 == elites
    np.testing.assert_array_equal(hl2, hl)


def _split_joint(p):
    """The joint head [H, 2D] as an smv pair (mean columns, log-var columns)."""
    q = dict(p, smv=True, W=list(p['W']), b=list(p['b']))
    W, b = p['W'][-1], p['b'][-1]
    D = W.shape[-1] // 2
    q['W'][-1], q['b'][-1], q['Wv'], q['bv'] = W[..., :D], b[..., :D], W[..., D:], b[..., D:]
    return q


def test_joint_head_equals_split_heads():
    """bnn.py:183-189 + constructor.py:34-36: the joint head carries the same 0.0001 decay as the
    smv mean and var heads, so its loss and gradients are the smv ones on the split columns (the
    identity the device trainer uses for separate_mean_var=False)."""
    rs = np.random.RandomState(5)
    p = _tiny(smv=False)
    X = rs.normal(size=(2, 9, 4))
    Y = rs.normal(size=(2, 9, 4))
    lj, gj = ot.loss_and_grads(p, X, Y)
    q = _split_joint(p)
    ls, gs = ot.loss_and_grads(q, X, Y)
    assert lj == pytest.approx(ls, rel=1e-13)
    for a, b in zip(gj[:8], gs[:8]):
        np.testing.assert_allclose(a, b, rtol=1e-13)
    np.testing.assert_allclose(gj[8], np.concatenate([gs[8], gs[10]], -1), rtol=1e-13)
    np.testing.assert_allclose(gj[9], np.concatenate([gs[9], gs[11]], -1), rtol=1e-13)
    np.testing.assert_allclose(gj[10], gs[12], rtol=1e-13)
    np.testing.assert_allclose(gj[11], gs[13], rtol=1e-13)
    _, mj, vj = ot.forward3d(p, X)
    _, ms, vs = ot.forward3d(q, X)
    np.testing.assert_allclose(mj, ms, rtol=1e-13)
    np.testing.assert_allclose(vj, vs, rtol=1e-13)
