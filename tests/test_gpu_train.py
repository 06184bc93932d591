"""GPU parity: ensemble training (csrc/bnn_train.hip + the BNN.train host loop) vs the oracle
restatement (oracle/bnn_train.py, pinned by finite differences in test_oracle_train.py).

Tolerances (fp32 device vs fp64 oracle on the same minibatch rows and scaler):
  * one Adam step: every optimised variable |d| <= 1e-6, or 1e-6 + 2.2 lr where the gradient vanishes
    (Adam's first step is lr * sign(g), so a sign flip of a ~0 gradient moves a variable by 2 lr);
  * several steps / an epoch with a partial last minibatch: |d| <= 2e-5 (1 + |ref|);
  * mse evaluation: rel 1e-5; the full train() loop: identical epochs and elites, holdout losses rel 1e-3,
    parameters rtol 1e-3 / atol 1e-4 (at the shipped shape at most 1 in 10^4 elements past that and none past
    2 lr: see assert_trained_close).
Shapes: E=3, O=11, A=3, H=32 (one k-group) and the shipped E=7, O=17, A=6, H=200, batch 256 / 250.
Integer work (shuffle_rows order, formatted rows) is bit-exact.
"""
import ctypes as C

import numpy as np
import pytest

from oracle import bnn as obnn
from oracle import bnn_train as ot

pytestmark = pytest.mark.gpu
E, O, A, H = 3, 11, 3, 32   # hopper-sized inputs (11 + 3 <= 16: one k-group)
IN, D = O + A, O + 1
SMALL = (E, O, A, H)
# the shipped shape: halfcheetah-mixed's ensemble as MOPO.train and bench.py train it (E=7, 23 inputs in two
# k-groups, H=200, 36 head columns): train_rows_kernel<2,13,3> and the H=200 weight-gradient tile lists
SHIPPED = (7, 17, 6, 200)
SHAPES = {'small': SMALL, 'shipped': SHIPPED}


def model(seed=0, shape=SMALL):
    from mopo_amd.bnn import construct_model
    e, o, a, h = shape
    m = construct_model(obs_dim=o, act_dim=a, hidden_dim=h, num_networks=e, num_elites=2, separate_mean_var=True,
                        seed=seed)
    mats = m.get_params()
    rs = np.random.RandomState(seed + 100)
    for i in range(3, 14, 2):                       # non-zero biases so the bias paths are exercised
        mats[i] = (rs.normal(size=mats[i].shape) * 0.1).astype(np.float32)
    mats[14] = np.full_like(mats[14], 0.5)
    mats[15] = np.full_like(mats[15], -3.0)
    m.set_params(mats)
    return m


def data(n, seed=1, shape=SMALL):
    _, o, a, _ = shape
    rs = np.random.RandomState(seed)
    X = rs.normal(size=(n, o + a)).astype(np.float32)
    Y = np.concatenate([X[:, :1] * 0.3 + 0.1 * rs.normal(size=(n, 1)), 0.2 * X[:, :o] + 0.05 * rs.normal(size=(n, o))],
                       1).astype(np.float32)
    return X, Y


def to_oracle(mats):
    p = obnn.from_mat_list([m.astype(np.float64) for m in mats], smv=True)
    return p


def assert_trained_close(got, ref, shape_key, what=''):
    """Parameters after a whole train() loop against the fp64 oracle: rtol 1e-3 / atol 1e-4 element-wise.  At
    the shipped shape (~2 M parameters, hundreds of steps) a handful of weights whose gradient sits at the f32
    rounding level of its batch sum may take Adam steps of opposite sign (Adam moves them by ~lr = 1e-3 whatever
    the gradient's size): there at most 1 in 10^4 elements may exceed that, and none by more than 2 lr."""
    for i, (g, r) in enumerate(zip(got, ref)):
        r = np.asarray(r).reshape(g.shape)
        if shape_key == 'small':
            np.testing.assert_allclose(g, r, rtol=1e-3, atol=1e-4, err_msg='%s %d' % (what, i))
            continue
        d = np.abs(g.astype(np.float64) - r)
        bad = d > 1e-4 + 1e-3 * np.abs(r)
        assert bad.mean() <= 1e-4 and d.max() <= 2e-3, (what, i, int(bad.sum()), bad.size, d.max())


def run_epoch(m, t, X, Y, idxs, batch):
    import torch
    from mopo_amd import _lib as L
    x = torch.from_numpy(X).cuda()
    y = torch.from_numpy(Y).cuda()
    ix = torch.from_numpy(idxs.astype(np.int32)).cuda()
    L.check(L.lib().mopo_bnn_train_epoch(t, L.ptr(x), L.ptr(y), L.ptr(ix), idxs.shape[1], batch, None))
    torch.cuda.synchronize()


def setup_trainer(m, X, batch, max_eval=64):
    import torch
    from mopo_amd import _lib as L
    t = m._trainer(batch, max_eval)
    m._train_params(t, m.get_params())
    x = torch.from_numpy(X).cuda()
    L.check(L.lib().mopo_bnn_train_fit_scaler(t, L.ptr(x), X.shape[0], None))
    got = m._train_params(t)
    return t, got


# (shape, rows, batch, epochs): one k-group at H=32 (incl. a batch of 40 = 2.5 row blocks), and the shipped shape
# with full graph-replayed minibatches, a partial last minibatch, batch % 16 != 0 (250: the staged gather's last
# row block is partial) and two consecutive epochs
EPOCH_CASES = [('small', 16, 16, 1), ('small', 48, 16, 1), ('small', 40, 16, 1), ('small', 200, 16, 1),
               ('small', 200, 40, 2), ('shipped', 256, 256, 1), ('shipped', 600, 256, 2), ('shipped', 2900, 256, 1),
               ('shipped', 1000, 250, 2)]


@pytest.mark.parametrize('shape_key,n_rows,batch,epochs', EPOCH_CASES,
                         ids=['%s-%d-b%d-e%d' % c for c in EPOCH_CASES])
def test_epoch_matches_oracle_steps(shape_key, n_rows, batch, epochs):
    shape = SHAPES[shape_key]
    e_ = shape[0]
    m = model(shape=shape)
    X, Y = data(n_rows, shape=shape)
    t, start = setup_trainer(m, X, batch)
    np.testing.assert_allclose(start[0], X.mean(0, keepdims=True), rtol=1e-5, atol=1e-6)   # scaler.fit
    np.testing.assert_allclose(start[1], X.std(0, keepdims=True), rtol=1e-5, atol=1e-6)
    rs = np.random.RandomState(7)
    st = ot.TrainState(to_oracle(start))
    nb = int(np.ceil(n_rows / batch))
    steps = 0
    for ep in range(epochs):
        idxs = rs.randint(n_rows, size=[e_, n_rows])
        run_epoch(m, t, X, Y, idxs, batch)
        for b in range(nb):
            bi = idxs[:, b * batch:(b + 1) * batch]
            st.step(X[bi].astype(np.float64), Y[bi].astype(np.float64))
            steps += 1
    got = m._train_params(t)
    ref = ot.optvars(st.params())
    ref = [st.vals[i] for i in range(len(ref))]
    names = ['W0', 'b0', 'W1', 'b1', 'W2', 'b2', 'W3', 'b3', 'Wm', 'bm', 'Wv', 'bv', 'maxlv', 'minlv']
    step1 = 1e-3   # Adam's first step: lr_t * m / sqrt(v) = lr * sign(g)
    if steps == 1:
        _, g_ref = ot.loss_and_grads(to_oracle(start), X[idxs].astype(np.float64), Y[idxs].astype(np.float64))
    for k, (g, r) in enumerate(zip(got[2:], ref)):
        r = r.reshape(g.shape)
        if steps == 1:   # a vanishing gradient may flip sign: Adam's first step then differs by 2 lr_t
            gr = np.abs(g_ref[k]).reshape(g.shape)
            tol = 1e-6 + 2.2 * step1 * (gr <= 1e-5 * gr.max())
            assert np.all(np.abs(g - r) <= tol), names[k]
        else:
            np.testing.assert_allclose(g, r, rtol=2e-5, atol=2e-5 * max(1.0, np.abs(r).max()), err_msg=names[k])


def test_one_step_is_close_to_lr_scale():
    """Adam's first step moves every variable by lr_t m / sqrt(v) = lr (1e-3) times sign(g)."""
    m = model()
    X, Y = data(16)
    t, start = setup_trainer(m, X, 16)
    idxs = np.random.RandomState(3).randint(16, size=[E, 16])
    run_epoch(m, t, X, Y, idxs, 16)
    got = m._train_params(t)
    d = np.concatenate([np.abs(g - s).ravel() for g, s in zip(got[2:], start[2:])])
    assert d.max() <= 1e-3 * 1.0001 and np.median(d) > 0.9e-3


def test_eval_mse_matches_oracle():
    import torch
    from mopo_amd import _lib as L
    m = model(3)
    X, Y = data(50, seed=4)
    t, start = setup_trainer(m, X, 16, max_eval=64)
    out = torch.empty(E, dtype=torch.float32, device='cuda')
    x, y = torch.from_numpy(X).cuda(), torch.from_numpy(Y).cuda()
    L.check(L.lib().mopo_bnn_train_eval_mse(t, L.ptr(x), L.ptr(y), None, 50, L.ptr(out), None))
    ref = ot.mse_losses(to_oracle(start), np.tile(X[None], [E, 1, 1]), np.tile(Y[None], [E, 1, 1]))
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-5)


@pytest.mark.parametrize('side', [False, True])
def test_shuffle_rows_is_numpy_argsort_order(side):
    """side: the order computed on a second stream (mopo_bnn_train_shuffle_async), three shuffles in a
    row so each order waits for the previous apply."""
    import torch
    from mopo_amd import _lib as L
    m = model()
    t = m._trainer(16, 64)
    rs = np.random.RandomState(5)
    n = 1000
    idxs = rs.randint(n, size=[E, n]).astype(np.int32)
    d_idx = torch.from_numpy(idxs.copy()).cuda()
    ref = idxs
    st = torch.cuda.Stream()
    for _ in range(3 if side else 1):
        keys = rs.uniform(size=[E, n])
        d_keys = torch.from_numpy(keys).cuda()
        torch.cuda.synchronize()
        if side:
            L.check(L.lib().mopo_bnn_train_shuffle_async(t, L.ptr(d_idx), L.ptr(d_keys), n, L.stream_ptr(st), None))
        else:
            L.check(L.lib().mopo_bnn_train_shuffle(t, L.ptr(d_idx), L.ptr(d_keys), n, None))
        ref = ref[np.arange(E)[:, None], np.argsort(keys, axis=-1)]               # bnn.py:385-387
    np.testing.assert_array_equal(d_idx.cpu().numpy(), ref)


def test_format_samples_matches_constructor():
    import torch
    from mopo_amd import _lib as L
    from mopo_amd.replay_pool import SimpleReplayPool
    rs = np.random.RandomState(6)
    n = 300
    s = {'observations': rs.normal(size=(n, O)).astype(np.float32),
         'actions': rs.normal(size=(n, A)).astype(np.float32),
         'next_observations': rs.normal(size=(n, O)).astype(np.float32),
         'rewards': rs.normal(size=(n, 1)).astype(np.float32), 'terminals': np.zeros((n, 1), bool)}
    pool = SimpleReplayPool(obs_dim=O, act_dim=A, max_size=n)
    pool.add_samples(s)
    rows = rs.permutation(n)
    x = torch.empty((n, IN), dtype=torch.float32, device='cuda')
    y = torch.empty((n, D), dtype=torch.float32, device='cuda')
    L.check(L.lib().mopo_bnn_format_samples(C.byref(pool.desc()), O, A, L.ptr(torch.from_numpy(rows).cuda()), n,
                                            L.ptr(x), L.ptr(y), None))
    ref_x = np.concatenate([s['observations'], s['actions']], 1)[rows]               # constructor.py:46-57
    ref_y = np.concatenate([s['rewards'], s['next_observations'] - s['observations']], 1)[rows]
    np.testing.assert_array_equal(x.cpu().numpy(), ref_x)
    np.testing.assert_array_equal(y.cpu().numpy(), ref_y)


# (shape, rows, batch, max_epochs, max_epochs_since_update); the shipped case: 2,400 training rows = 9 full
# minibatches of 256 (graph-replayed, staged gather) + a partial one of 96 per epoch
LOOP_CASES = [('small', 300, 32, 12, 3), ('shipped', 3000, 256, 40, 3)]


@pytest.mark.parametrize('shape_key,n_rows,batch,max_epochs,since', LOOP_CASES, ids=[c[0] for c in LOOP_CASES])
def test_train_loop_matches_oracle(shape_key, n_rows, batch, max_epochs, since):
    """BNN.train (bnn.py:369-503) end to end with the reference's RNG order on numpy's global stream."""
    shape = SHAPES[shape_key]
    m = model(5, shape=shape)
    X, Y = data(n_rows, seed=8, shape=shape)
    mats0 = m.get_params()
    np.random.seed(11)
    out = m.train(X, Y, batch_size=batch, max_epochs=max_epochs, holdout_ratio=0.2, max_epochs_since_update=since)
    np.random.seed(11)
    p0 = to_oracle(mats0)
    q, elites, hl, epochs, updates = ot.train(p0, X, Y, num_elites=2, batch_size=batch, max_epochs=max_epochs,
                                              holdout_ratio=0.2, max_epochs_since_update=since)
    assert m._train_epochs == epochs and m._train_grad_updates == updates
    np.testing.assert_allclose(m._holdout_losses, hl, rtol=1e-3)
    assert m._model_inds == elites
    assert out['val_loss'] == pytest.approx(np.sort(hl)[:2].mean(), rel=1e-3)
    got = m.get_params()
    assert_trained_close(got, obnn.to_mat_list(q), shape_key)
    # the trained ensemble predicts with the published parameters
    mean, var = m.predict(X[:20])
    rm, rv = obnn.forward(obnn.from_mat_list(got, smv=True), X[:20])
    np.testing.assert_allclose(mean, rm, rtol=1e-4, atol=1e-5)


JOINT_CASES = [('small', 300, 32, 10), ('shipped', 3000, 256, 30)]


@pytest.mark.parametrize('shape_key,n_rows,batch,max_epochs', JOINT_CASES, ids=[c[0] for c in JOINT_CASES])
def test_train_loop_joint_head_matches_oracle(shape_key, n_rows, batch, max_epochs):
    """separate_mean_var=False: the joint [H, 2D] head trains through the smv trainer on its column
    halves (same 0.0001 decay, constructor.py:34-36); the oracle trains the joint head directly
    (bnn.py:644-654, pinned by tests/golden/ref_bnn_loss_E3_H32_joint.npz)."""
    from mopo_amd.bnn import construct_model
    shape = SHAPES[shape_key]
    e_, o_, a_, h_ = shape
    d_ = o_ + 1
    m = construct_model(obs_dim=o_, act_dim=a_, hidden_dim=h_, num_networks=e_, num_elites=2, separate_mean_var=False,
                        seed=9)
    mats = m.get_params()
    assert len(mats) == 14 and mats[10].shape == (e_, h_, 2 * d_)
    rs = np.random.RandomState(109)
    for i in range(3, 12, 2):
        mats[i] = (rs.normal(size=mats[i].shape) * 0.1).astype(np.float32)
    mats[12] = np.full_like(mats[12], 0.5)
    mats[13] = np.full_like(mats[13], -3.0)
    m.set_params(mats)
    X, Y = data(n_rows, seed=10, shape=shape)
    np.random.seed(12)
    out = m.train(X, Y, batch_size=batch, max_epochs=max_epochs, holdout_ratio=0.2, max_epochs_since_update=3)
    np.random.seed(12)
    p0 = obnn.from_mat_list([x.astype(np.float64) for x in mats], smv=False)
    q, elites, hl, epochs, updates = ot.train(p0, X, Y, num_elites=2, batch_size=batch, max_epochs=max_epochs,
                                              holdout_ratio=0.2, max_epochs_since_update=3)
    assert m._train_epochs == epochs and m._train_grad_updates == updates
    np.testing.assert_allclose(m._holdout_losses, hl, rtol=1e-3)
    assert m._model_inds == elites
    assert out['val_loss'] == pytest.approx(np.sort(hl)[:2].mean(), rel=1e-3)
    got = m.get_params()
    assert len(got) == 14
    assert_trained_close(got, obnn.to_mat_list(q), shape_key, 'joint')
    mean, var = m.predict(X[:20])
    rm, rv = obnn.forward(obnn.from_mat_list(got, smv=False), X[:20])
    np.testing.assert_allclose(mean, rm, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(var, rv, rtol=1e-4, atol=1e-6)


KNOBS = ['MOPO_TRAIN_WG2=1,MOPO_TRAIN_WG2_NT=512', 'MOPO_TRAIN_WG2=1,MOPO_TRAIN_WG2_NT=1024',
         'MOPO_TRAIN_WG2=1,MOPO_TRAIN_WG2_NT=256', 'MOPO_TRAIN_STAGE=0', 'MOPO_TRAIN_WG2=0',
         'MOPO_TRAIN_SHUFFLE_SIDE=0,MOPO_TRAIN_NUMPY_DRAWS=1']


@pytest.mark.parametrize('shape_key', ['small', 'shipped'])
@pytest.mark.parametrize('knobs', KNOBS)
def test_wgrad_launch_variants_match_oracle(knobs, shape_key):
    """The weight-gradient launch knobs (MOPO_TRAIN_WG2: the persistent XCD-local tile launch or the
    grouped-GEMM launch; MOPO_TRAIN_WG2_NT: 256-, 512- or 1024-thread tile workgroups;
    MOPO_TRAIN_STAGE=0: every row block gathers its own minibatch rows)
    are read once per process, so each setting runs the epoch and train-loop parity tests above in a
    fresh process, at one shape (the shipped one dispatches train_rows_kernel<2,13,3> and the H=200 tiles)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, **dict(kv.split('=') for kv in knobs.split(',')))
    r = subprocess.run([sys.executable, '-m', 'pytest', '-p', 'no:cacheprovider', '-q', '-x', '-m', 'gpu',
                        os.path.join(root, 'tests', 'test_gpu_train.py'),
                        '-k', '(epoch_matches_oracle_steps or train_loop_matches_oracle) and %s' % shape_key],
                       cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert ' passed' in r.stdout and 'skipped' not in r.stdout.splitlines()[-1], r.stdout[-500:]
