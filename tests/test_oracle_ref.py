"""CPU: pin the oracle's TF-only restatements (ensemble forward, ensemble training loss, actor, SAC
step) to vectors made by executing the reference's own graph code (tests/golden/make_ref_vectors.py:
mopo/models/{fc,bnn,utils}.py and mopo/algorithms/mopo.py run under a torch-backed TF stand-in).

Each reference case was executed twice: in f32 (the reference graph's dtype) and f64.  The f64
oracle must match the f64 execution to rounding (1e-10 relative) -- that pins the restatement's
algebra; the f32 execution is what the GPU tests compare the device against (test_gpu_ref.py).
"""
import glob
import os

import numpy as np
import pytest

from oracle import bnn as obnn
from oracle import bnn_train as obt
from oracle import sac as osac

GOLD = os.path.join(os.path.dirname(__file__), 'golden')
FWD = sorted(glob.glob(os.path.join(GOLD, 'ref_bnn_fwd_*.npz')))
SAC = sorted(glob.glob(os.path.join(GOLD, 'ref_sac_*.npz')))
SAC_KEYS = ('Q/q1_loss', 'sac_Q/q2_loss', 'sac_Q/q1', 'sac_Q/q2', 'sac_pi/alpha', 'sac_pi/logp_pi',
            'sac_pi/pi_entropy', 'sac_pi/std', 'sac_pi/pi_global_norm', 'sac_Q/q_global_norm')


def rel(a, b):
    return float(np.max(np.abs(np.asarray(a, np.float64) - b) / (1e-30 + np.abs(b)))) if np.size(b) else 0.0


def scaled(a, b):
    return float(np.max(np.abs(np.asarray(a, np.float64) - b) / (1 + np.abs(b))))


def ref_bnn_params(z):
    """Weights of a forward case: stored, or regenerated from the seed and checked by sha256."""
    E, H, smv, seed = int(z['E']), int(z['H']), bool(z['smv']), int(z['seed'])
    if 'w0' in z:
        n = 16 if smv else 14
        return obnn.from_mat_list([z['w%d' % i] for i in range(n)], smv=smv)
    import hashlib
    rs = np.random.RandomState(seed + 100)
    fit = rs.normal(size=(400, 23)) * 1.5 + 0.2
    p = obnn.init_params(E, 17, 6, hidden=H, seed=seed, smv=smv, inputs=fit)
    h = hashlib.sha256()
    for a in obnn.to_mat_list(p):
        h.update(np.ascontiguousarray(a, np.float32).tobytes())
    assert h.hexdigest() == str(z['weights_sha']), 'regenerated weights differ from the reference case'
    return p


def test_ref_fixture_count():
    assert len(FWD) >= 5 and len(SAC) >= 2


@pytest.mark.parametrize('path', FWD, ids=[os.path.basename(p) for p in FWD])
def test_bnn_forward_oracle_vs_reference_graph(path):
    z = dict(np.load(path))
    p = ref_bnn_params(z)
    m64, v64 = obnn.forward(p, z['x'], dtype=np.float64)
    assert rel(m64, z['mean_f64']) < 1e-10 or scaled(m64, z['mean_f64']) < 1e-13
    assert rel(v64, z['var_f64']) < 1e-10
    _, lv64 = obnn.forward(p, z['x'], dtype=np.float64, ret_log_var=True)
    assert scaled(lv64, z['logvar_f64']) < 1e-13
    # the reference graph in f32 vs the f64 restatement: the fp32 tolerance of the GPU tests
    assert scaled(m64, z['mean_f32']) < 2e-6
    assert rel(v64, z['var_f32']) < 2e-6


def test_bnn_train_loss_oracle_vs_reference_graph():
    z = dict(np.load(os.path.join(GOLD, 'ref_bnn_loss_E3_H32.npz')))
    p = obnn.from_mat_list([z['w%d' % i] for i in range(16)])
    loss, grads = obt.loss_and_grads(p, z['X'], z['Y'])
    assert rel(loss, z['loss_f64']) < 1e-12
    for i, g in enumerate(grads):   # optvars order: mean layers (W, b) x5, var layer W, b, maxlv, minlv
        ref = z['grad%d_f64' % i]
        assert np.max(np.abs(g - ref)) <= 1e-12 * max(1.0, np.max(np.abs(ref))), i
    np.testing.assert_allclose(obt.mse_losses(p, z['X'], z['Y']), z['mse_f64'], rtol=1e-12)


def test_bnn_train_loss_joint_head_vs_reference_graph():
    """The joint head (separate_mean_var=False, bnn.py:183-189 / 644-654) through the reference's
    _compile_losses + decays: 14 .mat arrays, one [H, 2D] head with one decay."""
    z = dict(np.load(os.path.join(GOLD, 'ref_bnn_loss_E3_H32_joint.npz')))
    assert int(z['smv']) == 0
    p = obnn.from_mat_list([z['w%d' % i] for i in range(14)], smv=False)
    loss, grads = obt.loss_and_grads(p, z['X'], z['Y'])
    assert rel(loss, z['loss_f64']) < 1e-12
    assert len(grads) == 12
    for i, g in enumerate(grads):   # optvars: layers (W, b) x5 (head [H, 2D]), maxlv, minlv
        ref = z['grad%d_f64' % i]
        assert np.max(np.abs(g - ref)) <= 1e-12 * max(1.0, np.max(np.abs(ref))), i
    np.testing.assert_allclose(obt.mse_losses(p, z['X'], z['Y']), z['mse_f64'], rtol=1e-12)


def _sac_batch(z, k):
    return {kk: z['b%d_%s' % (k, kk)] for kk in ('observations', 'actions', 'next_observations', 'rewards',
                                                  'terminals')}


@pytest.mark.parametrize('path', SAC, ids=[os.path.basename(p) for p in SAC])
def test_sac_oracle_vs_reference_graph(path):
    """MOPO._build / _do_training / _update_target executed from the reference, several steps."""
    z = dict(np.load(path))
    steps = int(z['steps'])
    st = osac.SACState([z['init%d' % i].astype(np.float64) for i in range(20)])
    for k in range(steps):
        g = {}
        # only the 1st (main(s)) and 3rd (main(s')) tf.random_normal draws reach the results
        logs = osac.sac_step(st, _sac_batch(z, k), z['b%d_noise0' % k][0].astype(np.float64),
                             z['b%d_noise2' % k][0].astype(np.float64), grads_out=g)
        for key in SAC_KEYS:
            ref = z['b%d_log_%s_f64' % (k, key.replace('/', '.'))]
            assert abs(logs[key] - ref) <= 1e-9 * max(1.0, abs(ref)), (k, key, logs[key], ref)
        if 'b%d_grad_pi0_f64' % k in z:
            for grp in ('pi', 'q1', 'q2'):
                for j, gg in enumerate(g[grp]):
                    ref = z['b%d_grad_%s%d_f64' % (k, grp, j)]
                    assert np.max(np.abs(gg - ref)) <= 1e-9 * max(1e-3, np.max(np.abs(ref))), (k, grp, j)
            assert abs(g['alpha'] - z['b%d_grad_alpha0_f64' % k]) < 1e-9
        if 'b%d_post0_f64' % k in z:
            for i in range(20):
                np.testing.assert_allclose(st.params[i], z['b%d_post%d_f64' % (k, i)], rtol=0, atol=1e-11)
        if 'b%d_target0_f64' % k in z:
            for i in range(20):
                np.testing.assert_allclose(st.target[i], z['b%d_target%d_f64' % (k, i)], rtol=0, atol=1e-11)
        assert abs(st.log_alpha - z['b%d_log_alpha_f64' % k]) < 1e-12


def test_sac_polyak_pairing_from_reference_graph():
    """zip(get_vars('main'), get_vars('target')) (mopo.py:446-447) pairs each target with its own
    main variable, the Adam slots excluded by truncation: the recorded assigns are exactly
    target <- 0.995 target + 0.005 main, in creation order."""
    z = dict(np.load(SAC[0]))
    pairs = [str(p) for p in z['polyak_pairs']]
    assert len(pairs) == 40
    for i in range(20):
        a, b = pairs[2 * i], pairs[2 * i + 1]
        ref_a, rest_a = a.split('<-')
        assert ref_a.startswith('target/')
        srcs = {rest_a.rsplit(':', 1)[0]: float(rest_a.rsplit(':', 1)[1])}
        ref_b, rest_b = b.split('<-')
        assert ref_b == ref_a
        srcs[rest_b.rsplit(':', 1)[0]] = float(rest_b.rsplit(':', 1)[1])
        assert srcs == {ref_a.replace('target/', 'main/', 1): 0.005, ref_a: 0.995}, srcs


def test_actor_oracle_vs_reference_graph():
    """get_action_meta (mopo.py:468-485) on the step-0 batch with the first tf.random_normal draw."""
    for path in SAC:
        z = dict(np.load(path))
        P = osac.split([z['init%d' % i].astype(np.float64) for i in range(20)])[0]
        a, mu = osac.actor_act(P, z['b0_observations'].astype(np.float64), z['b0_noise0'][0].astype(np.float64))
        np.testing.assert_allclose(a, z['actor_pi_f64'], rtol=0, atol=1e-12)
        np.testing.assert_allclose(mu, z['actor_mu_f64'], rtol=0, atol=1e-12)
        assert np.max(np.abs(a - z['actor_pi_f32'])) < 1e-6
