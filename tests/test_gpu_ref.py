"""GPU parity against vectors made by executing the reference's own graph code (the f32 runs of
tests/golden/make_ref_vectors.py: mopo/models/{fc,bnn,utils}.py and mopo/algorithms/mopo.py under a
torch-backed TF stand-in).  These pin the device path to the reference itself, not to the
restatement.

Tolerances (|d| <= tol * (1 + |ref|) unless stated):
  * ensemble mean / log-var, fp32, bf16x6 and f16x3 (~22-bit splits): 2e-5;  var rel 5e-5
  * ensemble, bf16x3 (~17 significand bits):                            2e-3
  * ensemble, bf16 (8 bits, reported separately):          3e-2 relative scale
  * actor pi / mu (tanh outputs):                                       2e-5 absolute
  * SAC logged fetches (losses, q means, alpha, logp, entropy, norms):  rel 2e-4
  * SAC parameters after each Adam step:                                1e-6 + 2 lr_t where the
    reference gradient is tiny (Adam's first steps are ~lr_t sign(g)), else 1e-6 (+1e-6 rel)
"""
import glob
import os

import numpy as np
import pytest

from test_oracle_ref import ref_bnn_params

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), 'golden')
FWD = sorted(glob.glob(os.path.join(GOLD, 'ref_bnn_fwd_*.npz')))
SAC = sorted(glob.glob(os.path.join(GOLD, 'ref_sac_*.npz')))
TOL = {'fp32': 2e-5, 'bf16x6': 2e-5, 'f16x3': 2e-5, 'bf16x3': 2e-3, 'bf16': 3e-2}


def close(a, b, tol, what=''):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    err = np.abs(a - b) / (1 + np.abs(b))
    assert err.max(initial=0) <= tol, '%s: max scaled err %.3g > %.3g' % (what, err.max(), tol)


@pytest.mark.parametrize('dtype', ['fp32', 'bf16x6', 'f16x3', 'bf16x3', 'bf16'])
@pytest.mark.parametrize('path', FWD, ids=[os.path.basename(p)[12:-4] for p in FWD])
def test_bnn_predict_vs_reference_graph(path, dtype):
    """BNN.predict (bnn.py:508-546) vs the reference's _compile_outputs executed in f32."""
    from oracle import bnn as obnn
    from mopo_amd.bnn import BNN
    z = dict(np.load(path))
    E, H, smv = int(z['E']), int(z['H']), bool(z['smv'])
    p = ref_bnn_params(z)
    if dtype == 'bf16x6' and H > 256:   # refused at construction (mopo_bnn_create): f16x3 covers H = 400
        with pytest.raises(RuntimeError, match='bf16x6'):
            BNN({'name': 'ref', 'num_networks': E, 'num_elites': min(5, E), 'separate_mean_var': smv, 'obs_dim': 17,
                 'act_dim': 6, 'hidden_dim': H, 'dtype': dtype})
        return
    m = BNN({'name': 'ref', 'num_networks': E, 'num_elites': min(5, E), 'separate_mean_var': smv, 'obs_dim': 17,
             'act_dim': 6, 'hidden_dim': H, 'dtype': dtype}).set_params(obnn.to_mat_list(p))
    mean, var = m.predict(z['x'], factored=True)
    tol = TOL[dtype]
    close(mean, z['mean_f32'], tol, 'mean')
    close(np.log(var), z['logvar_f32'], tol, 'log-var')
    if dtype in ('fp32', 'bf16x6', 'f16x3'):
        assert np.max(np.abs(var - z['var_f32']) / z['var_f32']) < 5e-5


def _sac_for_case(z):
    from mopo_amd.sac import SAC
    O, A, H, n = int(z['O']), int(z['A']), int(z['H']), int(z['n'])
    init = np.concatenate([z['init%d' % i].ravel() for i in range(20)]).astype(np.float32)
    return SAC(O, A, H, batch_size=n, real_ratio=0.05, target_entropy=-3, params=init, log_alpha=0.0)


def _pools_for_batch(b, n_env, O, A):
    """The reference batch as an env pool (its first n_env rows) + a model pool (the rest), drawn
    back by the device step through idx = [0..n_env) ++ [0..n - n_env) (mopo.py:801-816 order)."""
    import torch
    from mopo_amd.replay_pool import SimpleReplayPool
    n = b['observations'].shape[0]
    pools = []
    for lo, hi in ((0, n_env), (n_env, n)):
        p = SimpleReplayPool(obs_dim=O, act_dim=A, max_size=max(hi - lo, 1))
        p.add_samples({k: v[lo:hi] for k, v in b.items()})
        pools.append(p)
    torch.cuda.synchronize()
    idx = np.concatenate([np.arange(n_env), np.arange(n - n_env)]).astype(np.int64)
    return pools, idx


@pytest.mark.parametrize('path', SAC, ids=[os.path.basename(p)[8:-4] for p in SAC])
def test_sac_steps_vs_reference_graph(path):
    """MOPO._do_training + _update_target (mopo.py:834-853) for consecutive steps, injected batch and
    policy noise (the 1st and 3rd tf.random_normal draws of _build: main(s) and main(s'))."""
    z = dict(np.load(path))
    O, A, n, steps = int(z['O']), int(z['A']), int(z['n']), int(z['steps'])
    sac = _sac_for_case(z)
    lr_t = [3e-4 * np.sqrt(1 - 0.999 ** (k + 1)) / (1 - 0.9 ** (k + 1)) for k in range(steps)]
    for k in range(steps):
        b = {kk: z['b%d_%s' % (k, kk)] for kk in ('observations', 'actions', 'next_observations', 'rewards',
                                                   'terminals')}
        (env_p, mod_p), idx = _pools_for_batch(b, sac.n_env, O, A)
        sac._do_training(k, env_p, mod_p, idx=idx, eps_s=z['b%d_noise0' % k][0], eps_n=z['b%d_noise2' % k][0])
        lg = sac.logs()
        for key in ('Q/q1_loss', 'sac_Q/q2_loss', 'sac_Q/q1', 'sac_Q/q2', 'sac_pi/alpha', 'sac_pi/logp_pi',
                    'sac_pi/pi_entropy', 'sac_pi/std', 'sac_pi/pi_global_norm', 'sac_Q/q_global_norm'):
            ref = float(z['b%d_log_%s_f32' % (k, key.replace('/', '.'))])
            assert abs(lg[key] - ref) <= 2e-4 * abs(ref) + 1e-6, (k, key, lg[key], ref)
        p_new, la = sac.get_params()
        p_new = p_new.cpu().numpy()
        p_ref = np.concatenate([z['b%d_post%d_f32' % (k, i)].ravel() for i in range(20)])
        d = np.abs(p_new - p_ref)
        if 'b%d_grad_pi0_f32' % k in z:
            gr = np.concatenate([z['b%d_grad_%s%d_f32' % (k, g, j)].ravel() for g, nj in (('pi', 8), ('q1', 6), ('q2', 6))
                                 for j in range(nj)])
            tiny = np.abs(gr) < 1e-3 * np.abs(gr).max()
            assert d[~tiny].max() <= 1e-6 + 1e-6 * np.abs(p_ref).max(), d[~tiny].max()
            # a small gradient moves its parameter by ~lr_t m/sqrt(v) whatever its size, so the device's
            # gradient error (<= 1e-4 max|g| of the tensor, tests/test_gpu_sac.py) moves the update by
            # ~lr_t err/|g|: a sign may flip only where |g| is at that error level, elsewhere the allowance
            # shrinks with |g| (it was a flat 2 sum(lr_t) for every small gradient)
            allow = 1e-6 + 1e-6 * np.abs(p_ref).max() + 2 * sum(lr_t[:k + 1]) * np.minimum(
                1.0, 1e-4 * np.abs(gr).max() / np.maximum(np.abs(gr), 1e-30))
            bad = tiny & (d > allow)
            assert not bad.any(), (int(bad.sum()), d[bad].max(), np.abs(gr[bad]).max() / np.abs(gr).max())
        else:
            assert d.max() <= 1e-6 + 2 * sum(lr_t[:k + 1])
        assert abs(float(la.item()) - float(z['b%d_log_alpha_f32' % k])) < 1e-6
        if 'b%d_target0_f32' % k in z:
            tgt = sac.get_target().cpu().numpy()
            t_ref = np.concatenate([z['b%d_target%d_f32' % (k, i)].ravel() for i in range(20)])
            assert np.abs(tgt - t_ref).max() <= 2e-6 + 5e-3 * 2 * sum(lr_t[:k + 1])


@pytest.mark.parametrize('dtype', [0, 3, 4])   # fp32, bf16x6, f16x3
@pytest.mark.parametrize('path', SAC, ids=[os.path.basename(p)[8:-4] for p in SAC])
def test_actor_vs_reference_graph(path, dtype):
    """get_action_meta (mopo.py:468-485): pi and the deterministic mu for the step-0 batch."""
    import torch
    from mopo_amd import _lib as L
    z = dict(np.load(path))
    O, A, H, n = int(z['O']), int(z['A']), int(z['H']), int(z['n'])
    flat = np.concatenate([z['init%d' % i].ravel() for i in range(20)]).astype(np.float32)
    dev = torch.device('cuda')
    tp = torch.from_numpy(flat).to(dev)
    to = torch.from_numpy(z['b0_observations']).to(dev)
    te = torch.from_numpy(np.ascontiguousarray(z['b0_noise0'][0])).to(dev)
    act = torch.empty((n, A), device=dev)
    mu = torch.empty((n, A), device=dev)
    L.check(L.lib().mopo_actor_forward_dtype(L.ptr(tp), O, A, H, L.ptr(to), 0, n, L.ptr(te), 0, 0, L.ptr(act),
                                             L.ptr(mu), dtype, L.stream_ptr()))
    assert np.abs(act.cpu().numpy() - z['actor_pi_f32']).max() < 2e-5
    assert np.abs(mu.cpu().numpy() - z['actor_mu_f32']).max() < 2e-5


def test_softlearning_sac_api_vs_reference_graph():
    """softlearning/algorithms/sac.py:26-47's constructor form (environment spaces, policy / Qs, pool) and
    _do_training(iteration, batch) with a batch dict: step 0 of the reference-executed H=256 case."""
    import types
    from mopo_amd.sac import SAC
    z = dict(np.load(os.path.join(GOLD, 'ref_sac_H256.npz')))
    O, A, H, n = int(z['O']), int(z['A']), int(z['H']), int(z['n'])
    env = types.SimpleNamespace(observation_space=types.SimpleNamespace(shape=(O,)),
                                action_space=types.SimpleNamespace(shape=(A,)))
    policy = types.SimpleNamespace(hidden_layer_sizes=(H, H))
    init = np.concatenate([z['init%d' % i].ravel() for i in range(20)]).astype(np.float32)
    sac = SAC(env, env, policy, (policy, policy), None, lr=3e-4, target_entropy=-3, reparameterize=True,
              real_ratio=0.05, params=init)
    assert (sac.obs_dim, sac.act_dim, sac.hidden, sac.n_env) == (O, A, H, 12)
    b = {k: z['b0_%s' % k] for k in ('observations', 'actions', 'next_observations', 'rewards', 'terminals')}
    lg = sac._do_training(0, b, eps_s=z['b0_noise0'][0], eps_n=z['b0_noise2'][0])
    for key in ('Q/q1_loss', 'sac_Q/q2_loss', 'sac_pi/alpha', 'sac_pi/logp_pi', 'sac_Q/q_global_norm'):
        ref = float(z['b0_log_%s_f32' % key.replace('/', '.')])
        assert abs(lg[key] - ref) <= 2e-4 * abs(ref) + 1e-6, (key, lg[key], ref)
    with pytest.raises(NotImplementedError):
        SAC(env, env, policy, (policy,), None, reparameterize=False)


QUANTILES = (0.5, 0.9, 0.99, 1.0)


# bf16x6 has no H > 256 form (refused at mopo_bnn_create; the product default there is fp32)
SPLIT_CASES = [(p, d) for d in ('bf16x6', 'f16x3') for p in FWD if not (d == 'bf16x6' and '_H400' in p)]


@pytest.mark.parametrize('path,dtype', SPLIT_CASES, ids=['%s-%s' % (os.path.basename(p)[12:-4], d) for p, d in SPLIT_CASES])
def test_split_error_distribution_is_fp32_class(path, dtype):
    """The split dtypes -- bf16x6 (the product default: exact f32 operands, 6 bf16 products; H <= 256) and
    f16x3 (~22-bit operands) -- against the reference's own graph executed in f64:
    (1) an ABSOLUTE fp32 bound, |d| <= 2e-5 * (1 + |ref|) on mean and log-var, and (2) its error
    DISTRIBUTION (quantiles 50 / 90 / 99 / 100 % of |d| / (1 + |ref|)) no wider than 2x the wider of
    the exact-f32 MFMA kernel's and the reference's own f32 execution's (TF1's f32 rounding,
    z['*_f32'] vs z['*_f64']), with a floor of 2 f32 ulps (2^-23) for quantiles where both are ~0."""
    from oracle import bnn as obnn
    from mopo_amd.bnn import BNN
    z = dict(np.load(path))
    E, H, smv = int(z['E']), int(z['H']), bool(z['smv'])
    mats = obnn.to_mat_list(ref_bnn_params(z))

    def run(dtype):
        m = BNN({'name': 'ref', 'num_networks': E, 'num_elites': min(5, E), 'separate_mean_var': smv,
                 'obs_dim': 17, 'act_dim': 6, 'hidden_dim': H, 'dtype': dtype}).set_params(mats)
        mean, var = m.predict(z['x'], factored=True)
        return mean, np.log(var)

    def q(a, ref):
        e = np.abs(np.asarray(a, np.float64) - ref) / (1 + np.abs(ref))
        return np.quantile(e.ravel(), QUANTILES)

    got, f32 = run(dtype), run('fp32')
    tf32 = (z['mean_f32'], z['logvar_f32'])
    for i, key in enumerate(('mean_f64', 'logvar_f64')):
        ref = z[key]
        e16, e32, etf = q(got[i], ref), q(f32[i], ref), q(tf32[i], ref)
        assert e16[-1] <= 2e-5, (key, e16)
        bound = np.maximum(2 * np.maximum(e32, etf), 2.0 ** -23)
        assert np.all(e16 <= bound), (key, dtype, e16, 'fp32 kernel', e32, 'TF f32', etf)
