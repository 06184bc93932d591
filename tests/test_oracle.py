"""CPU: pin the oracle against golden vectors executed from the reference (tests/golden)."""
import glob
import os

import numpy as np
import pytest

from oracle import bnn as obnn
from oracle import fake_env as ofe
from oracle import replay_pool as opool
from oracle import sac as osac

GOLD = os.path.join(os.path.dirname(__file__), 'golden')
CASES = sorted(glob.glob(os.path.join(GOLD, 'fakeenv_*.npz')))


def load_params(E, H):
    z = np.load(os.path.join(GOLD, 'bnn_E%d_H%d.npz' % (E, H)))
    return obnn.from_mat_list([z['w%d' % i] for i in range(16)], smv=True)


def test_fixture_count():
    assert len(CASES) >= 40


@pytest.mark.parametrize('path', CASES, ids=[os.path.basename(c) for c in CASES])
def test_fakeenv_oracle_vs_reference(path):
    """Fixtures: the reference's FakeEnv.step driven by the reference graph's own f32 forward
    (make_golden.py).  Where the fixture stores that forward's mean/var (B <= 64) the oracle's
    post-processing is fed the same arrays and must be bit-identical; the oracle's own forward is
    then within f32 rounding of the reference graph's."""
    c = dict(np.load(path))
    E, H, B = int(c['E']), int(c['H']), int(c['B'])
    params = load_params(E, H)
    det = bool(c['deterministic'])
    term_fn = ofe.TERMINATION[str(c['domain'])]
    kw = dict(penalty_coeff=float(c['penalty_coeff']), penalty_learned_var=bool(c['learned_var']),
              deterministic=det)
    inputs = np.concatenate((c['obs'], c['act']), axis=-1)
    if 'ref_mean' in c:
        np.random.seed(int(c['seed']))
        nobs, rew, term, info = ofe.step(params, list(c['elites']), c['obs'], c['act'], term_fn,
                                         predicted=(c['ref_mean'], c['ref_var']), **kw)
        if not det:  # same RNG order -> identical integer choices
            np.testing.assert_array_equal(info['model_inds'], c['model_inds'])
        for got, key in ((nobs, 'next_obs'), (rew, 'rew'), (term, 'term'), (info['penalty'], 'penalty'),
                         (info['mean'], 'info_mean'), (info['std'], 'info_std'), (info['log_prob'], 'log_prob'),
                         (info['dev'], 'dev')):
            np.testing.assert_array_equal(got, c[key], err_msg=key)
        m, v = obnn.forward(params, inputs)
        assert np.max(np.abs(m - c['ref_mean']) / (1 + np.abs(c['ref_mean']))) < 2e-6
        assert np.max(np.abs(v - c['ref_var']) / np.abs(c['ref_var'])) < 2e-6
    np.random.seed(int(c['seed']))
    nobs, rew, term, info = ofe.step(params, list(c['elites']), c['obs'], c['act'], term_fn, **kw)
    if not det:
        np.testing.assert_array_equal(info['model_inds'], c['model_inds'])
    for got, key in ((nobs, 'next_obs'), (rew, 'rew'), (info['mean'], 'info_mean'), (info['std'], 'info_std')):
        assert np.max(np.abs(got - c[key]) / (1 + np.abs(c[key]))) < 5e-6, key
    if info['penalty'] is not None:
        assert np.max(np.abs(info['penalty'] - c['penalty']) / np.abs(c['penalty'])) < 5e-6
    bad = term[:, 0] != c['term'][:, 0]     # only where f32 rounding moves next_obs across a bound
    if bad.any():
        h, a = c['next_obs'][bad, 0], c['next_obs'][bad, 1]
        near = (np.abs(h[:, None] - np.array([0.7, 0.8, 2.0])).min(1) < 1e-4) | \
               (np.abs(np.abs(a)[:, None] - np.array([0.2, 1.0])).min(1) < 1e-4)
        assert near.all()


def test_termination_vs_reference():
    z = np.load(os.path.join(GOLD, 'termination.npz'))
    nobs = z['next_obs']
    dummy = np.zeros((len(nobs), 17)), np.zeros((len(nobs), 6))
    for d in ('halfcheetah', 'walker2d', 'hopper'):
        np.testing.assert_array_equal(ofe.TERMINATION[d](dummy[0], dummy[1], nobs), z['done_' + d])


def test_termination_more_domains_vs_reference():
    """ant, antangle, humanoid and the never-done domains: oracle and the host StaticFns vs the reference's
    own termination_fn outputs (tests/golden/make_termination_more.py)."""
    from mopo_amd.static import static_fns, term_kind_of
    z = np.load(os.path.join(GOLD, 'termination_more.npz'))
    nobs = z['next_obs']
    dummy = np.zeros((len(nobs), 17)), np.zeros((len(nobs), 6))
    for d in ('ant', 'antangle', 'humanoid', 'halfcheetahjump', 'halfcheetahvel', 'halfcheetahveljump',
              'point2denv', 'point2dwallenv', 'pendulum'):
        ref = np.asarray(z['done_' + d]).astype(bool)         # pendulum.py returns float zeros
        with np.errstate(invalid='ignore'):
            np.testing.assert_array_equal(ofe.TERMINATION[d](dummy[0], dummy[1], nobs), ref)
        np.testing.assert_array_equal(static_fns[d].termination_fn(dummy[0], dummy[1], nobs), ref)
        # the reference's StaticFns classes map to the same device kind by module name
        ref_like = type('StaticFns', (), {'__module__': 'ref_static_' + d})
        assert term_kind_of(ref_like) == static_fns[d].term_kind
    assert z['done_ant'].any() and z['done_humanoid'].any() and not z['done_ant'].all()
    # the host StaticFns on torch tensors returns the same mask as a tensor
    import torch
    t = torch.from_numpy(nobs)
    for d in ('ant', 'humanoid', 'walker2d', 'hopper', 'pendulum'):
        got = static_fns[d].termination_fn(torch.zeros(len(nobs), 17), torch.zeros(len(nobs), 6), t)
        assert isinstance(got, torch.Tensor) and got.dtype == torch.bool and tuple(got.shape) == (len(nobs), 1)
        with np.errstate(invalid='ignore'):
            np.testing.assert_array_equal(got.numpy(), ofe.TERMINATION[d](dummy[0], dummy[1], nobs))


def test_pool_vs_reference():
    z = np.load(os.path.join(GOLD, 'pool_trace.npz'))
    pool = opool.Pool(17, 6, int(z['max_size']))
    for i, n in enumerate(z['adds']):
        if n == 0:
            continue
        s = {k: z['add%d_%s' % (i, k)] for k in opool.FIELDS}
        pool.add_samples(s)
        assert pool._pointer == int(z['add%d_ptr' % i]) and pool.size == int(z['add%d_size' % i])
        np.random.seed(50 + i)
        idx = pool.random_indices(33)
        np.testing.assert_array_equal(idx, z['add%d_batch_idx' % i])
        b = pool.batch_by_indices(idx)
        for k in opool.FIELDS:
            np.testing.assert_array_equal(b[k], z['add%d_batch_%s' % (i, k)])
    for k, v in pool.return_all_samples().items():
        np.testing.assert_array_equal(v, z['final_' + k])


def test_numpy_choice_is_randint_index():
    """bnn.py:343 np.random.choice(list, n) == list[randint(0, len, n)] (legacy stream)."""
    el = [4, 0, 6, 2, 5]
    np.random.seed(3); a = np.random.choice(el, size=1000)
    np.random.seed(3); b = np.array(el)[np.random.randint(0, len(el), 1000)]
    np.testing.assert_array_equal(a, b)


def test_sac_oracle_matches_torch_autograd():
    torch = pytest.importorskip('torch')
    O, A, H, n = 17, 6, 32, 64
    rs = np.random.RandomState(0)
    params = osac.init_params(O, A, H, seed=5)
    params = [p + rs.normal(size=p.shape) * 0.05 for p in params]   # non-zero biases
    st = osac.SACState(params, log_alpha=0.1)
    batch = {'observations': rs.normal(size=(n, O)), 'actions': rs.uniform(-1, 1, (n, A)),
             'next_observations': rs.normal(size=(n, O)), 'rewards': rs.normal(size=(n, 1)),
             'terminals': rs.uniform(size=(n, 1)) < 0.2}
    e1, e2 = rs.normal(size=(n, A)), rs.normal(size=(n, A))
    # torch restatement of the same graph (autograd gradients)
    T = [torch.tensor(p, dtype=torch.float64, requires_grad=True) for p in params]
    la = torch.tensor(0.1, dtype=torch.float64, requires_grad=True)
    s = torch.tensor(batch['observations']); a = torch.tensor(batch['actions'])
    s2 = torch.tensor(batch['next_observations']); r = torch.tensor(batch['rewards'][:, 0])
    d = torch.tensor(batch['terminals'][:, 0].astype(np.float64))

    def pi(P, x, eps):
        h = torch.relu(x @ P[0] + P[1]); h = torch.relu(h @ P[2] + P[3])
        mu = h @ P[4] + P[5]
        ls = torch.clamp(h @ P[6] + P[7], -20, 2)
        std = torch.exp(ls); u = mu + torch.tensor(eps) * std
        logp = torch.sum(-0.5 * (((u - mu) / (std + 1e-8)) ** 2 + 2 * ls + np.log(2 * np.pi)), -1)
        logp = logp - torch.sum(2 * (np.log(2) - u - torch.nn.functional.softplus(-2 * u)), -1)
        return torch.tanh(u), logp

    def q(Q, x, act):
        z = torch.cat([x, act], -1)
        h = torch.relu(z @ Q[0] + Q[1]); h = torch.relu(h @ Q[2] + Q[3])
        return (h @ Q[4] + Q[5])[:, 0]

    P, Q1, Q2 = T[0:8], T[8:14], T[14:20]
    Tg = [torch.tensor(p) for p in params]
    alpha = torch.exp(la)
    api, logp = pi(P, s, e1)
    q1p, q2p = q(Q1, s, api), q(Q2, s, api)
    an, logpn = pi(P, s2, e2)
    y = (r + 0.99 * (1 - d) * (torch.minimum(q(Tg[8:14], s2, an), q(Tg[14:20], s2, an)) - alpha * logpn)).detach()
    l1 = 0.5 * torch.mean((q(Q1, s, a) - y) ** 2)
    l2 = 0.5 * torch.mean((q(Q2, s, a) - y) ** 2)
    lpi = torch.mean(alpha.detach() * logp - torch.minimum(q1p, q2p))
    gpi = torch.autograd.grad(lpi, P, retain_graph=True)
    gq1 = torch.autograd.grad(l1, Q1, retain_graph=True)
    gq2 = torch.autograd.grad(l2, Q2, retain_graph=True)
    # oracle gradients via one step with lr -> recover through Adam's first-step sign? compare directly:
    Pn, Q1n, Q2n = osac.split(st.params)
    _, a_pi, logp_pi, _, cpi = osac.pi_forward(Pn, batch['observations'], e1)
    q1_pi, c1p = osac.q_forward(Q1n, batch['observations'], a_pi)
    q2_pi, c2p = osac.q_forward(Q2n, batch['observations'], a_pi)
    sel = q1_pi <= q2_pi
    _, dx1 = osac.q_backward(Q1n, c1p, np.where(sel, -1.0 / n, 0.0), need_params=False)
    _, dx2 = osac.q_backward(Q2n, c2p, np.where(sel, 0.0, -1.0 / n), need_params=False)
    g_pi = osac.pi_backward(Pn, cpi, np.full(n, np.exp(0.1) / n), dx1[:, O:] + dx2[:, O:])
    for go, gt in zip(g_pi, gpi):
        np.testing.assert_allclose(go, gt.numpy(), rtol=1e-9, atol=1e-12)
    logs = osac.sac_step(st, batch, e1, e2)
    np.testing.assert_allclose(logs['Q/q1_loss'], l1.item(), rtol=1e-12)
    np.testing.assert_allclose(logs['sac_Q/q2_loss'], l2.item(), rtol=1e-12)
    np.testing.assert_allclose(logs['pi_loss'], lpi.item(), rtol=1e-12)
    # q1 gradients through the Adam first step: param delta = -lr * g/(|g|+eps') elementwise sign-like
    lr_t = 3e-4 * np.sqrt(1 - 0.999) / (1 - 0.9)
    for p0, p1, gt in zip(params[8:14], st.params[8:14], gq1):
        g = gt.numpy()
        m, v = 0.1 * g, 0.001 * g * g
        np.testing.assert_allclose(p1, p0 - lr_t * m / (np.sqrt(v) + 1e-8), rtol=1e-9, atol=1e-15)
    for p0, p1, gt in zip(params[14:20], st.params[14:20], gq2):
        g = gt.numpy()
        np.testing.assert_allclose(p1, p0 - lr_t * 0.1 * g / (np.sqrt(0.001 * g * g) + 1e-8), rtol=1e-9, atol=1e-15)


def test_philox_known_answers():
    """oracle/rng.py Philox4x32-10 against the Random123 known-answer vectors (counter, key -> out)."""
    from oracle.rng import philox4x32_10
    kat = [((0, 0, 0, 0, 0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
           ((0xffffffff,) * 6, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
           ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344, 0xa4093822, 0x299f31d0),
            (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    for inp, out in kat:
        assert tuple(int(x) for x in philox4x32_10(*inp)) == out


def test_perf_streams_shape_and_range():
    from oracle import rng
    uid = np.arange(5000)
    idx = rng.start_rows(uid, 7, 0, 333)
    assert idx.min() >= 0 and idx.max() < 333 and len(np.unique(idx)) == 333
    z = rng.obs_noise(uid, 7, 1, 18)
    assert z.shape == (5000, 18) and abs(z.mean()) < 0.02 and abs(z.std() - 1) < 0.02
    assert (rng.act_noise(uid, 7, 1, 6) != rng.act_noise(uid, 7, 2, 6)).all()   # step is in the counter
    sel = rng.model_choice(uid, 7, 1, [4, 1, 0, 6, 2])
    assert set(np.unique(sel)) == {0, 1, 2, 4, 6}


# ---- rollout-length schedule and model-pool sizing (mopo.py:675-711) ----------------
SCHEDULES = [[20, 100, 1, 1], [20, 100, 5, 5], [20, 100, 1, 5], [0, 10, 5, 1], [3, 7, 1, 15]]


@pytest.mark.parametrize('schedule', SCHEDULES, ids=[str(s) for s in SCHEDULES])
def test_set_rollout_length_vs_oracle(schedule):
    """MOPO._set_rollout_length (the host mirror) against oracle.rollout.rollout_length for every
    epoch of a 0..150 sweep, on a stub carrying only the fields the method reads."""
    from types import SimpleNamespace
    from mopo_amd.mopo import MOPO
    from oracle import rollout as orl
    for epoch in range(151):
        stub = SimpleNamespace(_rollout_schedule=schedule, _epoch=epoch)
        MOPO._set_rollout_length(stub)
        assert stub._rollout_length == orl.rollout_length(epoch, schedule), epoch
    # hand values of the ramp (mopo.py:680-684): int() truncates
    assert orl.rollout_length(21, [20, 100, 1, 5]) == 1
    assert orl.rollout_length(40, [20, 100, 1, 5]) == 2
    assert orl.rollout_length(99, [20, 100, 1, 5]) == 4
    assert orl.rollout_length(100, [20, 100, 1, 5]) == 5


def test_model_pool_size_configs():
    """mopo.py:693-695 at the D4RL configs' values (rollout_batch 50k, epoch_length 1000 = model_train_freq,
    retain 5): h=5 -> 1.25e6 rows, h=1 -> 2.5e5."""
    from oracle import rollout as orl
    assert orl.model_pool_size(50000, 1000, 1000, 5, 5) == 1250000
    assert orl.model_pool_size(50000, 1000, 1000, 1, 5) == 250000
    assert orl.model_pool_size(100000, 1000, 250, 1, 20) == 8000000


def test_sac_oracle_normal_action_prior_matches_torch_autograd():
    """softlearning SAC's action_prior='normal' (sac.py:285-289): the policy loss subtracts the standard-
    normal log-prob of pi's action; the oracle's policy gradient and loss against torch autograd."""
    torch = pytest.importorskip('torch')
    O, A, H, n = 11, 3, 32, 48
    rs = np.random.RandomState(4)
    params = [p + rs.normal(size=p.shape) * 0.05 for p in osac.init_params(O, A, H, seed=6)]
    st = osac.SACState(params, log_alpha=-0.2)
    batch = {'observations': rs.normal(size=(n, O)), 'actions': rs.uniform(-1, 1, (n, A)),
             'next_observations': rs.normal(size=(n, O)), 'rewards': rs.normal(size=(n, 1)),
             'terminals': rs.uniform(size=(n, 1)) < 0.2}
    e1, e2 = rs.normal(size=(n, A)), rs.normal(size=(n, A))
    T = [torch.tensor(p, dtype=torch.float64, requires_grad=True) for p in params]
    s = torch.tensor(batch['observations'])

    def pi(P, x, eps):
        h = torch.relu(x @ P[0] + P[1]); h = torch.relu(h @ P[2] + P[3])
        mu = h @ P[4] + P[5]
        ls = torch.clamp(h @ P[6] + P[7], -20, 2)
        std = torch.exp(ls); u = mu + torch.tensor(eps) * std
        logp = torch.sum(-0.5 * (((u - mu) / (std + 1e-8)) ** 2 + 2 * ls + np.log(2 * np.pi)), -1)
        logp = logp - torch.sum(2 * (np.log(2) - u - torch.nn.functional.softplus(-2 * u)), -1)
        return torch.tanh(u), logp

    def q(Q, x, act):
        z = torch.cat([x, act], -1)
        h = torch.relu(z @ Q[0] + Q[1]); h = torch.relu(h @ Q[2] + Q[3])
        return (h @ Q[4] + Q[5])[:, 0]

    P, Q1, Q2 = T[0:8], T[8:14], T[14:20]
    api, logp = pi(P, s, e1)
    prior = -0.5 * torch.sum(api * api, -1) - 0.5 * A * np.log(2 * np.pi)
    lpi = torch.mean(np.exp(-0.2) * logp - torch.minimum(q(Q1, s, api), q(Q2, s, api)) - prior)
    gpi = torch.autograd.grad(lpi, P)
    got = {}
    logs = osac.sac_step(st, batch, e1, e2, grads_out=got, action_prior='normal')
    np.testing.assert_allclose(logs['pi_loss'], lpi.item(), rtol=1e-12)
    for go, gt in zip(got['pi'], gpi):
        np.testing.assert_allclose(go, gt.numpy(), rtol=1e-9, atol=1e-12)
