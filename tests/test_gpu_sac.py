"""GPU parity: the SAC update (K6/K7) vs the fp64 oracle restatement of mopo.py's graph.

Tolerances (fp32 device vs fp64 oracle, identical batch rows and policy noise):
  * losses / logged means / alpha / grad norms:      rel 2e-4
  * gradients (every parameter):                      |d| <= 1e-4 * max|g| of that tensor + 1e-7
  * Adam m, v after one step: follow from the gradient tolerance (checked the same way)
  * params after one step: |d| <= 1e-6 + 2*lr_t where a gradient is ~0 (Adam's first step is
    lr_t*sign(g), so a sign flip of a vanishing gradient moves a param by <= 2 lr_t); all others 1e-6
  * 20 steps: losses within 1e-3 relative (chaotic divergence afterwards is expected)
"""
import numpy as np
import pytest

from oracle import replay_pool as opool
from oracle import sac as osac

pytestmark = pytest.mark.gpu
O, A, H = 17, 6, 256


def pools(rs, n_env_rows=500, n_model_rows=3000):
    import torch
    from mopo_amd.replay_pool import SimpleReplayPool
    out = []
    for n in (n_env_rows, n_model_rows):
        s = {'observations': rs.normal(size=(n, O)).astype(np.float32),
             'actions': rs.uniform(-1, 1, (n, A)).astype(np.float32),
             'next_observations': rs.normal(size=(n, O)).astype(np.float32),
             'rewards': rs.normal(size=(n, 1)).astype(np.float32),
             'terminals': rs.uniform(size=(n, 1)) < 0.1}
        p = SimpleReplayPool(obs_dim=O, act_dim=A, max_size=n + 10)
        p.add_samples(s)
        op = opool.Pool(O, A, n + 10)
        op.add_samples(s)
        out.append((p, op))
    torch.cuda.synchronize()
    return out


def draw(rs, env_size, model_size, n=256, n_env=12):
    idx = np.concatenate([rs.randint(0, env_size, n_env), rs.randint(0, model_size, n - n_env)])
    return idx, rs.normal(size=(n, A)).astype(np.float32), rs.normal(size=(n, A)).astype(np.float32)


def host_batch(env_op, mod_op, idx, n_env=12):
    b1 = env_op.batch_by_indices(idx[:n_env])
    b2 = mod_op.batch_by_indices(idx[n_env:])
    return {k: np.concatenate([b1[k], b2[k]]).astype(np.float64) for k in b1}   # mopo.py:815-816


def oracle_grads(st, batch, e1, e2, gamma=0.99, tent=-3.0):
    """Gradients of one step (pre-update params), same math as osac.sac_step."""
    s, a, s2 = batch['observations'], batch['actions'], batch['next_observations']
    r, d = batch['rewards'][:, 0], batch['terminals'][:, 0]
    n = s.shape[0]
    P, Q1, Q2 = osac.split(st.params)
    T = osac.split(st.target)
    alpha = np.exp(st.log_alpha)
    _, a_pi, logp_pi, _, cpi = osac.pi_forward(P, s, e1)
    q1_pi, c1p = osac.q_forward(Q1, s, a_pi)
    q2_pi, c2p = osac.q_forward(Q2, s, a_pi)
    _, a_n, logp_n, _, _ = osac.pi_forward(P, s2, e2)
    y = r + gamma * (1 - d) * (np.minimum(osac.q_forward(T[1], s2, a_n)[0], osac.q_forward(T[2], s2, a_n)[0])
                               - alpha * logp_n)
    q1, c1 = osac.q_forward(Q1, s, a)
    q2, c2 = osac.q_forward(Q2, s, a)
    g1, _ = osac.q_backward(Q1, c1, (q1 - y) / n)
    g2, _ = osac.q_backward(Q2, c2, (q2 - y) / n)
    sel = q1_pi <= q2_pi
    _, dx1 = osac.q_backward(Q1, c1p, np.where(sel, -1.0 / n, 0.0), need_params=False)
    _, dx2 = osac.q_backward(Q2, c2p, np.where(sel, 0.0, -1.0 / n), need_params=False)
    gp = osac.pi_backward(P, cpi, np.full(n, alpha / n), dx1[:, O:] + dx2[:, O:])
    return gp + g1 + g2, -np.mean(logp_pi + tent)


def flat(ts):
    return np.concatenate([np.asarray(t).ravel() for t in ts])


def test_sac_one_step_parity():
    from mopo_amd.sac import SAC
    rs = np.random.RandomState(0)
    (env_p, env_op), (mod_p, mod_op) = pools(rs)
    params = osac.init_params(O, A, H, seed=5)
    params = [p + rs.normal(size=p.shape) * 0.02 for p in params]        # non-zero biases
    fl = flat(params).astype(np.float32)
    sac = SAC(O, A, H, batch_size=256, real_ratio=0.05, target_entropy=-3, params=fl, log_alpha=0.1)
    assert sac.n_env == 12
    idx, e1, e2 = draw(rs, env_p.size, mod_p.size)
    st = osac.SACState([p.astype(np.float32).astype(np.float64) for p in params], log_alpha=np.float32(0.1))
    batch = host_batch(env_op, mod_op, idx)
    gref, garef = oracle_grads(st, batch, e1.astype(np.float64), e2.astype(np.float64))
    logs_ref = osac.sac_step(st, batch, e1.astype(np.float64), e2.astype(np.float64))
    sac._do_training(0, env_p, mod_p, idx=idx, eps_s=e1, eps_n=e2)
    lg = sac.logs()
    for k in ['Q/q1_loss', 'sac_Q/q2_loss', 'sac_Q/q1', 'sac_Q/q2', 'sac_pi/alpha', 'sac_pi/pi_entropy',
              'sac_pi/logp_pi', 'sac_pi/pi_global_norm', 'sac_Q/q_global_norm']:
        np.testing.assert_allclose(lg[k], logs_ref[k], rtol=2e-4, atol=1e-6, err_msg=k)
    np.testing.assert_allclose(lg['policy_loss'], logs_ref['pi_loss'], rtol=2e-4, atol=1e-6)
    g, ga = sac.get_grads()
    g = g.cpu().numpy()
    off = 0
    for i, gr in enumerate(gref):
        n = gr.size
        scale = np.abs(gr).max() + 1e-12
        err = np.abs(g[off:off + n] - gr.ravel()).max()
        assert err <= 1e-4 * scale + 1e-7, 'grad tensor %d: err %.3g scale %.3g' % (i, err, scale)
        off += n
    np.testing.assert_allclose(float(ga.item()), garef, rtol=1e-4, atol=1e-6)
    # updated params: Adam's first step is ~lr_t*sign(g)
    lr_t = 3e-4 * np.sqrt(1 - 0.999) / (1 - 0.9)
    p_new, la_new = sac.get_params()
    p_new = p_new.cpu().numpy()
    p_ref = flat(st.params)
    gr = flat(gref)
    d = np.abs(p_new - p_ref)
    tiny = np.abs(gr) < 1e-3 * np.abs(gr).max()
    assert d[~tiny].max() <= 1e-6 + 1e-6 * np.abs(p_ref[~tiny]).max()
    assert d[tiny].max() <= 1e-6 + 2 * lr_t
    np.testing.assert_allclose(float(la_new.item()), float(st.log_alpha), atol=1e-6)
    # Polyak target after the update
    tgt = sac.get_target().cpu().numpy()
    np.testing.assert_allclose(tgt, flat(st.target), atol=2e-6 + 5e-3 * 2 * lr_t)


def test_sac_twenty_steps_track_oracle():
    from mopo_amd.sac import SAC
    rs = np.random.RandomState(1)
    (env_p, env_op), (mod_p, mod_op) = pools(rs)
    params = osac.init_params(O, A, H, seed=6)
    sac = SAC(O, A, H, batch_size=256, real_ratio=0.05, target_entropy=-3, params=flat(params).astype(np.float32))
    st = osac.SACState([p.astype(np.float64) for p in params])
    for it in range(20):
        idx, e1, e2 = draw(rs, env_p.size, mod_p.size)
        ref = osac.sac_step(st, host_batch(env_op, mod_op, idx), e1.astype(np.float64), e2.astype(np.float64))
        sac._do_training(it, env_p, mod_p, idx=idx, eps_s=e1, eps_n=e2)
        lg = sac.logs()
        for k in ['Q/q1_loss', 'sac_Q/q2_loss', 'sac_pi/alpha', 'sac_pi/logp_pi']:
            np.testing.assert_allclose(lg[k], ref[k], rtol=1e-3, atol=1e-5, err_msg='%s @ step %d' % (k, it))


def test_sac_target_update_interval_vs_oracle():
    """target_update_interval = 2 (mopo.py:843-845): the Polyak update runs after the steps whose
    iteration is even; the others leave the targets as they were (oracle: tau = 0 on those steps)."""
    from mopo_amd.sac import SAC
    rs = np.random.RandomState(3)
    (env_p, env_op), (mod_p, mod_op) = pools(rs)
    params = osac.init_params(O, A, H, seed=7)
    sac = SAC(O, A, H, batch_size=256, real_ratio=0.05, target_entropy=-3, params=flat(params).astype(np.float32),
              target_update_interval=2)
    st = osac.SACState([p.astype(np.float64) for p in params])
    lr_t = 3e-4 * np.sqrt(1 - 0.999) / (1 - 0.9)
    for it in range(4):
        idx, e1, e2 = draw(rs, env_p.size, mod_p.size)
        before = sac.get_target().cpu().numpy()
        osac.sac_step(st, host_batch(env_op, mod_op, idx), e1.astype(np.float64), e2.astype(np.float64),
                      tau=5e-3 if it % 2 == 0 else 0.0)
        sac._do_training(it, env_p, mod_p, idx=idx, eps_s=e1, eps_n=e2)
        tgt = sac.get_target().cpu().numpy()
        if it % 2:
            np.testing.assert_array_equal(tgt, before)
        else:
            assert not np.array_equal(tgt, before)
        np.testing.assert_allclose(tgt, flat(st.target), atol=2e-6 + 5e-3 * 2 * lr_t * (it + 1), err_msg='step %d' % it)


@pytest.mark.parametrize('interval,repeat', [(3, 1), (2, 2)])
def test_sac_target_schedule_graph_matches_eager(interval, repeat):
    """The target schedule inside replayed graphs (8-step, 2-step, 1-step) equals eager steps, over two
    calls whose first timesteps are 0 and 5 (the base moves with the call), and differs from interval 1."""
    import torch
    from mopo_amd.rollout import init_sac_params
    from mopo_amd.sac import SAC
    rs = np.random.RandomState(4)
    (env_p, _), (mod_p, _) = pools(rs)
    init = init_sac_params(O, A, H, seed=10)
    runs = []
    for graph, every in ((True, interval), (False, interval), (True, 1)):
        s = SAC(O, A, H, params=init, use_graph=graph, target_entropy=-3, target_update_interval=every)
        s._do_training(0, env_p, mod_p, n_steps=5 * repeat, seed=77, n_train_repeat=repeat)
        s._do_training(5, env_p, mod_p, n_steps=13 * repeat, seed=77, n_train_repeat=repeat)
        torch.cuda.synchronize()
        runs.append((s.get_params()[0], s.get_target()))
    assert torch.equal(runs[0][0], runs[1][0]) and torch.equal(runs[0][1], runs[1][1])
    assert not torch.equal(runs[0][1], runs[2][1])


def test_sac_graph_replay_matches_eager():
    import torch
    from mopo_amd.sac import SAC
    rs = np.random.RandomState(2)
    (env_p, _), (mod_p, _) = pools(rs)
    fl = init = None
    from mopo_amd.rollout import init_sac_params
    init = init_sac_params(O, A, H, seed=9)
    a = SAC(O, A, H, params=init, use_graph=True, target_entropy=-3)
    b = SAC(O, A, H, params=init, use_graph=False, target_entropy=-3)
    a._do_training(0, env_p, mod_p, n_steps=50, seed=123)
    b._do_training(0, env_p, mod_p, n_steps=50, seed=123)
    torch.cuda.synchronize()
    pa, pb = a.get_params()[0], b.get_params()[0]
    assert torch.equal(pa, pb)
    assert torch.isfinite(pa).all()
    lg = a.logs()
    assert all(np.isfinite(v) for v in lg.values())


def test_training_batch_mirror():
    """SAC._training_batch (mopo.py:801-821): int(256 * 0.05) = 12 env rows then 244 model rows, each
    drawn with np.random.randint over the pool's size (flexible_replay_pool.py:85-87)."""
    from mopo_amd.sac import SAC
    rs = np.random.RandomState(7)
    (env, env_op), (mod, mod_op) = pools(rs)
    sac = SAC(O, A, H, batch_size=256, real_ratio=0.05, target_entropy=-3)
    np.random.seed(11)
    got = sac._training_batch(env, mod, as_numpy=True)
    np.random.seed(11)
    idx = np.concatenate([np.random.randint(0, env.size, 12), np.random.randint(0, mod.size, 244)])
    ref = host_batch(env_op, mod_op, idx)
    assert set(got) == set(ref)
    for k in ref:
        np.testing.assert_array_equal(np.asarray(got[k], np.float64), ref[k], err_msg=k)


@pytest.mark.parametrize('o,a,h,n', [(11, 3, 32, 100), (17, 6, 64, 250), (8, 8, 256, 40), (17, 6, (256, 128), 256),
                                     (11, 3, (48, 200), 100)])
def test_sac_one_step_gradients_odd_shapes(o, a, h, n):
    """One step's gradients at shapes the headline never uses: a batch that is not a multiple of 16
    (the policy-row blocks' and tiles' out-of-range rows), H < 256 (the policy-row MFMA's partial
    K split, column tiles not divisible by the 8 XCDs), A = 8 (the widest head), and non-square
    hidden_sizes [H1, H2] (mopo.py:275-280; run as the zero-padded square network, rollout.device_hidden)."""
    from mopo_amd.replay_pool import SimpleReplayPool
    from mopo_amd.sac import SAC
    import torch
    rs = np.random.RandomState(7)
    pl = []
    for rows in (300, 900):
        s = {'observations': rs.normal(size=(rows, o)).astype(np.float32),
             'actions': rs.uniform(-1, 1, (rows, a)).astype(np.float32),
             'next_observations': rs.normal(size=(rows, o)).astype(np.float32),
             'rewards': rs.normal(size=(rows, 1)).astype(np.float32),
             'terminals': rs.uniform(size=(rows, 1)) < 0.1}
        p = SimpleReplayPool(obs_dim=o, act_dim=a, max_size=rows)
        p.add_samples(s)
        op = opool.Pool(o, a, rows)
        op.add_samples(s)
        pl.append((p, op))
    torch.cuda.synchronize()
    (env_p, env_op), (mod_p, mod_op) = pl
    params = [p + rs.normal(size=p.shape) * 0.02 for p in osac.init_params(o, a, h, seed=9)]
    sac = SAC(o, a, h, batch_size=n, real_ratio=0.05, target_entropy=-3, params=flat(params).astype(np.float32),
              log_alpha=0.1)
    ne = sac.n_env
    idx = np.concatenate([rs.randint(0, 300, ne), rs.randint(0, 900, n - ne)])
    e1 = rs.normal(size=(n, a)).astype(np.float32)
    e2 = rs.normal(size=(n, a)).astype(np.float32)
    st = osac.SACState([p.astype(np.float32).astype(np.float64) for p in params], log_alpha=np.float32(0.1))
    batch = host_batch(env_op, mod_op, idx, n_env=ne)
    # oracle_grads reads the module's O for the action slice: pass this case's split explicitly
    s, act, s2 = batch['observations'], batch['actions'], batch['next_observations']
    r, d = batch['rewards'][:, 0], batch['terminals'][:, 0]
    P, Q1, Q2 = osac.split(st.params)
    T = osac.split(st.target)
    alpha = np.exp(st.log_alpha)
    _, a_pi, logp_pi, _, cpi = osac.pi_forward(P, s, e1.astype(np.float64))
    q1_pi, c1p = osac.q_forward(Q1, s, a_pi)
    q2_pi, c2p = osac.q_forward(Q2, s, a_pi)
    _, a_n, logp_n, _, _ = osac.pi_forward(P, s2, e2.astype(np.float64))
    y = r + 0.99 * (1 - d) * (np.minimum(osac.q_forward(T[1], s2, a_n)[0], osac.q_forward(T[2], s2, a_n)[0])
                              - alpha * logp_n)
    g1, _ = osac.q_backward(Q1, osac.q_forward(Q1, s, act)[1], (osac.q_forward(Q1, s, act)[0] - y) / n)
    g2, _ = osac.q_backward(Q2, osac.q_forward(Q2, s, act)[1], (osac.q_forward(Q2, s, act)[0] - y) / n)
    sel = q1_pi <= q2_pi
    _, dx1 = osac.q_backward(Q1, c1p, np.where(sel, -1.0 / n, 0.0), need_params=False)
    _, dx2 = osac.q_backward(Q2, c2p, np.where(sel, 0.0, -1.0 / n), need_params=False)
    gp = osac.pi_backward(P, cpi, np.full(n, alpha / n), dx1[:, o:] + dx2[:, o:])
    gref = gp + g1 + g2
    sac._do_training(0, env_p, mod_p, idx=idx, eps_s=e1, eps_n=e2)
    g = sac.get_grads()[0].cpu().numpy()
    off = 0
    for i, gr in enumerate(gref):
        m = gr.size
        scale = np.abs(gr).max() + 1e-12
        err = np.abs(g[off:off + m] - gr.ravel()).max()
        assert err <= 1e-4 * scale + 1e-7, 'grad tensor %d: err %.3g scale %.3g' % (i, err, scale)
        off += m


def test_sac_normal_action_prior_one_step_vs_oracle():
    """softlearning SAC's action_prior='normal' (sac.py:285-289) through the device step: the policy loss
    log and every gradient against the fp64 oracle with the prior (tolerances as test_sac_one_step_parity),
    then a graph-replayed second run of the same step equals the eager one (the flag is captured)."""
    from mopo_amd.sac import SAC
    rs = np.random.RandomState(8)
    (env_p, env_op), (mod_p, mod_op) = pools(rs)
    params = [p + rs.normal(size=p.shape) * 0.02 for p in osac.init_params(O, A, H, seed=5)]
    fl = flat(params).astype(np.float32)
    sac = SAC(O, A, H, batch_size=256, real_ratio=0.05, target_entropy=-3, params=fl, log_alpha=0.1,
              action_prior='normal')
    idx, e1, e2 = draw(rs, env_p.size, mod_p.size)
    st = osac.SACState([p.astype(np.float32).astype(np.float64) for p in params], log_alpha=np.float32(0.1))
    batch = host_batch(env_op, mod_op, idx)
    got = {}
    logs_ref = osac.sac_step(st, batch, e1.astype(np.float64), e2.astype(np.float64), grads_out=got,
                             action_prior='normal')
    sac._do_training(0, env_p, mod_p, idx=idx, eps_s=e1, eps_n=e2)
    lg = sac.logs()
    np.testing.assert_allclose(lg['policy_loss'], logs_ref['pi_loss'], rtol=2e-4, atol=1e-6)
    np.testing.assert_allclose(lg['Q/q1_loss'], logs_ref['Q/q1_loss'], rtol=2e-4, atol=1e-6)
    g = sac.get_grads()[0].cpu().numpy()
    off = 0
    for i, gr in enumerate(got['pi'] + got['q1'] + got['q2']):
        n = gr.size
        err = np.abs(g[off:off + n] - gr.ravel()).max()
        assert err <= 1e-4 * (np.abs(gr).max() + 1e-12) + 1e-7, 'grad tensor %d: err %.3g' % (i, err)
        off += n
    # perf mode: graph replay with the prior equals the eager path
    outs = []
    for use_graph in (True, False):
        s2 = SAC(O, A, H, batch_size=256, real_ratio=0.05, target_entropy=-3, params=fl, log_alpha=0.1,
                 action_prior='normal', use_graph=use_graph)
        s2._do_training(0, env_p, mod_p, n_steps=3, seed=11)
        outs.append(s2.get_params()[0].cpu().numpy())
    np.testing.assert_array_equal(outs[0], outs[1])


def test_sac_nonsquare_hidden_steps_vs_oracle():
    """hidden_sizes [256, 128] (mopo.py:275-280, 311-325) over 30 perf-mode steps (graph replay, device
    Philox batches and noise) against the fp64 oracle run on the same restated streams (oracle/rng.py):
    losses within 1e-3 relative at the last step, parameters / targets / Adam moments scaled error p99
    <= 1e-4; and the zero padding of the device's square network stays exactly 0 in every buffer."""
    import torch
    from oracle import rng as orng
    from mopo_amd.sac import SAC
    hs = (256, 128)
    rs = np.random.RandomState(12)
    (env_p, env_op), (mod_p, mod_op) = pools(rs)
    params = [p + rs.normal(size=p.shape) * 0.02 for p in osac.init_params(O, A, hs, seed=13)]
    fl = flat(params).astype(np.float32)
    sac = SAC(O, A, list(hs), batch_size=256, real_ratio=0.05, target_entropy=-3, params=fl)
    assert sac.hidden == 256 and sac.hidden_sizes == hs and sac.n_params == fl.size
    K, seed = 30, 77
    sac._do_training(0, env_p, mod_p, n_steps=K, seed=seed)
    torch.cuda.synchronize()
    st = osac.SACState([p.astype(np.float32).astype(np.float64) for p in params])
    for k in range(K):
        idx = orng.sac_batch_indices(256, 12, env_p.size, mod_p.size, seed, k)
        lg = osac.sac_step(st, host_batch(env_op, mod_op, idx), orng.sac_noise(256, A, seed, k, 0).astype(np.float64),
                           orng.sac_noise(256, A, seed, k, 1).astype(np.float64), target_entropy=-3.0)
    dl = sac.logs()
    for dk, rk in (('Q/q1_loss', 'Q/q1_loss'), ('sac_Q/q2_loss', 'sac_Q/q2_loss'), ('policy_loss', 'pi_loss')):
        assert abs(dl[dk] - lg[rk]) <= 1e-3 * (1 + abs(lg[rk])), (dk, dl[dk], lg[rk])
    dev = {k: v.cpu().numpy().astype(np.float64) for k, v in sac.state_dict().items()}
    ref = {'params': np.append(flat(st.params), st.log_alpha), 'target': flat(st.target),
           'adam_m': np.concatenate([flat(st.opt_pi.m), flat(st.opt_q1.m), flat(st.opt_q2.m), flat(st.opt_a.m)]),
           'adam_v': np.concatenate([flat(st.opt_pi.v), flat(st.opt_q1.v), flat(st.opt_q2.v), flat(st.opt_a.v)])}
    for k in ref:
        err = np.abs(dev[k] - ref[k]) / (1 + np.abs(ref[k]))
        assert np.quantile(err, 0.99) <= 1e-4 and err.max() <= 1e-2, (k, np.quantile(err, 0.99), err.max())
    # the raw device buffers: everything outside the [H1, H2] corner of each tensor is exactly zero
    pad = np.ones(sac._n_dev, bool)
    pad[sac._pad] = False
    for w, extra in ((0, 1), (1, 0), (2, 1), (3, 1), (4, 1)):
        raw = sac._copy(w, sac._n_dev + extra).cpu().numpy()[:sac._n_dev]
        assert np.all(raw[pad] == 0), (w, np.abs(raw[pad]).max())


@pytest.mark.parametrize('o,a,h,n', [(17, 6, 256, 256), (11, 3, 64, 100)])
def test_sac_fused_launches_bit_identical_to_separate_launches(o, a, h, n, monkeypatch):
    """The fused launches (sac_rows.h sac_f2b1_kernel: F2 + B1, sac_f12b1_kernel: F1 + F2 + B1, with
    in-launch row-block hand-offs instead of kernel boundaries) compute exactly the separate launches'
    arithmetic, so 300 graph-replayed steps must end bit-identical to MOPO_SAC_FUSE=0 -- any stale read of a handed-off line (L1 / L2 non-coherence,
    sac_rows.h handoff_wait) would show as a difference -- and the logs must stay finite (a consumer that
    gave up waiting poisons them)."""
    import torch
    from mopo_amd.replay_pool import SimpleReplayPool
    from mopo_amd.sac import SAC
    rs = np.random.RandomState(21)
    pl = []
    for rows in (400, 2000):
        s = {'observations': rs.normal(size=(rows, o)).astype(np.float32),
             'actions': rs.uniform(-1, 1, (rows, a)).astype(np.float32),
             'next_observations': rs.normal(size=(rows, o)).astype(np.float32),
             'rewards': rs.normal(size=(rows, 1)).astype(np.float32),
             'terminals': rs.uniform(size=(rows, 1)) < 0.1}
        p = SimpleReplayPool(obs_dim=o, act_dim=a, max_size=rows)
        p.add_samples(s)
        pl.append(p)
    fl = flat(osac.init_params(o, a, h, seed=3)).astype(np.float32)
    out = {}
    for fuse in ('0', '1', '2'):
        monkeypatch.setenv('MOPO_SAC_FUSE', fuse)
        sac = SAC(o, a, h, batch_size=n, real_ratio=0.05, target_entropy=-3, params=fl)
        sac._do_training(0, pl[0], pl[1], n_steps=300, seed=19)
        torch.cuda.synchronize()
        lg = sac.logs()
        assert all(np.isfinite(v) for v in lg.values()), (fuse, lg)
        out[fuse] = {k: v.cpu().numpy() for k, v in sac.state_dict().items()}
    for f in ('1', '2'):
        for k in out['0']:
            np.testing.assert_array_equal(out[f][k], out['0'][k], err_msg='MOPO_SAC_FUSE=%s %s' % (f, k))


def test_sac_handoff_timeout_holds_updates_and_is_reported():
    """A bounded hand-off wait that gives up (sac_rows.h handoff_wait) sets the sticky timeout word: every later
    step must then hold its parameter / Adam / target updates (no update computed from stale operands), write
    NaN logs, and SAC.check() / logs() must raise once and clear the word, after which steps update again."""
    import ctypes as C

    import torch
    from mopo_amd import _lib as L
    from mopo_amd.replay_pool import SimpleReplayPool
    from mopo_amd.sac import SAC
    o, a, h, n = 11, 3, 64, 100
    rs = np.random.RandomState(23)
    pl = []
    for rows in (400, 2000):
        s = {'observations': rs.normal(size=(rows, o)).astype(np.float32),
             'actions': rs.uniform(-1, 1, (rows, a)).astype(np.float32),
             'next_observations': rs.normal(size=(rows, o)).astype(np.float32),
             'rewards': rs.normal(size=(rows, 1)).astype(np.float32),
             'terminals': rs.uniform(size=(rows, 1)) < 0.1}
        p = SimpleReplayPool(obs_dim=o, act_dim=a, max_size=rows)
        p.add_samples(s)
        pl.append(p)
    sac = SAC(o, a, h, batch_size=n, real_ratio=0.05, target_entropy=-3,
              params=flat(osac.init_params(o, a, h, seed=3)).astype(np.float32))
    sac._do_training(0, pl[0], pl[1], n_steps=5, seed=19)
    sac.check()                                          # no give-up so far
    before = {k: v.cpu().numpy() for k, v in sac.state_dict().items()}
    L.check(L.lib().mopo_sac_inject_timeout(sac._h))
    sac._do_training(5, pl[0], pl[1], n_steps=9, seed=19)
    torch.cuda.synchronize()
    held = {k: v.cpu().numpy() for k, v in sac.state_dict().items()}
    for k in before:
        np.testing.assert_array_equal(held[k], before[k], err_msg=k)
    v = sac._copy(5, 10).cpu().numpy()
    assert np.all(np.isnan(v[[0, 1, 2, 3, 4, 5, 6, 9]])), v   # losses, means, alpha (7, 8: the gradient norms)
    with pytest.raises(RuntimeError, match='timed out'):
        sac.logs()
    flag = C.c_int(-1)
    L.check(L.lib().mopo_sac_check(sac._h, C.byref(flag)))   # cleared by the report
    assert flag.value == 0
    sac._do_training(14, pl[0], pl[1], n_steps=3, seed=19)
    lg = sac.logs()
    assert all(np.isfinite(x) for x in lg.values()), lg
    after = sac.state_dict()['params'].cpu().numpy()
    assert np.abs(after - before['params']).max() > 0
