"""Generate golden fixtures by EXECUTING the reference's own numpy code.

Run in the build container only (needs /root/reference; nothing here runs on the GPU box):

    python tests/golden/make_golden.py

What executes from the reference (read-only, imported by file path with a stub
``tensorflow`` module, since TF 1.14 is not installed and is not needed by these
functions):
  * mopo/models/fake_env.py  ``FakeEnv.step`` / ``_get_logprob``          (fake_env.py:20-131)
  * mopo/models/bnn.py       ``BNN.random_inds``                         (bnn.py:342-344)
  * mopo/static/{halfcheetah,walker2d,hopper}.py ``termination_fn``
  * softlearning/replay_pools/flexible_replay_pool.py ``FlexibleReplayPool``
The TF-only ensemble forward (bnn.py:631-675) is the reference's own ``BNN._compile_outputs``
executed in f32 under the torch-backed TF stand-in (make_ref_vectors.py / tfstub.py), so every
float in the rollout fixtures comes from reference code; for B <= 64 the forward's mean/var are
stored too (``ref_mean`` / ``ref_var``) so the oracle's post-processing can be pinned bit-exactly.
Outputs: tests/golden/*.npz (inputs + expected outputs only; no reference source).
"""
import importlib.util
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = '/root/reference'
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from oracle import bnn as obnn  # noqa: E402


def _load(modname, path):
    spec = importlib.util.spec_from_file_location(modname, path)
    m = importlib.util.module_from_spec(spec)
    sys.modules[modname] = m
    spec.loader.exec_module(m)
    return m


def load_reference():
    from make_ref_vectors import load_reference as load_graph_code
    refs = load_graph_code()                 # tfstub as ``tensorflow``; fc / utils / bnn / mopo
    bnn = refs[2]
    fe = _load('mopo.models.fake_env', os.path.join(REF, 'mopo/models/fake_env.py'))
    static = {d: _load('ref_static_' + d, os.path.join(REF, 'mopo/static/%s.py' % d)).StaticFns
              for d in ('halfcheetah', 'walker2d', 'hopper')}
    _load('softlearning.replay_pools.replay_pool', os.path.join(REF, 'softlearning/replay_pools/replay_pool.py'))
    frp = _load('softlearning.replay_pools.flexible_replay_pool',
                os.path.join(REF, 'softlearning/replay_pools/flexible_replay_pool.py'))
    return refs, bnn, fe, static, frp


class _Model:
    """Stand-in for the TF BNN: reference ``random_inds`` + the reference graph's forward (f32)."""

    def __init__(self, refs, bnn_mod, params, E, elites):
        import torch
        from make_ref_vectors import build_bnn
        self._refs, self._p, self.num_nets, self._model_inds = refs, params, E, list(elites)
        self.random_inds = types.MethodType(bnn_mod.BNN.random_inds, self)
        self._obj = build_bnn(refs, params, E, 17, 6, params['W'][1].shape[1], True, torch.float32)
        self.last = None

    def predict(self, inputs, factored=True):
        import torch
        import tfstub
        assert factored
        x = tfstub.w(torch.as_tensor(np.asarray(inputs, np.float32)))       # the f32 placeholder feed
        mean, var = self._refs[2].BNN._compile_outputs(self._obj, x)
        self.last = (mean.detach().numpy().copy(), var.detach().numpy().copy())
        return self.last


def make_fakeenv_cases(refs, bnn_mod, fe_mod, static):
    cases = []
    rs = np.random.RandomState(1234)
    cid = 0
    for (E, H) in ((7, 64), (32, 32)):
        O, A = 17, 6
        params = obnn.init_params(E, O, A, hidden=H, seed=10 + E,
                                  inputs=rs.normal(size=(500, O + A)) * 2 + 0.3)
        elites = list(rs.permutation(E)[:5])
        np.savez_compressed(os.path.join(HERE, 'bnn_E%d_H%d.npz' % (E, H)),
                            **{'w%d' % i: a for i, a in enumerate(obnn.to_mat_list(params))})
        for B in (1, 7, 64, 257):
            for domain in ('halfcheetah', 'walker2d', 'hopper'):
                for learned_var in (True, False):
                    for det in (False, True):
                        if det and B not in (7, 257):
                            continue
                        if E == 32 and (domain != 'walker2d' or B == 1):
                            continue
                        obs = rs.normal(size=(B, O)).astype(np.float32)
                        if domain == 'walker2d':
                            obs[:, 0] = rs.uniform(0.5, 2.3, size=B)
                            obs[:, 1] = rs.uniform(-1.3, 1.3, size=B)
                        if domain == 'hopper':
                            obs[:, 0] = rs.uniform(0.5, 1.5, size=B)
                            obs[:, 1] = rs.uniform(-0.4, 0.4, size=B)
                        if cid % 3 == 1:
                            obs = obs.astype(np.float64) + 1e-3  # later horizon steps feed f64 next_obs
                        act = rs.uniform(-1, 1, size=(B, A)).astype(np.float32)
                        coeff = 1.0 if cid % 2 == 0 else 5.0
                        seed = 1000 + cid
                        model = _Model(refs, bnn_mod, params, E, elites)
                        env = fe_mod.FakeEnv(model, static[domain], penalty_coeff=coeff,
                                             penalty_learned_var=learned_var)
                        np.random.seed(seed)
                        nobs, rew, term, info = env.step(obs, act, deterministic=det)
                        after = np.random.get_state()[2]
                        np.random.seed(seed)
                        noise = np.zeros((E, B, O + 1)) if det else np.random.normal(size=(E, B, O + 1))
                        inds = np.zeros(B, np.int64) if det else np.random.choice(elites, size=B)
                        assert det or np.random.get_state()[2] == after
                        # the normal stream is not stored: the test regenerates it from ``seed``
                        # (numpy's legacy stream is frozen) and checks model_inds bit-exact.
                        case = dict(E=E, H=H, B=B, domain=domain, learned_var=int(learned_var),
                                    deterministic=int(det), penalty_coeff=coeff, seed=seed,
                                    elites=np.array(elites, np.int64), obs=obs, act=act,
                                    model_inds=np.asarray(inds, np.int64),
                                    next_obs=nobs, rew=rew, term=term,
                                    info_mean=info['mean'], info_std=info['std'],
                                    log_prob=info['log_prob'], dev=info['dev'],
                                    unpenalized=info['unpenalized_rewards'], penalty=info['penalty'])
                        if B <= 64:
                            case['ref_mean'], case['ref_var'] = model.last
                        cases.append(case)
                        cid += 1
    return cases


def make_termination_cases(static):
    rs = np.random.RandomState(7)
    out = {}
    n = 4096
    nobs = rs.normal(size=(n, 17))
    nobs[:, 0] = rs.uniform(0.0, 2.5, size=n)
    nobs[:, 1] = rs.uniform(-1.5, 1.5, size=n)
    # exact boundary values and non-finite rows
    nobs[:8, 0] = [0.8, 2.0, 0.7, 0.8000001, 1.9999999, 0.69999, 0.70001, 1.0]
    nobs[8:16, 1] = [1.0, -1.0, 0.2, -0.2, 0.19999, -0.20001, 0.0, 0.99999]
    nobs[16, 3] = np.nan; nobs[17, 4] = np.inf; nobs[18, 5] = 100.0; nobs[19, 6] = 99.999; nobs[20, 2] = -np.inf
    obs = rs.normal(size=(n, 17)); act = rs.normal(size=(n, 6))
    out['next_obs'] = nobs
    for d, fns in static.items():
        out['done_' + d] = fns.termination_fn(obs, act, nobs)
    return out


def make_pool_trace(frp):
    fields = {
        'actions': {'shape': (6,), 'dtype': 'float32'},
        'rewards': {'shape': (1,), 'dtype': 'float32'},
        'terminals': {'shape': (1,), 'dtype': 'bool'},
        'observations': {'shape': (17,), 'dtype': 'float32'},
        'next_observations': {'shape': (17,), 'dtype': 'float32'},
    }
    rs = np.random.RandomState(3)
    pool = frp.FlexibleReplayPool(100, fields)
    out = {'max_size': 100}
    adds = [37, 50, 1, 25, 0, 60]
    for i, n in enumerate(adds):
        s = {'observations': rs.normal(size=(n, 17)), 'actions': rs.normal(size=(n, 6)).astype(np.float32),
             'next_observations': rs.normal(size=(n, 17)), 'rewards': rs.normal(size=(n, 1)),
             'terminals': rs.uniform(size=(n, 1)) < 0.3}
        if n == 0:
            continue
        pool.add_samples(s)
        for k, v in s.items():
            out['add%d_%s' % (i, k)] = v
        out['add%d_ptr' % i] = pool._pointer
        out['add%d_size' % i] = pool.size
        np.random.seed(50 + i)
        b = pool.random_batch(33)
        np.random.seed(50 + i)
        out['add%d_batch_idx' % i] = np.random.randint(0, pool.size, 33)
        for k, v in b.items():
            out['add%d_batch_%s' % (i, k)] = v
    out['adds'] = np.array(adds)
    for k, v in pool.return_all_samples().items():
        out['final_' + k] = v
    return out


def main():
    refs, bnn_mod, fe_mod, static, frp = load_reference()
    cases = make_fakeenv_cases(refs, bnn_mod, fe_mod, static)
    for i, c in enumerate(cases):
        np.savez_compressed(os.path.join(HERE, 'fakeenv_%03d.npz' % i), **c)
    np.savez_compressed(os.path.join(HERE, 'termination.npz'), **make_termination_cases(static))
    np.savez_compressed(os.path.join(HERE, 'pool_trace.npz'), **make_pool_trace(frp))
    print('wrote %d fakeenv cases' % len(cases))


if __name__ == '__main__':
    main()
