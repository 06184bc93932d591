"""Golden vectors for the TF-only parts of the path, made by EXECUTING the reference's own graph code
under a torch-backed TensorFlow stand-in (tests/golden/tfstub.py).

Run in the build container only (reads /root/reference; nothing here runs on the GPU box):

    python tests/golden/make_ref_vectors.py

Executed from the reference (read-only, loaded by file path; every other import stubbed):
  * ensemble forward: ``BNN.add`` (bnn.py:112-144) builds the layer stack exactly as
    ``construct_model`` does (constructor.py:28-36, joint head: finalize's set_output_dim /
    unset_activation, bnn.py:186-193), ``FC.construct_vars`` (fc.py:134-158) names the variables,
    then ``BNN._compile_outputs`` (bnn.py:631-675) -> ``TensorStandardScaler.transform``
    (utils.py:88-96) -> ``FC.compute_output_tensor`` (fc.py:84-106) on 2-D inputs (predict, bnn.py:530-536)
  * ensemble training loss: ``BNN._compile_losses`` (bnn.py:677-701) on 3-D inputs + the finalize
    loss terms (bnn.py:241-249: decays, 0.01 sum(maxlv) - 0.01 sum(minlv)); gradient by autograd
  * SAC: ``MOPO._build`` (mopo.py:204-466), ``get_action_meta`` (468-485), ``_do_training`` /
    ``_get_feed_dict`` / ``_update_target`` (834-874), for 3 consecutive steps (Adam state carried)
Each case is run twice: in f32 (the reference graph's dtype) and in f64 (to pin the f64 oracle
tightly).  Outputs: tests/golden/ref_*.npz -- inputs and outputs only, no reference source.
Large weight sets are not stored: they are regenerated from ``oracle.bnn.init_params(seed)`` and
pinned by their sha256 (stored with the case).
"""
import hashlib
import importlib.util
import io
import os
import sys
import types
from contextlib import redirect_stdout

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = '/root/reference'
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import tfstub  # noqa: E402
from oracle import bnn as obnn  # noqa: E402
from oracle import sac as osac  # noqa: E402


def _stub(name, **attrs):
    m = sys.modules.get(name) or types.ModuleType(name)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


def _load(modname, path):
    spec = importlib.util.spec_from_file_location(modname, path)
    m = importlib.util.module_from_spec(spec)
    sys.modules[modname] = m
    spec.loader.exec_module(m)
    return m


class _Sink:
    def __getattr__(self, name):
        return _Sink()

    def __call__(self, *a, **k):
        return _Sink()


def load_reference():
    tfstub.install()
    _stub('RLA'); _stub('RLA.easy_log', logger=_Sink()); _stub('RLA.easy_log.logger')
    _stub('RLA.easy_log.tester', tester=_Sink())
    for pkg in ('mopo', 'mopo.models', 'mopo.utils', 'mopo.algorithms', 'mopo.off_policy', 'softlearning',
                'softlearning.algorithms', 'softlearning.replay_pools', 'softlearning.samplers', 'softlearning.misc'):
        _stub(pkg)
    utils = _load('mopo.models.utils', os.path.join(REF, 'mopo/models/utils.py'))
    fc = _load('mopo.models.fc', os.path.join(REF, 'mopo/models/fc.py'))
    _load('mopo.utils.logging', os.path.join(REF, 'mopo/utils/logging.py'))
    bnn = _load('mopo.models.bnn', os.path.join(REF, 'mopo/models/bnn.py'))
    # mopo.py's other imports are not on the executed lines
    _stub('gtimer')
    _stub('softlearning.algorithms.rl_algorithm', RLAlgorithm=object)
    _stub('softlearning.replay_pools.simple_replay_pool', SimpleReplayPool=object)
    _stub('mopo.models.constructor', construct_model=None, format_samples_for_training=None)
    _stub('mopo.models.fake_env', FakeEnv=None)
    _stub('mopo.utils.writer', Writer=None)
    _stub('mopo.utils.visualization', visualize_policy=None)
    _stub('mopo.utils.filesystem')
    _stub('mopo.off_policy.loader')
    _stub('d4rl', infos=_Sink())
    mopo = _load('mopo.algorithms.mopo', os.path.join(REF, 'mopo/algorithms/mopo.py'))
    return utils, fc, bnn, mopo


def sha(arrs):
    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a, np.float32).tobytes())
    return h.hexdigest()


# ------------------------------------------------------------------------------------ ensemble
WD = (0.000025, 0.00005, 0.000075, 0.000075, 0.0001)    # constructor.py:30-34


def build_bnn(refs, p, E, O, A, H, smv, dtype):
    """Stand-in BNN whose layers are built by the reference's BNN.add / FC.construct_vars."""
    utils, fc, bnn, _ = refs
    tfstub.reset(dtype)
    obj = object.__new__(bnn.BNN)
    obj.name, obj.num_nets, obj.separate_mean_var = 'BNN', E, smv
    obj.finalized, obj.model_loaded = False, False
    obj.layers, obj.var_layers, obj.decays, obj.optvars, obj.nonoptvars = [], [], [], [], []
    obj.end_act = None
    D = O + 1
    with redirect_stdout(io.StringIO()):
        bnn.BNN.add(obj, fc.FC(H, input_dim=O + A, activation='swish', weight_decay=WD[0]))
        bnn.BNN.add(obj, fc.FC(H, activation='swish', weight_decay=WD[1]))
        bnn.BNN.add(obj, fc.FC(H, activation='swish', weight_decay=WD[2]))
        bnn.BNN.add(obj, fc.FC(H, activation='swish', weight_decay=WD[3]))
        bnn.BNN.add(obj, fc.FC(D, weight_decay=WD[4]))
        if smv:
            bnn.BNN.add(obj, fc.FC(D, input_dim=H, weight_decay=0.0001), var_layer=True)
    if not smv:  # bnn.py:186-193
        obj.layers[-1].set_output_dim(2 * obj.layers[-1].get_output_dim())
        obj.end_act = obj.layers[-1].get_activation()
        obj.end_act_name = obj.layers[-1].get_activation(as_func=False)
        obj.layers[-1].unset_activation()
    # variable values (names as finalize's scopes create them, bnn.py:196-227)
    iv = tfstub.S.init_values
    for i in range(5):
        iv['BNN/Layer%i%s/FC_weights:0' % (i, '_mean' if smv else '')] = p['W'][i]
        iv['BNN/Layer%i%s/FC_biases:0' % (i, '_mean' if smv else '')] = p['b'][i]
    if smv:
        iv['BNN/Layer0_var/FC_weights:0'] = p['Wv']
        iv['BNN/Layer0_var/FC_biases:0'] = p['bv']
    iv['BNN/Scaler/scaler_mu:0'], iv['BNN/Scaler/scaler_std:0'] = p['mu'], p['sigma']
    iv['BNN/max_log_var:0'], iv['BNN/min_log_var:0'] = p['max_logvar'], p['min_logvar']
    with tfstub.variable_scope('BNN'):
        obj.scaler = utils.TensorStandardScaler(O + A)
        obj.max_logvar = tfstub.Variable(np.ones([1, D]) / 2., name='max_log_var')
        obj.min_logvar = tfstub.Variable(-np.ones([1, D]) * 10., name='min_log_var')
        for i, layer in enumerate(obj.layers):
            with tfstub.variable_scope('Layer%i%s' % (i, '_mean' if smv else '')):
                layer.construct_vars()
                obj.decays.extend(layer.get_decays())
        for i, layer in enumerate(obj.var_layers):
            with tfstub.variable_scope('Layer%i_var' % i):
                layer.construct_vars()
                obj.decays.extend(layer.get_decays())
    assert not tfstub.S.missing_init, tfstub.S.missing_init
    return obj


def bnn_forward_case(refs, name, E, H, B, smv, seed, store_weights, x_f64=False):
    O, A = 17, 6
    rs = np.random.RandomState(seed + 100)
    fit = rs.normal(size=(400, O + A)) * 1.5 + 0.2
    p = obnn.init_params(E, O, A, hidden=H, seed=seed, smv=smv, inputs=fit)
    mats = obnn.to_mat_list(p)
    x = rs.normal(size=(B, O + A)) * 1.5 + 0.2
    x[0] = 0.0
    x[1] = 40.0 * np.sign(rs.normal(size=O + A))   # far outside the data: saturated swish / bounds
    if not x_f64:
        x = x.astype(np.float32)
    out = dict(E=E, H=H, B=B, O=O, A=A, smv=int(smv), seed=seed, x=x, weights_sha=sha(mats))
    if store_weights:
        for i, m in enumerate(mats):
            out['w%d' % i] = m
    bnn = refs[2]
    for tag, dt in (('f32', torch.float32), ('f64', torch.float64)):
        obj = build_bnn(refs, p, E, O, A, H, smv, dt)
        xin = tfstub.w(torch.as_tensor(np.asarray(x, np.float32 if dt == torch.float32 else np.float64)))
        mean, var = bnn.BNN._compile_outputs(obj, xin)
        _, lv = bnn.BNN._compile_outputs(obj, xin, ret_log_var=True)
        out['mean_' + tag] = tfstub.u(mean).detach().numpy()
        out['var_' + tag] = tfstub.u(var).detach().numpy()
        out['logvar_' + tag] = tfstub.u(lv).detach().numpy()
    np.savez_compressed(os.path.join(HERE, 'ref_bnn_fwd_%s.npz' % name), **out)
    return out


def bnn_loss_case(refs, name, E, H, n, seed, smv=True):
    """train_loss = sum(_compile_losses(inc_var_loss=True)) + add_n(decays) + 0.01 sum maxlv - 0.01 sum minlv
    (bnn.py:241-246) and mse_loss (bnn.py:248), 3-D inputs [E, n, IN]; gradients w.r.t. optvars."""
    O, A = 17, 6
    rs = np.random.RandomState(seed + 200)
    p = obnn.init_params(E, O, A, hidden=H, seed=seed, smv=smv, inputs=rs.normal(size=(300, O + A)))
    X = rs.normal(size=(E, n, O + A)).astype(np.float32)
    Y = (rs.normal(size=(E, n, O + 1)) * 0.5).astype(np.float32)
    out = dict(E=E, H=H, n=n, seed=seed, X=X, Y=Y, smv=int(smv))
    for i, m in enumerate(obnn.to_mat_list(p)):
        out['w%d' % i] = m
    bnn = refs[2]
    for tag, dt in (('f32', torch.float32), ('f64', torch.float64)):
        obj = build_bnn(refs, p, E, O, A, H, smv, dt)
        xin, yin = tfstub.w(torch.as_tensor(X, dtype=dt)), tfstub.w(torch.as_tensor(Y, dtype=dt))
        loss = tfstub.reduce_sum(bnn.BNN._compile_losses(obj, xin, yin, inc_var_loss=True))
        loss = loss + tfstub.add_n(obj.decays)
        loss = loss + 0.01 * tfstub.reduce_sum(obj.max_logvar) - 0.01 * tfstub.reduce_sum(obj.min_logvar)
        mse = bnn.BNN._compile_losses(obj, xin, yin, inc_var_loss=False)
        optvars = []
        for l in obj.layers + obj.var_layers:
            optvars += l.get_vars()
        optvars += [obj.max_logvar, obj.min_logvar]
        grads = torch.autograd.grad(tfstub.u(loss), [tfstub.u(v) for v in optvars])
        out['loss_' + tag] = float(loss)
        out['mse_' + tag] = tfstub.u(mse).detach().numpy()
        for i, g in enumerate(grads):
            out['grad%d_%s' % (i, tag)] = g.numpy()
    np.savez_compressed(os.path.join(HERE, 'ref_bnn_loss_%s.npz' % name), **out)


# ------------------------------------------------------------------------------------ SAC
PI_LAYERS = ('dense', 'dense_1', 'dense_2', 'dense_3')
Q_LAYERS = ('dense', 'dense_1', 'dense_2')


def main_var_names(scope='main'):
    """tf.layers.dense variable names in creation order (mlp_actor_critic, mopo.py:311-325)."""
    names = []
    for part, layers in (('pi', PI_LAYERS), ('q1', Q_LAYERS), ('q2', Q_LAYERS)):
        for l in layers:
            names += ['%s/%s/%s/kernel:0' % (scope, part, l), '%s/%s/%s/bias:0' % (scope, part, l)]
    return names


class _Progress:
    def update(self, *a):
        pass

    def set_description(self, *a):
        pass


def sac_case(refs, name, O, A, H, n, seed, steps=3, term_frac=0.2, compact=False):
    """compact: store arrays as float32, gradients of step 0 only and targets of the last step only,
    and of the f64 run only the logs (the H=256 case would otherwise be ~24 MB)."""
    mopo = refs[3]
    rs = np.random.RandomState(seed)
    params = osac.init_params(O, A, H, seed=seed + 1, dtype=np.float64)
    out = dict(O=O, A=A, H=H, n=n, seed=seed, steps=steps)
    for i, prm in enumerate(params):
        out['init%d' % i] = prm.astype(np.float32)
    batches, noises = [], []
    for k in range(steps):
        b = {'observations': rs.normal(size=(n, O)).astype(np.float32),
             'actions': rs.uniform(-0.999, 0.999, size=(n, A)).astype(np.float32),
             'next_observations': rs.normal(size=(n, O)).astype(np.float32),
             'rewards': rs.normal(size=(n, 1)).astype(np.float32),
             'terminals': rs.uniform(size=(n, 1)) < term_frac}
        batches.append(b)
        noises.append([rs.normal(size=(1, n, A)).astype(np.float32) for _ in range(4)])   # 4 tf.random_normal calls per build
        for kk, v in b.items():
            out['b%d_%s' % (k, kk)] = v
        for j in range(4):
            out['b%d_noise%d' % (k, j)] = noises[-1][j].astype(np.float32)
    names = main_var_names()
    st = np.float32 if compact else np.float64
    for tag, dt in (('f32', torch.float32), ('f64', torch.float64)):
        state = {nm: params[i] for i, nm in enumerate(names)}
        state['log_alpha:0'] = np.float64(0.0)
        # the graph is evaluated eagerly at build time, so the target variables must already hold
        # what target_init (mopo.py:449-450, run at the end of _build) gives them before the first
        # training step: the main weights
        for nm in main_var_names('target'):
            state[nm] = state[nm.replace('target/', 'main/', 1)].copy()
        for k in range(steps):
            S = tfstub.reset(dt)
            S.init_values.update(state)
            b = batches[k]
            S.feeds.update({'observation': b['observations'][None], 'next_observation': b['next_observations'][None],
                            'actions': b['actions'][None], 'rewards': b['rewards'][None],
                            'terminals': b['terminals'][None].astype(np.float64), 'iteration': np.int64(k)})
            S.noise = [x for x in noises[k]]
            m = object.__new__(mopo.MOPO)
            m._observation_shape, m._action_shape, m.gru_state_dim = (O,), (A,), 256
            m._store_extra_policy_info, m.adapt = False, False
            m.network_kwargs = {'hidden_sizes': [H, H], 'activation': tfstub.relu, 'output_activation': None}
            m._reward_scale, m._discount, m._tau = 1.0, 0.99, 5e-3       # base.py / mopo.py defaults
            m._Q_lr = m._policy_lr = 3e-4
            m._target_entropy, m._reparameterize, m._action_prior = -3, True, 'uniform'
            m._target_update_interval = 1
            m._training_progress = _Progress()
            sess = m._session = tfstub.Session()
            if k > 0:   # target_init runs inside _build (mopo.py:466); later steps keep the targets
                orig = tfstub.Session._fetch

                def _fetch(self, f, orig=orig):
                    if isinstance(f, tfstub.Op) and f is getattr(m, 'target_init', None):
                        return None
                    return orig(self, f)
                sess._fetch = types.MethodType(_fetch, sess)
            with redirect_stdout(io.StringIO()):
                mopo.MOPO._build(m)
            assert k == 0 or not S.missing_init, S.missing_init
            if k == 0:
                hidden = np.zeros((n, 256))
                pi_act, _ = mopo.MOPO.get_action_meta(m, b['observations'], hidden, deterministic=False)
                mu_act, _ = mopo.MOPO.get_action_meta(m, b['observations'], hidden, deterministic=True)
                out['actor_pi_' + tag], out['actor_mu_' + tag] = pi_act, mu_act
            logs = mopo.MOPO._do_training(m, k, b)
            for kk, v in logs.items():
                out['b%d_log_%s_%s' % (k, kk.replace('/', '.'), tag)] = np.float64(v)
            # gradients per optimizer (pi, q1 on q1_loss, q2 on q2_loss, alpha), pre-step
            for opt in S.optimizers:
                if opt.grads is None:
                    continue
                key = opt.grads[0][1].name.split('/')[0] if opt.name == 'Adam' else 'alpha'
                if key == 'main':
                    key = opt.grads[0][1].name.split('/')[1]
                for j, (g, v) in enumerate(opt.grads):
                    if not compact or (k == 0 and tag == 'f32'):
                        out['b%d_grad_%s%d_%s' % (k, key, j, tag)] = g.numpy().astype(st)
            state = {v.name: tfstub.u(v).detach().numpy().astype(np.float64) for v in S.variables}
            if k == 0:
                pairs = [p for op in m.target_update.deps for p in op.pairs]
                out['polyak_pairs'] = np.array(['%s<-%s:%g' % p for p in pairs])
            for i, nm in enumerate(names):
                if compact and tag == 'f64':   # the f64 oracle is pinned in full by the small case
                    break
                out['b%d_post%d_%s' % (k, i, tag)] = state[nm].astype(st)
                if not compact or k + 1 == steps:
                    out['b%d_target%d_%s' % (k, i, tag)] = state[nm.replace('main/', 'target/', 1)].astype(st)
            out['b%d_log_alpha_%s' % (k, tag)] = state['log_alpha:0']
            used = tfstub.S.noise_used
            assert len(used) == 4
    np.savez_compressed(os.path.join(HERE, 'ref_sac_%s.npz' % name), **out)


def bnn_save_case(refs, E=3, H=32, seed=41, smv=True, dirname='ref_save'):
    """BNN.save (bnn.py:559-592) executed from the reference on a stand-in model: the structure files
    ('<name>_<t>.nns', '<name>_<t>_var.nns': one repr(FC) per line) and the '.mat' of nonoptvars +
    optvars, written to tests/golden/ref_save/."""
    utils, fc, bnn, _ = refs
    O, A = 17, 6
    rs = np.random.RandomState(seed)
    p = obnn.init_params(E, O, A, hidden=H, seed=seed, smv=smv, inputs=rs.normal(size=(200, O + A)))
    obj = build_bnn(refs, p, E, O, A, H, smv, torch.float32)
    obj.finalized, obj.name, obj.model_dir = True, 'BNN', None
    obj.nonoptvars = obj.scaler.get_vars()
    obj.optvars = []
    for layer in obj.layers + obj.var_layers:
        obj.optvars.extend(layer.get_vars())
    obj.optvars += [obj.max_logvar, obj.min_logvar]
    obj._sess = tfstub.Session()   # BNN.sess is a property over _sess
    out = os.path.join(HERE, dirname)
    os.makedirs(out, exist_ok=True)
    bnn.BNN.save(obj, out, 0)
    # the inputs / outputs of one predict with these weights, for the load test
    x = rs.normal(size=(32, O + A)).astype(np.float32)
    xin = tfstub.w(torch.as_tensor(x))
    mean, var = bnn.BNN._compile_outputs(obj, xin)
    np.savez_compressed(os.path.join(out, 'predict.npz'), x=x, mean=tfstub.u(mean).detach().numpy(),
                        var=tfstub.u(var).detach().numpy())


def main(argv):
    refs = load_reference()
    if argv[1:] == ['joint']:   # the joint-head (separate_mean_var=False) training and save cases only
        bnn_loss_case(refs, 'E3_H32_joint', 3, 32, 40, 22, smv=False)
        bnn_save_case(refs, seed=42, smv=False, dirname='ref_save_joint')
        print('ok')
        return
    bnn_save_case(refs)
    # ensemble forward: the headline shapes and the stress shape (weights regenerated from the seed
    # for the large ones), the joint-head branch, f64 inputs (the rollout feeds f64 next_obs)
    bnn_forward_case(refs, 'E7_H200', 7, 200, 96, True, 11, store_weights=False)
    bnn_forward_case(refs, 'E7_H64', 7, 64, 64, True, 12, store_weights=True)
    bnn_forward_case(refs, 'E7_H64_joint', 7, 64, 64, False, 13, store_weights=True)
    bnn_forward_case(refs, 'E32_H400', 32, 400, 40, True, 14, store_weights=False)
    bnn_forward_case(refs, 'E32_H64_x64', 32, 64, 48, True, 15, store_weights=False, x_f64=True)
    bnn_loss_case(refs, 'E3_H32', 3, 32, 40, 21)
    sac_case(refs, 'H256', 17, 6, 256, 256, 31, steps=2, compact=True)
    sac_case(refs, 'H32', 11, 3, 32, 64, 32, term_frac=0.5)
    print('ok')


if __name__ == '__main__':
    main(sys.argv)
