"""Probabilistic ensemble (BNN) host mirror over libmopo_hip.

Mirrors the reference surface used on the hot path:
  * ``construct_model(...)``                 mopo/models/constructor.py:7-43
  * ``BNN.predict(inputs, factored=True)``   mopo/models/bnn.py:508-546
  * ``BNN.random_inds(batch_size)``          mopo/models/bnn.py:342-344
  * ``BNN.load_params`` / ``.mat`` layout    mopo/models/bnn.py:276-281, 588-592
  * ``num_nets``, ``num_elites``, ``_model_inds``, ``scaler.cached_mu/cached_sigma``
The forward runs in the HIP kernel ``bnn_fwd_kernel`` (csrc/bnn.hip); there is no CPU path.
Ensemble training (BNN.train, bnn.py:369-503) is a later-round item.
"""
import ctypes as C
import os

import numpy as np

from . import _lib as L

N_HIDDEN = 4


class _Scaler:
    def __init__(self, mu, sigma):
        self.cached_mu, self.cached_sigma = mu, sigma


def tf_init_params(E, obs_dim, act_dim, hidden, separate_mean_var=True, rng=None):
    """Initial values of the reference variables: truncated_normal(1/(2 sqrt(in))) weights,
    zero biases (fc.py:145-154), max/min log-var 0.5 / -10 (bnn.py:196-213), scaler (0, 1)."""
    rng = rng or np.random.RandomState()
    IN, D = obs_dim + act_dim, obs_dim + 1

    def tn(shape, std):
        w = rng.normal(size=shape) * std
        bad = np.abs(w) > 2 * std
        while bad.any():
            w[bad] = rng.normal(size=int(bad.sum())) * std
            bad = np.abs(w) > 2 * std
        return w.astype(np.float32)

    dims = [IN] + [hidden] * N_HIDDEN + [D if separate_mean_var else 2 * D]
    arrs = [np.zeros([1, IN], np.float32), np.ones([1, IN], np.float32)]
    for i in range(len(dims) - 1):
        arrs += [tn((E, dims[i], dims[i + 1]), 1 / (2 * np.sqrt(dims[i]))), np.zeros((E, 1, dims[i + 1]), np.float32)]
    if separate_mean_var:
        arrs += [tn((E, hidden, D), 1 / (2 * np.sqrt(hidden))), np.zeros((E, 1, D), np.float32)]
    arrs += [np.full([1, D], 0.5, np.float32), np.full([1, D], -10.0, np.float32)]
    return arrs


class BNN:
    """Device-resident probabilistic ensemble (smv or joint head), fp32 or bf16 forward."""

    def __init__(self, params):
        self.name = params.get('name', 'BNN')
        self.model_dir = params.get('model_dir', None)
        self.num_nets = int(params.get('num_networks', 1))
        self.num_elites = int(params['num_elites'])
        self.separate_mean_var = bool(params.get('separate_mean_var', False))
        self.deterministic = bool(params.get('deterministic', False))
        self.obs_dim = int(params['obs_dim'])
        self.act_dim = int(params['act_dim'])
        self.hidden_dim = int(params.get('hidden_dim', 200))
        self.dtype = params.get('dtype', 'fp32')
        self.model_loaded = False
        self._model_inds = list(range(min(self.num_elites, self.num_nets)))   # set by _end_train
        self._mats = None
        h = C.c_void_p()
        L.check(L.lib().mopo_bnn_create(C.byref(h), self.num_nets, self.obs_dim, self.act_dim, self.hidden_dim,
                                        int(self.separate_mean_var), 0 if self.dtype == 'fp32' else 1))
        self._h = h

    def __del__(self):
        h = getattr(self, '_h', None)
        if h is not None and h.value:
            L.lib().mopo_bnn_destroy(h)
            self._h = None

    @property
    def handle(self):
        return self._h

    @property
    def is_probabilistic(self):
        return True

    # -- parameters ---------------------------------------------------------------------------------
    def set_params(self, mats):
        """``mats``: the 16 (smv) / 14 arrays of the reference .mat file, keys '0'..'15'."""
        mats = [np.ascontiguousarray(np.asarray(m, np.float32)) for m in mats]
        n = 16 if self.separate_mean_var else 14
        if len(mats) != n:
            raise ValueError('expected %d parameter arrays, got %d' % (n, len(mats)))
        E, IN, H, D = self.num_nets, self.obs_dim + self.act_dim, self.hidden_dim, self.obs_dim + 1
        exp = [(1, IN), (1, IN)]
        dims = [IN] + [H] * N_HIDDEN + [D if self.separate_mean_var else 2 * D]
        for i in range(len(dims) - 1):
            exp += [(E, dims[i], dims[i + 1]), (E, 1, dims[i + 1])]
        if self.separate_mean_var:
            exp += [(E, H, D), (E, 1, D)]
        exp += [(1, D), (1, D)]
        for i, (m, s) in enumerate(zip(mats, exp)):
            if m.shape != s:
                raise ValueError('parameter %d has shape %s, expected %s' % (i, m.shape, s))
        arr = (C.c_void_p * n)(*[m.ctypes.data for m in mats])
        L.check(L.lib().mopo_bnn_set_params(self._h, arr, n))
        self._mats = mats
        self.scaler = _Scaler(mats[0], mats[1])
        return self

    def get_params(self):
        return [m.copy() for m in self._mats]

    def load_params(self, path=None):
        """bnn.py:276-281: loadmat('<model_dir>/<name>.mat'), keys '0'..'15'."""
        from scipy.io import loadmat
        path = path or os.path.join(self.model_dir, '%s.mat' % self.name)
        d = loadmat(path)
        n = 16 if self.separate_mean_var else 14
        self.set_params([d[str(i)] for i in range(n)])
        self.model_loaded = True

    def save(self, savedir, timestep):
        """bnn.py:588-592 parameter file ('<name>_<timestep>.mat', keys '0'..'15')."""
        from scipy.io import savemat
        savemat(os.path.join(savedir, '{}_{}.mat'.format(self.name, timestep)),
                {str(i): m for i, m in enumerate(self._mats)})

    # -- inference ----------------------------------------------------------------------------------
    def predict(self, inputs, factored=True, stream=None):
        """BNN.predict for 2-D inputs (bnn.py:530-541).  numpy in -> numpy out; torch cuda in -> torch out."""
        import torch
        is_np = isinstance(inputs, np.ndarray)
        x = torch.from_numpy(np.ascontiguousarray(inputs)).cuda() if is_np else inputs.contiguous()
        if x.dim() != 2:
            raise ValueError('BNN.predict: only 2-D inputs are supported on the device path')
        if x.dtype not in (torch.float32, torch.float64):
            x = x.float()
        B = x.shape[0]
        E, D = self.num_nets, self.obs_dim + 1
        mean = torch.empty((E, B, D), dtype=torch.float32, device=x.device)
        var = torch.empty_like(mean)
        L.check(L.lib().mopo_bnn_predict(self._h, L.ptr(x), int(x.dtype == torch.float64), B, L.ptr(mean),
                                         L.ptr(var), L.stream_ptr(stream)))
        if not factored:  # bnn.py:261-263 / 552-556
            m = mean.mean(0)
            v = var.mean(0) + ((mean - m) ** 2).mean(0)
            mean, var = m, v
        if is_np:
            return mean.cpu().numpy(), var.cpu().numpy()
        return mean, var

    def random_inds(self, batch_size):
        """bnn.py:342-344 (numpy legacy global stream, as the reference)."""
        return np.random.choice(self._model_inds, size=batch_size)

    def set_elites(self, elites):
        self._model_inds = [int(e) for e in elites]

    def __repr__(self):
        return 'BNN(name=%r, num_nets=%d, hidden=%d, smv=%s, dtype=%s)' % (
            self.name, self.num_nets, self.hidden_dim, self.separate_mean_var, self.dtype)


def construct_model(obs_dim=11, act_dim=3, rew_dim=1, hidden_dim=200, num_networks=7, num_elites=5, session=None,
                    model_type='mlp', separate_mean_var=False, name=None, load_dir=None, deterministic=False,
                    dtype='fp32', seed=None):
    """constructor.py:7-43.  Without ``load_dir`` the weights take the reference's initial values."""
    if model_type != 'mlp':
        raise NotImplementedError('only model_type="mlp" is on the accelerated path')
    if rew_dim != 1:
        raise ValueError('rew_dim must be 1')
    name = name or 'BNN'
    model = BNN({'name': name, 'num_networks': num_networks, 'num_elites': num_elites,
                 'separate_mean_var': separate_mean_var, 'deterministic': deterministic,
                 'obs_dim': obs_dim, 'act_dim': act_dim, 'hidden_dim': hidden_dim, 'dtype': dtype,
                 'model_dir': load_dir})
    if load_dir is not None:
        model.load_params()
    else:
        rng = np.random.RandomState(seed) if seed is not None else None
        model.set_params(tf_init_params(num_networks, obs_dim, act_dim, hidden_dim, separate_mean_var, rng))
    return model
