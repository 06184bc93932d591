"""Probabilistic ensemble (BNN) host mirror over libmopo_hip.

Mirrors the reference surface used on the hot path:
  * ``construct_model(...)``                 mopo/models/constructor.py:7-43
  * ``BNN.predict(inputs, factored=True)``   mopo/models/bnn.py:508-546
  * ``BNN.random_inds(batch_size)``          mopo/models/bnn.py:342-344
  * ``BNN.load_params`` / ``.mat`` layout    mopo/models/bnn.py:276-281, 588-592
  * ``BNN.train(inputs, targets, ...)``      mopo/models/bnn.py:369-503 (+ validate :351-362)
  * ``num_nets``, ``num_elites``, ``_model_inds``, ``scaler.cached_mu/cached_sigma``
The forward runs in the HIP kernel ``bnn_fwd_kernel`` (csrc/bnn.hip); training steps in
csrc/bnn_train.hip (the loop control and numpy's RNG stream stay here, in the reference's order).
There is no CPU path.
"""
import ctypes as C
import itertools
import os
import time
from collections import OrderedDict

import numpy as np

from . import _lib as L

# ensemble-forward arithmetic (mopo_bnn_create dtype): 'fp32' f32 MFMA; 'bf16' bf16 operands;
# 'bf16x3' / 'bf16x6' f32 operands split into 2 / 3 round-to-nearest bf16 parts (3 / 6 bf16 MFMAs per
# product, f32 accumulate): bf16x6's split is EXACT (x0 + x1 + x2 == x for 2^-100 <= |x| < 2^127,
# csrc/mlp_tile.h split_bf16, tests/test_split.py) and its 3 dropped products total <= 2^-23 |x w|;
# bf16x3 keeps ~17 significand bits; 'f16x3' f32 operands as 2 fp16 parts under power-of-two scales
# (3 f16 MFMAs per product, ~22-bit operands, the dropped product <= 2^-22 |x w|).
_DTYPES = {'fp32': 0, 'bf16': 1, 'bf16x3': 2, 'bf16x6': 3, 'f16x3': 4}
DTYPES = tuple(_DTYPES)
# what MOPO (and so `mopo run_local` and bench.py's headline) runs unless told otherwise: the exact
# bf16x6 split -- the reference's f32 operands exactly, 6 bf16 MFMA products per f32 product, f32
# accumulate, held to the fp32 parity tolerances over whole rollouts (tests/test_gpu_rollout.py) -- at
# ~1.5x the exact-f32 MFMA kernel's rate (the f32 MFMA peak caps that one below it).  bf16x6 has no H > 256
# form: there the default is 'fp32' (default_ensemble_dtype).  'f16x3' (~22-bit operands, ~2.4x fp32) and
# 'fp32' stay selectable everywhere (ensemble_dtype).
DEFAULT_ENSEMBLE_DTYPE = 'bf16x6'


def default_ensemble_dtype(hidden_dim):
    """The product default for an ensemble of this width: bf16x6 up to H = 256, exact-f32 MFMA above."""
    return DEFAULT_ENSEMBLE_DTYPE if int(hidden_dim) <= 256 else 'fp32'

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


# ---- structure files ('<name>.nns', bnn.py:559-582 / 594-625): one repr(FC) per line, fc.py:47-51
WEIGHT_DECAYS = (0.000025, 0.00005, 0.000075, 0.000075, 0.0001)   # constructor.py:30-34
VAR_WEIGHT_DECAY = 0.0001                                         # constructor.py:36


def fc_repr(output_dim, input_dim, activation, weight_decay, ensemble_size):
    """FC.__repr__ (fc.py:47-51)."""
    return 'FC(output_dim={!r}, input_dim={!r}, activation={!r}, weight_decay={!r}, ensemble_size={!r})'.format(
        output_dim, input_dim, activation, weight_decay, ensemble_size)


def structure_lines(E, obs_dim, act_dim, hidden):
    """The smv structure construct_model builds (constructor.py:28-36): (mean-layer lines, var-layer lines)."""
    IN, D = obs_dim + act_dim, obs_dim + 1
    dims = [IN] + [hidden] * N_HIDDEN
    mean = [fc_repr(hidden, dims[i], 'swish', WEIGHT_DECAYS[i], E) for i in range(N_HIDDEN)]
    mean.append(fc_repr(D, hidden, None, WEIGHT_DECAYS[N_HIDDEN], E))
    return mean, [fc_repr(D, hidden, None, VAR_WEIGHT_DECAY, E)]


def structure_files(E, obs_dim, act_dim, hidden, smv):
    """BNN.save's structure files (bnn.py:572-585) as {suffix: text}: smv writes '' (mean layers)
    and '_var'; the joint branch as written writes the halved last layer (output D, activation
    None) after EVERY hidden layer -- a file the reference's own _load_structure cannot read back
    (nor load_model=True here)."""
    mean, var = structure_lines(E, obs_dim, act_dim, hidden)
    files = {'': mean, '_var': var} if smv else {'': [ln for hid in mean[:-1] for ln in (hid, mean[-1])]}
    return {k: ''.join('%s\n' % ln for ln in v) for k, v in files.items()}


def parse_structure(path):
    """BNN._load_structure's line parser (bnn.py:594-625): a list of FC keyword dicts."""
    layers = []
    with open(path) as f:
        for line in f:
            kw = dict(a.split('=') for a in line[3:-2].split(', '))
            layers.append({'input_dim': int(kw['input_dim']), 'output_dim': int(kw['output_dim']),
                           'weight_decay': None if kw['weight_decay'] == 'None' else float(kw['weight_decay']),
                           'activation': None if kw['activation'] == 'None' else kw['activation'][1:-1],
                           'ensemble_size': int(kw['ensemble_size'])})
    return layers


def _smv_shapes(shapes):
    """.mat shapes of the smv layout for a (joint or smv) list of shapes."""
    if len(shapes) == 16:
        return shapes
    W, b = shapes[10], shapes[11]
    D = W[-1] // 2
    half_w, half_b = W[:-1] + (D,), b[:-1] + (D,)
    return shapes[:10] + [half_w, half_b, half_w, half_b] + shapes[12:]


def _joint_to_smv(mats):
    """14 joint arrays -> 16 smv arrays: head [E, H, 2D] split into mean / log-var columns."""
    W, b = mats[10], mats[11]
    D = W.shape[-1] // 2
    c = np.ascontiguousarray
    return list(mats[:10]) + [c(W[..., :D]), c(b[..., :D]), c(W[..., D:]), c(b[..., D:])] + list(mats[12:])


def _smv_to_joint(mats):
    return list(mats[:10]) + [np.concatenate([mats[10], mats[12]], -1),
                              np.concatenate([mats[11], mats[13]], -1)] + list(mats[14:])


class BNN:
    """Device-resident probabilistic ensemble (smv or joint head), fp32 or bf16 forward."""

    def __init__(self, params):
        self.name = params.get('name', 'BNN')
        self.model_dir = params.get('model_dir', None)
        if params.get('load_model', False):   # bnn.py:72-80: the structure file fixes the shapes
            if self.model_dir is None:
                raise ValueError('Cannot load model without providing model directory.')
            layers = parse_structure(os.path.join(self.model_dir, '%s.nns' % self.name))
            if len(layers) != N_HIDDEN + 1 or layers[0]['activation'] != 'swish':
                raise ValueError('unsupported structure in %s.nns (expected 4 swish FC layers + a head)' % self.name)
            D, IN = layers[-1]['output_dim'], layers[0]['input_dim']
            params = dict(params, num_networks=layers[0]['ensemble_size'], hidden_dim=layers[0]['output_dim'],
                          obs_dim=D - 1, act_dim=IN - (D - 1))
        self.num_nets = int(params.get('num_networks', 1))
        self.num_elites = int(params['num_elites'])
        self.separate_mean_var = bool(params.get('separate_mean_var', False))
        self.deterministic = bool(params.get('deterministic', False))
        self.obs_dim = int(params['obs_dim'])
        self.act_dim = int(params['act_dim'])
        self.hidden_dim = int(params.get('hidden_dim', 200))
        self.dtype = params.get('dtype', 'fp32')
        if self.dtype not in _DTYPES:
            raise ValueError('dtype must be one of %s, got %r' % (sorted(_DTYPES), self.dtype))
        self.model_loaded = False
        self._model_inds = list(range(min(self.num_elites, self.num_nets)))   # set by _end_train
        self._mats = None
        h = C.c_void_p()
        L.check(L.lib().mopo_bnn_create(C.byref(h), self.num_nets, self.obs_dim, self.act_dim, self.hidden_dim,
                                        int(self.separate_mean_var), _DTYPES[self.dtype]))
        self._h = h
        if params.get('load_model', False):
            self.load_params()                                                     # finalize: bnn.py:266-267

    def __del__(self):
        t = getattr(self, '_train_h', None)
        if t is not None and t.value:
            L.lib().mopo_bnn_train_destroy(t)
            self._train_h = None
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
        return [m.copy() for m in self._require_mats('get_params')]

    # -- packed device image (multi-GPU broadcast) ------------------------------------------------------
    def packed_nbytes(self):
        n = int(L.lib().mopo_bnn_packed_bytes(self._h))
        if n < 0:
            raise RuntimeError('BNN: parameters not set')
        return n

    def export_packed(self, out=None, stream=None):
        """The packed device parameters as a uint8 cuda tensor (mopo_bnn_packed_copy)."""
        import torch
        n = self.packed_nbytes()
        out = torch.empty(n, dtype=torch.uint8, device='cuda') if out is None else out
        L.check(L.lib().mopo_bnn_packed_copy(self._h, 0, L.ptr(out), n, L.stream_ptr(stream)))
        return out

    def import_packed(self, buf, stream=None, mats=None, holdout_losses=None):
        """Load a packed image exported by a handle of the same shapes and dtype.  ``mats``: the
        sender's .mat arrays (``flat_params``) -- with them this handle's host state (``get_params``,
        ``scaler``, ``save``, ``train``, ``validate``) describes the imported weights; without them
        the host state is dropped and those methods raise."""
        L.check(L.lib().mopo_bnn_packed_copy(self._h, 1, L.ptr(buf), int(buf.numel()), L.stream_ptr(stream)))
        self._mats = None
        self.scaler = None
        self._holdout_losses = None if holdout_losses is None else np.asarray(holdout_losses, np.float64)
        if mats is not None:
            mats = [np.ascontiguousarray(np.asarray(m, np.float32)) for m in mats]
            shapes = [m.shape for m in self._mat_shapes()]
            if [m.shape for m in mats] != shapes:
                raise ValueError('import_packed: .mat arrays do not match this ensemble')
            self._mats = mats
            self.scaler = _Scaler(mats[0], mats[1])

    def _mat_shapes(self):
        """Zero arrays of the .mat shapes (set_params' expectation)."""
        E, IN, H, D = self.num_nets, self.obs_dim + self.act_dim, self.hidden_dim, self.obs_dim + 1
        exp = [(1, IN), (1, IN)]
        dims = [IN] + [H] * N_HIDDEN + [D if self.separate_mean_var else 2 * D]
        for i in range(len(dims) - 1):
            exp += [(E, dims[i], dims[i + 1]), (E, 1, dims[i + 1])]
        if self.separate_mean_var:
            exp += [(E, H, D), (E, 1, D)]
        exp += [(1, D), (1, D)]
        return [np.zeros(s, np.float32) for s in exp]

    def flat_params(self):
        """The .mat arrays concatenated (f32), the broadcast form of ``import_packed(mats=...)``."""
        return np.concatenate([m.ravel() for m in self._require_mats('flat_params')])

    def unflatten_params(self, flat):
        out, off = [], 0
        for z in self._mat_shapes():
            out.append(np.asarray(flat[off:off + z.size], np.float32).reshape(z.shape))
            off += z.size
        if off != len(flat):
            raise ValueError('unflatten_params: %d values for %d parameters' % (len(flat), off))
        return out

    def _require_mats(self, what):
        if self._mats is None:
            raise RuntimeError('BNN.%s: this handle holds only a packed device image (import_packed without '
                               'mats); the .mat arrays live on the broadcasting rank' % what)
        return self._mats

    def load_params(self, path=None):
        """bnn.py:276-281: loadmat('<model_dir>/<name>.mat'), keys '0'..'15'."""
        from scipy.io import loadmat
        path = path or os.path.join(self.model_dir, '%s.mat' % self.name)
        d = loadmat(path)
        n = 16 if self.separate_mean_var else 14
        self.set_params([d[str(i)] for i in range(n)])
        self.model_loaded = True

    def save(self, savedir, timestep):
        """BNN.save (bnn.py:559-592): '<name>_<t>.nns' (+ '<name>_<t>_var.nns' for smv; the
        structure, one repr(FC) per line, ``structure_files``) and '<name>_<t>.mat' (keys '0'..'15',
        joint '0'..'13' = nonoptvars + optvars)."""
        from scipy.io import savemat
        self._require_mats('save')
        savedir = self.model_dir if savedir is None else savedir
        files = structure_files(self.num_nets, self.obs_dim, self.act_dim, self.hidden_dim, self.separate_mean_var)
        for suffix, text in files.items():   # joint: one file, the reference's interleaved text
            with open(os.path.join(savedir, '{}_{}{}.nns'.format(self.name, timestep, suffix)), 'w+') as f:
                f.write(text)
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

    # -- training (bnn.py:369-503) ---------------------------------------------------------------------
    def _trainer(self, batch_size, max_eval):
        t = getattr(self, '_train_h', None)
        if t is None or self._train_dims != (batch_size, max_eval):
            if t is not None:
                L.lib().mopo_bnn_train_destroy(t)
            t = C.c_void_p()
            L.check(L.lib().mopo_bnn_train_create(C.byref(t), self.num_nets, self.obs_dim, self.act_dim,
                                                  self.hidden_dim, int(batch_size), int(max_eval), 1e-3))
            self._train_h, self._train_dims = t, (batch_size, max_eval)
        return t

    def _train_params(self, t, mats=None):
        """Move the .mat arrays into / out of the trainer.  The trainer holds the smv layout; a
        joint head (bnn.py:183-189) goes in as its mean / log-var column halves, which carry the
        same 0.0001 decay (constructor.py:34-36), so the loss and every Adam update are the
        joint model's (oracle: tests/test_oracle_train.py::test_joint_head_equals_split_heads)."""
        if mats is not None:
            mats = mats if self.separate_mean_var else _joint_to_smv(mats)
            arr = (C.c_void_p * 16)(*[m.ctypes.data for m in mats])
            L.check(L.lib().mopo_bnn_train_set_params(t, arr))
            return None
        out = [np.empty(s, np.float32) for s in _smv_shapes([z.shape for z in self._mat_shapes()])]
        arr = (C.c_void_p * 16)(*[m.ctypes.data for m in out])
        L.check(L.lib().mopo_bnn_train_get_params(t, arr))
        return out if self.separate_mean_var else _smv_to_joint(out)

    def train(self, inputs, targets, batch_size=32, max_epochs=None, max_epochs_since_update=5,
              hide_progress=False, holdout_ratio=0.0, max_logging=1000, max_grad_updates=None, timer=None,
              max_t=None, permuted=False):
        """BNN.train (bnn.py:369-503).  ``inputs`` [N, O+A] / ``targets`` [N, O+1]: numpy (the
        reference API) or cuda tensors.  ``permuted=True``: the rows are already in
        ``np.random.permutation`` order (the permutation was drawn by the caller, as
        ``MOPO._train_model`` does when it formats the device pool in that order)."""
        import torch
        E = self.num_nets
        N = int(inputs.shape[0])
        num_holdout = min(int(N * holdout_ratio), max_logging)
        if not permuted:
            permutation = np.random.permutation(N)                                  # bnn.py:391-394
            if isinstance(inputs, np.ndarray):
                inputs, targets = inputs[permutation], targets[permutation]
            else:
                p = torch.from_numpy(permutation).to(inputs.device)
                inputs, targets = inputs[p], targets[p]
        dev = 'cuda'

        def dt(x):
            if isinstance(x, np.ndarray):
                return torch.from_numpy(np.ascontiguousarray(x, np.float32)).to(dev)
            return x.to(dev, torch.float32).contiguous()

        x_all, y_all = dt(inputs), dt(targets)
        hold_x, hold_y = x_all[:num_holdout], y_all[:num_holdout]
        x, y = x_all[num_holdout:], y_all[num_holdout:]
        n = N - num_holdout
        t = self._trainer(batch_size, max(max_logging, 1))
        self._train_params(t, self._mats)
        L.check(L.lib().mopo_bnn_train_fit_scaler(t, L.ptr(x), n, None))          # bnn.py:399-400
        # np.random's draws come from the native MT19937 replica (the global stream is moved in and out,
        # so it advances exactly as the reference's), written straight into pinned buffers kept across
        # calls: numpy's randint + a pageable copy held the first epoch's launch back ~8 ms per call
        mt = self._host_rng()
        if getattr(self, '_pinned_free', None) is not None:
            self._pinned_free.synchronize()              # the previous call's copies out of the buffers
        idxs_h = self._pinned('idxs', E * n, torch.int32)
        numpy_draws = os.environ.get('MOPO_TRAIN_NUMPY_DRAWS') == '1'               # A/B knob
        if numpy_draws:
            idxs_h.numpy()[:] = np.random.randint(n, size=E * n)
        else:
            mt.sync_from_numpy()
            mt.randint(0, n, [E, n], out=idxs_h.numpy())                            # bnn.py:402
            mt.sync_to_numpy()
        idxs = torch.empty(E * n, dtype=torch.int32, device=dev)
        idxs.copy_(idxs_h, non_blocking=True)
        self._start_train()
        losses_d = torch.empty(E, dtype=torch.float32, device=dev)
        break_train, grad_updates, epoch = False, 0, 0
        self._max_epochs_since_update = max_epochs_since_update
        # the shuffle uniforms are drawn on the host while the epoch's steps run and reach the device by one
        # DMA from a pinned buffer queued behind them (a pageable copy was staged in chunks by the host and
        # left the GPU idle ~5 ms per epoch); the event keeps the next draw from overwriting a pending copy
        keys_h = self._pinned('keys', E * n, torch.float64)
        keys_hn = keys_h.numpy()
        keys = torch.empty(E * n, dtype=torch.float64, device=dev)
        copied = torch.cuda.Event()
        copied.record()
        # the keys' copy and sort run on a side stream beside the epoch's steps (which leave CUs idle);
        # only the apply to idxs waits for the epoch (mopo_bnn_train_shuffle_async)
        side = None if os.environ.get('MOPO_TRAIN_SHUFFLE_SIDE') == '0' else self._side_stream()
        if side is not None:
            keys.record_stream(side)
            # the block may have been in use on the current stream until just now: the side stream's first
            # write of it must wait for that (record_stream only protects the free)
            side.wait_stream(torch.cuda.current_stream())
        t0 = time.time()
        for epoch in (range(max_epochs) if max_epochs is not None else itertools.count()):
            L.check(L.lib().mopo_bnn_train_epoch(t, L.ptr(x), L.ptr(y), L.ptr(idxs), n, int(batch_size), None))
            grad_updates += int(np.ceil(n / batch_size))
            copied.synchronize()
            if numpy_draws:
                keys_hn[:] = np.random.uniform(size=E * n)
            else:
                mt.sync_from_numpy()
                mt.random_sample([E, n], out=keys_hn)                               # shuffle_rows :385-387
                mt.sync_to_numpy()
            copied = torch.cuda.Event()
            if side is None:
                keys.copy_(keys_h, non_blocking=True)
                copied.record()
                L.check(L.lib().mopo_bnn_train_shuffle(t, L.ptr(idxs), L.ptr(keys), n, None))
            else:
                with torch.cuda.stream(side):
                    keys.copy_(keys_h, non_blocking=True)
                    copied.record(side)
                L.check(L.lib().mopo_bnn_train_shuffle_async(t, L.ptr(idxs), L.ptr(keys), n,
                                                             L.stream_ptr(side), None))
            if not hide_progress and holdout_ratio >= 1e-12 and num_holdout > 0:
                L.check(L.lib().mopo_bnn_train_eval_mse(t, L.ptr(hold_x), L.ptr(hold_y), None, num_holdout,
                                                        L.ptr(losses_d), None))
                holdout_losses = losses_d.cpu().numpy().astype(np.float64)
                break_train = self._save_best(t, epoch, holdout_losses)
            if break_train or (max_grad_updates and grad_updates > max_grad_updates):
                break
            if max_t and time.time() - t0 > max_t:
                break
        self._pinned_free = copied
        L.check(L.lib().mopo_bnn_train_restore(t, None))                           # _set_state :491
        if num_holdout > 0:
            L.check(L.lib().mopo_bnn_train_eval_mse(t, L.ptr(hold_x), L.ptr(hold_y), None, num_holdout,
                                                    L.ptr(losses_d), None))
            holdout_losses = losses_d.cpu().numpy().astype(np.float64)
        else:
            holdout_losses = np.full(E, np.nan)
        self._end_train(holdout_losses)
        self.set_params(self._train_params(t))                                     # repack for inference
        self._train_epochs, self._train_grad_updates = epoch + 1, grad_updates
        val_loss = np.sort(holdout_losses)[:self.num_elites].mean()
        return OrderedDict({'val_loss': val_loss})

    def _host_rng(self):
        mt = getattr(self, '_mt', None)
        if mt is None:
            from .rng import LegacyRandomState
            mt = self._mt = LegacyRandomState(0)
        return mt

    def _side_stream(self):
        import torch
        st = getattr(self, '_side', None)
        if st is None:
            st = self._side = torch.cuda.Stream()
        return st

    def _pinned(self, name, n, dtype):
        """A pinned host buffer of n elements kept across train() calls (pinning costs ~ms per MB)."""
        import torch
        bufs = self.__dict__.setdefault('_pinned_bufs', {})
        b = bufs.get(name)
        if b is None or b.numel() < n or b.dtype != dtype:
            b = bufs[name] = torch.empty(n, dtype=dtype, pin_memory=True)
        return b[:n]

    def _start_train(self):                                                         # bnn.py:324-327
        self._snapshots = {i: (None, 1e10) for i in range(self.num_nets)}
        self._epochs_since_update = 0

    def _save_best(self, t, epoch, holdout_losses):                                  # bnn.py:301-322
        updated = []
        for i in range(len(holdout_losses)):
            current = holdout_losses[i]
            _, best = self._snapshots[i]
            if (best - current) / best > 0.01:
                self._snapshots[i] = (epoch, current)
                updated.append(i)
        if updated:                                                                 # one launch
            arr = (C.c_int * len(updated))(*updated)
            L.check(L.lib().mopo_bnn_train_snapshot_members(t, arr, len(updated), None))
        self._epochs_since_update = 0 if updated else self._epochs_since_update + 1
        return self._epochs_since_update > self._max_epochs_since_update

    def _end_train(self, holdout_losses):                                            # bnn.py:329-332
        self._model_inds = np.argsort(holdout_losses)[:self.num_elites].tolist()
        self._holdout_losses = holdout_losses

    def validate(self, inputs, targets):
        """bnn.py:351-362: mean of the num_elites smallest per-member mse losses."""
        import torch
        t = self._trainer(*getattr(self, '_train_dims', (256, max(int(inputs.shape[0]), 1))))
        self._train_params(t, self._mats)
        x = torch.from_numpy(np.ascontiguousarray(inputs, np.float32)).cuda()
        y = torch.from_numpy(np.ascontiguousarray(targets, np.float32)).cuda()
        out = torch.empty(self.num_nets, dtype=torch.float32, device='cuda')
        L.check(L.lib().mopo_bnn_train_eval_mse(t, L.ptr(x), L.ptr(y), None, int(x.shape[0]), L.ptr(out), None))
        return np.sort(out.cpu().numpy())[:self.num_elites].mean()

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
