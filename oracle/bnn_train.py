"""Oracle: probabilistic-ensemble training (BNN.train), numpy restatement.  TEST INFRASTRUCTURE ONLY.

Follows (reference xionghuichen/mopo):
  * train loss (not deterministic)     mopo/models/bnn.py:241-249 -- sum over members of
      mean((mu - y)^2 exp(-lv)) + mean(lv), + sum of decays, + 0.01 sum(maxlv) - 0.01 sum(minlv)
  * _compile_losses                    mopo/models/bnn.py:677-701 (mse_loss = inc_var_loss False)
  * joint head (separate_mean_var=False) bnn.py:183-189 (last layer widened to 2D outputs, one
      weight_decay 0.0001 on the whole [H, 2D] matrix), bnn.py:644-654 (mean = out[..., :D],
      log-var raw = out[..., D:])
  * 3-D forward (per-member batches)   mopo/models/fc.py:99-104 (matmul), bnn.py:656-675
  * weight decay                       mopo/models/fc.py:156-157 (wd * tf.nn.l2_loss(W)),
                                       rates constructor.py:30-36
  * optimizer                          constructor.py:41 (tf.train.AdamOptimizer, lr 1e-3), TF1
                                       ApplyAdam semantics (oracle.sac.Adam)
  * train() loop                       bnn.py:369-503: holdout split, scaler fit, bootstrap
                                       indices, minibatches, shuffle_rows, _save_best (287-322),
                                       _set_state (268-285), _end_train (329-332)

The gradients are derived by hand (TF autodiff of the expressions above: softplus' = sigmoid,
swish' = s + x s (1 - s)).  Parity: restatement-pinned (TensorFlow 1.14 is not installed here).
"""
import numpy as np

from .bnn import N_HIDDEN, softplus, scaler_fit
from .sac import Adam

WD = [0.000025, 0.00005, 0.000075, 0.000075, 0.0001]  # constructor.py:30-34 (hidden x4, mean head)
WD_VAR = 0.0001                                        # constructor.py:36 (var head)


def _sigmoid(x):
    one = x.dtype.type(1)
    return one / (one + np.exp(-x))


def _smv(p):
    return p.get('smv', True)


def optvars(p):
    """The optimised variables in bnn.py optvars order (mean layers W,b; var layer W,b (smv only);
    maxlv, minlv) -- bnn.py:199-222."""
    out = []
    for w, b in zip(p['W'], p['b']):
        out += [w, b]
    if _smv(p):
        out += [p['Wv'], p['bv']]
    out += [p['max_logvar'], p['min_logvar']]
    return out


def set_optvars(p, vals):
    q = dict(p)
    q['W'] = [vals[2 * i] for i in range(N_HIDDEN + 1)]
    q['b'] = [vals[2 * i + 1] for i in range(N_HIDDEN + 1)]
    k = 2 * (N_HIDDEN + 1)
    if _smv(p):
        q['Wv'], q['bv'] = vals[k], vals[k + 1]
        k += 2
    q['max_logvar'], q['min_logvar'] = vals[k], vals[k + 1]
    return q


def forward3d(p, X, dtype=np.float64):
    """X: [E, B, IN] raw inputs (each member its own rows).  Returns caches + (mean, lv)."""
    x = X.astype(dtype)
    h = (x - p['mu'].astype(dtype)) / p['sigma'].astype(dtype)
    zs, hs = [], [h]
    for l in range(N_HIDDEN):
        z = np.matmul(h, p['W'][l].astype(dtype)) + p['b'][l].astype(dtype)
        h = z * _sigmoid(z)
        zs.append(z)
        hs.append(h)
    out = np.matmul(h, p['W'][N_HIDDEN].astype(dtype)) + p['b'][N_HIDDEN].astype(dtype)
    if _smv(p):
        mean = out
        raw = np.matmul(h, p['Wv'].astype(dtype)) + p['bv'].astype(dtype)
    else:                                                                   # bnn.py:644-654
        D = out.shape[-1] // 2
        mean, raw = out[..., :D], out[..., D:]
    mx, mn = p['max_logvar'].astype(dtype), p['min_logvar'].astype(dtype)
    lv1 = mx - softplus(mx - raw)                                           # bnn.py:669
    lv = mn + softplus(lv1 - mn)                                            # bnn.py:670
    return {'zs': zs, 'hs': hs, 'raw': raw, 'lv1': lv1}, mean, lv


def mse_losses(p, X, Y, dtype=np.float64):
    """_compile_losses(inc_var_loss=False): per-member mean((mean - y)^2)."""
    _, mean, _ = forward3d(p, X, dtype)
    return np.mean(np.mean((mean - Y.astype(dtype)) ** 2, -1), -1)


def loss_and_grads(p, X, Y, dtype=np.float64):
    """Training loss (bnn.py:241-249) and its gradient w.r.t. optvars(p), in optvars order."""
    c, mean, lv = forward3d(p, X, dtype)
    y = Y.astype(dtype)
    E, B, D = mean.shape
    inv = np.exp(-lv)
    err = mean - y
    loss = np.sum(np.mean(np.mean(err * err * inv, -1), -1) + np.mean(np.mean(lv, -1), -1))
    Ws = [w.astype(dtype) for w in p['W']]
    smv = _smv(p)
    decay = sum(wd * 0.5 * np.sum(w * w) for wd, w in zip(WD, Ws))
    if smv:
        Wv = p['Wv'].astype(dtype)
        decay = decay + WD_VAR * 0.5 * np.sum(Wv * Wv)
    mx, mn = p['max_logvar'].astype(dtype), p['min_logvar'].astype(dtype)
    loss = loss + decay + 0.01 * np.sum(mx) - 0.01 * np.sum(mn)
    s = 1.0 / (B * D)
    dmean = 2.0 * err * inv * s
    dlv = (1.0 - err * err * inv) * s
    sig_b = _sigmoid(c['lv1'] - mn)                                         # d softplus(lv1 - mn)
    dlv1 = dlv * sig_b
    dmn = np.sum(dlv * (1.0 - sig_b), axis=(0, 1))[None] - 0.01
    sig_a = _sigmoid(mx - c['raw'])                                         # d softplus(mx - raw)
    draw = dlv1 * sig_a
    dmx = np.sum(dlv1 * (1.0 - sig_a), axis=(0, 1))[None] + 0.01
    h4 = c['hs'][N_HIDDEN]
    gW = [None] * (N_HIDDEN + 1)
    gb = [None] * (N_HIDDEN + 1)
    if smv:
        gW[N_HIDDEN] = np.matmul(h4.transpose(0, 2, 1), dmean) + WD[N_HIDDEN] * Ws[N_HIDDEN]
        gb[N_HIDDEN] = np.sum(dmean, 1, keepdims=True)
        gWv = np.matmul(h4.transpose(0, 2, 1), draw) + WD_VAR * Wv
        gbv = np.sum(draw, 1, keepdims=True)
        dh = np.matmul(dmean, Ws[N_HIDDEN].transpose(0, 2, 1)) + np.matmul(draw, Wv.transpose(0, 2, 1))
    else:                        # one [H, 2D] head: d out = [d mean | d raw]
        dout = np.concatenate([dmean, draw], -1)
        gW[N_HIDDEN] = np.matmul(h4.transpose(0, 2, 1), dout) + WD[N_HIDDEN] * Ws[N_HIDDEN]
        gb[N_HIDDEN] = np.sum(dout, 1, keepdims=True)
        dh = np.matmul(dout, Ws[N_HIDDEN].transpose(0, 2, 1))
    for l in range(N_HIDDEN - 1, -1, -1):
        z = c['zs'][l]
        sg = _sigmoid(z)
        dz = dh * (sg + z * sg * (1.0 - sg))
        gW[l] = np.matmul(c['hs'][l].transpose(0, 2, 1), dz) + WD[l] * Ws[l]
        gb[l] = np.sum(dz, 1, keepdims=True)
        if l > 0:
            dh = np.matmul(dz, Ws[l].transpose(0, 2, 1))
    grads = []
    for l in range(N_HIDDEN + 1):
        grads += [gW[l], gb[l]]
    if smv:
        grads += [gWv, gbv]
    grads += [dmx, dmn]
    return loss, grads


class TrainState:
    """Optimizer state of one BNN (tf.train.AdamOptimizer(1e-3) over optvars)."""

    def __init__(self, p, lr=1e-3, dtype=np.float64):
        self.p = p
        self.vals = [np.array(v, dtype) for v in optvars(p)]
        self.opt = Adam(self.vals, lr)

    def step(self, X, Y, dtype=np.float64):
        loss, g = loss_and_grads(set_optvars(self.p, self.vals), X, Y, dtype)
        self.vals = self.opt.apply(self.vals, g)
        return loss

    def params(self):
        return set_optvars(self.p, [v.astype(np.float32) for v in self.vals])


def shuffle_rows(arr):
    """bnn.py:385-387."""
    idxs = np.argsort(np.random.uniform(size=arr.shape), axis=-1)
    return arr[np.arange(arr.shape[0])[:, None], idxs]


def train(p, inputs, targets, num_elites, batch_size=32, max_epochs=None, max_epochs_since_update=5,
          holdout_ratio=0.0, max_logging=1000, max_grad_updates=None, dtype=np.float64):
    """BNN.train (bnn.py:369-503) with the reference's numpy RNG call order on the global stream.
    Returns (trained params, elites, holdout losses, epochs run, grad updates)."""
    E = p['W'][0].shape[0]
    num_holdout = min(int(inputs.shape[0] * holdout_ratio), max_logging)
    permutation = np.random.permutation(inputs.shape[0])
    inputs, holdout_inputs = inputs[permutation[num_holdout:]], inputs[permutation[:num_holdout]]
    targets, holdout_targets = targets[permutation[num_holdout:]], targets[permutation[:num_holdout]]
    holdout_inputs = np.tile(holdout_inputs[None], [E, 1, 1])
    holdout_targets = np.tile(holdout_targets[None], [E, 1, 1])
    p = dict(p)
    p['mu'], p['sigma'] = scaler_fit(inputs)
    idxs = np.random.randint(inputs.shape[0], size=[E, inputs.shape[0]])
    st = TrainState(p, dtype=dtype)
    snapshots = {i: (None, 1e10) for i in range(E)}
    state = {}
    since = 0
    grad_updates = 0
    epoch = 0
    while max_epochs is None or epoch < max_epochs:
        for b in range(int(np.ceil(idxs.shape[-1] / batch_size))):
            bi = idxs[:, b * batch_size:(b + 1) * batch_size]
            st.step(inputs[bi], targets[bi], dtype)
            grad_updates += 1
        idxs = shuffle_rows(idxs)
        cur = st.params()
        holdout_losses = mse_losses(cur, holdout_inputs, holdout_targets, dtype)
        updated = False                                                     # _save_best :287-312
        for i in range(E):
            _, best = snapshots[i]
            if (best - holdout_losses[i]) / best > 0.01:
                snapshots[i] = (epoch, holdout_losses[i])
                state[i] = [np.array(v[i]) for v in _member_vars(cur)]
                updated = True
        since = 0 if updated else since + 1
        epoch += 1
        if since > max_epochs_since_update or (max_grad_updates and grad_updates > max_grad_updates):
            break
    cur = st.params()
    vals = _member_vars(cur)                                                # _set_state :268-285
    for i, sv in state.items():
        for v, s in zip(vals, sv):
            v[i] = s
    cur = _set_member_vars(cur, vals)
    holdout_losses = mse_losses(cur, holdout_inputs, holdout_targets, dtype)
    elites = np.argsort(holdout_losses)[:num_elites].tolist()              # _end_train :329-332
    return cur, elites, holdout_losses, epoch, grad_updates


def _member_vars(p):
    """Per-member layer variables (weights, biases of every mean and var layer) -- the _state
    snapshot (bnn.py:264-266); maxlv / minlv are shared and not snapshotted."""
    out = []
    for w, b in zip(p['W'], p['b']):
        out += [np.array(w), np.array(b)]
    if _smv(p):
        out += [np.array(p['Wv']), np.array(p['bv'])]
    return out


def _set_member_vars(p, vals):
    q = dict(p)
    q['W'] = [vals[2 * i] for i in range(N_HIDDEN + 1)]
    q['b'] = [vals[2 * i + 1] for i in range(N_HIDDEN + 1)]
    if _smv(p):
        q['Wv'], q['bv'] = vals[-2], vals[-1]
    return q
