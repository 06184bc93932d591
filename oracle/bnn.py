"""Oracle: probabilistic-ensemble (BNN) forward, numpy restatement.  TEST INFRASTRUCTURE ONLY.

Follows (reference xionghuichen/mopo):
  * ``TensorStandardScaler.transform``      mopo/models/utils.py:88-96
  * ``TensorStandardScaler.fit``            mopo/models/utils.py:69-86
  * ``FC.compute_output_tensor`` + swish    mopo/models/fc.py:84-106, 15-22
  * ``BNN._compile_outputs`` (smv branch)   mopo/models/bnn.py:656-675
  * ``BNN._compile_outputs`` (joint head)   mopo/models/bnn.py:644-655
  * max/min log-var init                    mopo/models/bnn.py:196-213
  * ``construct_model`` layer stack         mopo/models/constructor.py:28-36
  * ``.mat`` key order (nonoptvars+optvars) mopo/models/bnn.py:224-225, 276-281, 588-592

Parity: restatement-pinned (TensorFlow 1.14 is not installed here).
"""
import numpy as np

N_HIDDEN = 4  # constructor.py:30-33: four swish FC layers


def softplus(x):
    # tf.nn.softplus == log(1 + exp(x)), evaluated stably
    return np.logaddexp(np.zeros((), dtype=x.dtype), x).astype(x.dtype)


def swish(x):
    # fc.py:21  lambda x: x * tf.sigmoid(x)
    one = x.dtype.type(1)
    return x * (one / (one + np.exp(-x)))


def init_params(E, obs_dim, act_dim, hidden=200, seed=1, smv=True, bias_std=0.01,
                inputs=None):
    """Synthetic ensemble weights.

    Weights ~ truncated_normal(std = 1/(2*sqrt(in))) as fc.py:145-149, then
    biases ~ N(0, bias_std) (so the bias path is exercised), max/min logvar as
    bnn.py:210-213, scaler fitted on ``inputs`` (utils.py:79-81) or identity.
    """
    rng = np.random.RandomState(seed)
    IN, D = obs_dim + act_dim, obs_dim + 1

    def tn(shape, std):
        w = rng.normal(size=shape) * std
        bad = np.abs(w) > 2 * std
        while bad.any():  # truncated normal: re-draw beyond two std
            w[bad] = rng.normal(size=int(bad.sum())) * std
            bad = np.abs(w) > 2 * std
        return w.astype(np.float32)

    dims = [IN] + [hidden] * N_HIDDEN + [D if smv else 2 * D]
    Ws, bs = [], []
    for i in range(len(dims) - 1):
        Ws.append(tn((E, dims[i], dims[i + 1]), 1.0 / (2 * np.sqrt(dims[i]))))
        bs.append((rng.normal(size=(E, 1, dims[i + 1])) * bias_std).astype(np.float32))
    p = {'W': Ws, 'b': bs}
    if smv:
        p['Wv'] = tn((E, hidden, D), 1.0 / (2 * np.sqrt(hidden)))
        p['bv'] = (rng.normal(size=(E, 1, D)) * bias_std).astype(np.float32)
    p['max_logvar'] = (np.ones([1, D]) / 2.0).astype(np.float32)
    p['min_logvar'] = (-np.ones([1, D]) * 10.0).astype(np.float32)
    if inputs is None:
        p['mu'] = np.zeros([1, IN], np.float32)
        p['sigma'] = np.ones([1, IN], np.float32)
    else:
        p['mu'], p['sigma'] = scaler_fit(inputs)
    p['smv'] = smv
    return p


def scaler_fit(data):
    """utils.py:79-81 (computed in numpy f64 for f64 data, stored as f32 tf vars)."""
    mu = np.mean(data, axis=0, keepdims=True)
    sigma = np.std(data, axis=0, keepdims=True)
    sigma[sigma < 1e-12] = 1.0
    return mu.astype(np.float32), sigma.astype(np.float32)


def forward(p, inputs, dtype=np.float32, ret_log_var=False):
    """``BNN.predict(inputs2d, factored=True)`` (bnn.py:530-536 -> 631-675).

    inputs: [B, IN] (any float dtype; the TF placeholder casts to f32).
    returns mean, var: [E, B, D].
    """
    x = np.asarray(inputs).astype(dtype)
    mu, sigma = p['mu'].astype(dtype), p['sigma'].astype(dtype)
    h = (x - mu) / sigma                                            # utils.py:96
    Ws = [w.astype(dtype) for w in p['W']]
    bs = [b.astype(dtype) for b in p['b']]
    h = np.einsum('ij,ajk->aik', h, Ws[0]) + bs[0]                   # fc.py:99
    h = swish(h)
    for l in range(1, N_HIDDEN):
        h = swish(np.matmul(h, Ws[l]) + bs[l])                      # fc.py:101,106
    maxlv, minlv = p['max_logvar'].astype(dtype), p['min_logvar'].astype(dtype)
    if p['smv']:
        mean = np.matmul(h, Ws[N_HIDDEN]) + bs[N_HIDDEN]            # bnn.py:661-663
        lv = np.matmul(h, p['Wv'].astype(dtype)) + p['bv'].astype(dtype)  # bnn.py:665-667 (taps means[-2])
    else:
        out = np.matmul(h, Ws[N_HIDDEN]) + bs[N_HIDDEN]
        D = out.shape[-1] // 2
        mean, lv = out[:, :, :D], out[:, :, D:]                     # bnn.py:650,654
    lv = maxlv - softplus(maxlv - lv)                                # bnn.py:669
    lv = minlv + softplus(lv - minlv)                                # bnn.py:670
    if ret_log_var:
        return mean, lv
    return mean, np.exp(lv)                                          # bnn.py:675


def to_mat_list(p):
    """The 16 arrays of the reference ``.mat`` file, keys '0'..'15' (bnn.py:588-592):
    nonoptvars (scaler mu, sigma) + optvars (mean-layer W,b x5, var-layer W,b, maxlv, minlv)."""
    out = [p['mu'], p['sigma']]
    for w, b in zip(p['W'], p['b']):
        out += [w, b]
    if p['smv']:
        out += [p['Wv'], p['bv']]
    out += [p['max_logvar'], p['min_logvar']]
    return out


def from_mat_list(arrs, smv=True):
    arrs = [np.asarray(a, np.float32) for a in arrs]
    p = {'mu': arrs[0], 'sigma': arrs[1], 'smv': smv}
    n_mean = N_HIDDEN + 1
    p['W'] = [arrs[2 + 2 * i] for i in range(n_mean)]
    p['b'] = [arrs[3 + 2 * i] for i in range(n_mean)]
    k = 2 + 2 * n_mean
    if smv:
        p['Wv'], p['bv'] = arrs[k], arrs[k + 1]
        k += 2
    p['max_logvar'], p['min_logvar'] = arrs[k], arrs[k + 1]
    return p


def flops_per_row(E, IN, H, D):
    """GEMM FLOPs of one ensemble forward per input row."""
    return 2 * E * (IN * H + (N_HIDDEN - 1) * H * H + 2 * H * D)
