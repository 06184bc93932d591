"""Oracle: MOPO's in-graph SAC step, numpy restatement with hand-written backprop.
TEST INFRASTRUCTURE ONLY.

Follows (reference xionghuichen/mopo, ``mopo/algorithms/mopo.py``):
  * mlp / gaussian_likelihood / apply_squashing_func / mlp_gaussian_policy   :275-308
  * mlp_actor_critic (pi, q1, q2; Q on concat(s, a))                          :311-325
  * the four forward instances main(s,a), main(s,pi), main(s'), target(s',pi') :337-350
  * alpha = exp(log_alpha), policy loss with stop_gradient(alpha)              :357-377
  * q_target / 0.5-weighted MSE (SUM_BY_NONZERO_WEIGHTS)                       :380-405
  * four TF1 Adam optimizers (pi, q1, q2, alpha), alpha loss on pre-step logp  :407-443
  * Polyak target update, zip(main, target) in creation order                 :446-447
  * logged fetches                                                             :453-463, _do_training :834-850
Semantics decision: every forward and gradient uses the pre-step
parameters; then pi, q1, q2, alpha are updated; then Polyak.
Parity: restatement-pinned; cross-checked against torch autograd in tests.
"""
import numpy as np

LOG_STD_MAX, LOG_STD_MIN, EPS = 2.0, -20.0, 1e-8          # mopo.py:271-273
LOG2PI = np.log(2 * np.pi)

def _hs(H):
    """hidden_sizes (mopo.py:275-280): an int H is [H, H]."""
    return (H, H) if np.isscalar(H) else tuple(H)


PI_SHAPES = lambda O, A, H: [(O, _hs(H)[0]), (_hs(H)[0],), _hs(H), (_hs(H)[1],), (_hs(H)[1], A), (A,),
                             (_hs(H)[1], A), (A,)]
Q_SHAPES = lambda O, A, H: [(O + A, _hs(H)[0]), (_hs(H)[0],), _hs(H), (_hs(H)[1],), (_hs(H)[1], 1), (1,)]


def param_shapes(O, A, H=256):
    """Creation order of get_vars('main') (mopo.py:32-33): pi (dense..dense_3), q1, q2; ``H`` an int or
    the two hidden widths [H1, H2]."""
    return PI_SHAPES(O, A, H) + Q_SHAPES(O, A, H) + Q_SHAPES(O, A, H)


def init_params(O, A, H=256, seed=2, dtype=np.float64):
    """tf.layers.dense defaults: glorot_uniform kernels, zero biases."""
    rng = np.random.RandomState(seed)
    out = []
    for shp in param_shapes(O, A, H):
        if len(shp) == 2:
            lim = np.sqrt(6.0 / (shp[0] + shp[1]))
            out.append(rng.uniform(-lim, lim, size=shp).astype(np.float32).astype(dtype))
        else:
            out.append(np.zeros(shp, dtype))
    return out


def split(params):
    return params[0:8], params[8:14], params[14:20]


def softplus(x):
    return np.logaddexp(0.0, x)


def sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


# ------------------------------------------------------------------ forward pieces
def pi_forward(P, s, eps):
    W1, b1, W2, b2, Wm, bm, Wl, bl = P
    z1 = s @ W1 + b1; h1 = np.maximum(z1, 0)
    z2 = h1 @ W2 + b2; h2 = np.maximum(z2, 0)                       # mlp(x, hs, act, act): :301
    mu = h2 @ Wm + bm                                               # :302
    ls_raw = h2 @ Wl + bl                                           # :303
    ls = np.clip(ls_raw, LOG_STD_MIN, LOG_STD_MAX)                  # :304
    std = np.exp(ls)                                                # :305
    u = mu + eps * std                                              # :306
    zz = (u - mu) / (std + EPS)
    logp = np.sum(-0.5 * (zz ** 2 + 2 * ls + LOG2PI), axis=-1)       # :282-284
    logp = logp - np.sum(2 * (np.log(2) - u - softplus(-2 * u)), axis=-1)   # :292
    a = np.tanh(u)
    cache = dict(s=s, z1=z1, h1=h1, z2=z2, h2=h2, mu=mu, ls_raw=ls_raw, ls=ls, std=std, u=u, zz=zz,
                 a=a, eps=eps)
    return np.tanh(mu), a, logp, std, cache


def q_forward(Q, s, a):
    W1, b1, W2, b2, W3, b3 = Q
    x = np.concatenate([s, a], axis=-1)                             # :322
    z1 = x @ W1 + b1; h1 = np.maximum(z1, 0)
    z2 = h1 @ W2 + b2; h2 = np.maximum(z2, 0)
    q = (h2 @ W3 + b3)[:, 0]                                        # :319 squeeze
    return q, dict(x=x, z1=z1, h1=h1, z2=z2, h2=h2)


def q_backward(Q, c, dq, need_params=True):
    """Backprop dq [n] through Q. returns (param grads or None, dx [n, O+A])."""
    W1, b1, W2, b2, W3, b3 = Q
    dq = dq[:, None]
    gW3 = c['h2'].T @ dq; gb3 = dq.sum(0)
    dh2 = dq @ W3.T
    dz2 = dh2 * (c['z2'] > 0)
    gW2 = c['h1'].T @ dz2; gb2 = dz2.sum(0)
    dh1 = dz2 @ W2.T
    dz1 = dh1 * (c['z1'] > 0)
    gW1 = c['x'].T @ dz1; gb1 = dz1.sum(0)
    dx = dz1 @ W1.T
    grads = [gW1, gb1, gW2, gb2, gW3, gb3] if need_params else None
    return grads, dx


def pi_backward(P, c, dlogp, da):
    """Backprop d(logp) [n] and d(a) [n,A] (a = tanh(u)) to pi params."""
    W1, b1, W2, b2, Wm, bm, Wl, bl = P
    u, mu, std, ls, zz, eps = c['u'], c['mu'], c['std'], c['ls'], c['zz'], c['eps']
    g = dlogp[:, None]
    inv = 1.0 / (std + EPS)
    du = da * (1 - c['a'] ** 2)                                     # tanh grad (y-based)
    du = du + g * (-zz * inv)                                       # d(-0.5 zz^2)/du
    du = du + g * (2.0 - 4.0 * sigmoid(-2 * u))                     # squash correction
    dmu = g * (zz * inv)
    dstd = g * (zz * zz * inv)
    dls = -g * np.ones_like(ls)                                     # d(-ls)/dls
    dmu = dmu + du                                                  # u = mu + eps*std
    dstd = dstd + du * eps
    dls = dls + dstd * std                                          # std = exp(ls)
    r = c['ls_raw']
    dls_raw = dls * ((r >= LOG_STD_MIN) & (r <= LOG_STD_MAX))       # clip_by_value grad
    gWm = c['h2'].T @ dmu; gbm = dmu.sum(0)
    gWl = c['h2'].T @ dls_raw; gbl = dls_raw.sum(0)
    dh2 = dmu @ Wm.T + dls_raw @ Wl.T
    dz2 = dh2 * (c['z2'] > 0)
    gW2 = c['h1'].T @ dz2; gb2 = dz2.sum(0)
    dh1 = dz2 @ W2.T
    dz1 = dh1 * (c['z1'] > 0)
    gW1 = c['s'].T @ dz1; gb1 = dz1.sum(0)
    return [gW1, gb1, gW2, gb2, gWm, gbm, gWl, gbl]


# ------------------------------------------------------------------ optimizer
class Adam:
    """tf.train.AdamOptimizer (TF1 ApplyAdam kernel semantics)."""

    def __init__(self, params, lr=3e-4, b1=0.9, b2=0.999, eps=1e-8):
        self.lr, self.b1, self.b2, self.eps = lr, b1, b2, eps
        self.m = [np.zeros_like(p) for p in params]
        self.v = [np.zeros_like(p) for p in params]
        self.b1p, self.b2p = b1, b2                                 # beta powers start at beta

    def apply(self, params, grads):
        lr_t = self.lr * np.sqrt(1 - self.b2p) / (1 - self.b1p)
        for i, (p, g) in enumerate(zip(params, grads)):
            self.m[i] = self.m[i] + (g - self.m[i]) * (1 - self.b1)
            self.v[i] = self.v[i] + (g * g - self.v[i]) * (1 - self.b2)
            params[i] = p - lr_t * self.m[i] / (np.sqrt(self.v[i]) + self.eps)
        self.b1p *= self.b1
        self.b2p *= self.b2
        return params


class SACState:
    def __init__(self, params, log_alpha=0.0, lr=3e-4):
        self.params = [np.array(p, np.float64) for p in params]
        self.target = [p.copy() for p in self.params]               # target_init :449-450
        self.log_alpha = np.array(log_alpha, np.float64)
        P, Q1, Q2 = split(self.params)
        self.opt_pi, self.opt_q1, self.opt_q2 = Adam(P, lr), Adam(Q1, lr), Adam(Q2, lr)
        self.opt_a = Adam([self.log_alpha], lr)


def prior_log_prob(a):
    """softlearning sac.py:285-289: MultivariateNormalDiag(0, 1).log_prob(actions), per row."""
    return -0.5 * np.sum(a * a, axis=-1) - 0.5 * a.shape[-1] * np.log(2 * np.pi)


def sac_step(st, batch, eps_s, eps_s2, gamma=0.99, tau=5e-3, reward_scale=1.0, target_entropy=-3.0, grads_out=None,
             action_prior='uniform'):
    """One ``_do_training`` + ``_update_target`` (mopo.py:834-853). Mutates ``st``; returns logs.
    ``grads_out`` (dict): receives the pre-step gradients 'pi', 'q1', 'q2' (lists) and 'alpha'.
    ``action_prior='normal'``: softlearning's SAC (sac.py:285-289, 304-306) subtracts the standard-normal
    log-prob of the policy's action from the policy loss (MOPO's own graph asserts 'uniform',
    mopo.py:364)."""
    s, a, s2 = batch['observations'], batch['actions'], batch['next_observations']
    r, d = batch['rewards'][:, 0], batch['terminals'][:, 0].astype(np.float64)
    n = s.shape[0]
    P, Q1, Q2 = split(st.params)
    T = split(st.target)
    alpha = np.exp(st.log_alpha)
    # forwards with pre-step params
    _, a_pi, logp_pi, std, cpi = pi_forward(P, s, eps_s)
    q1_pi, c1p = q_forward(Q1, s, a_pi)
    q2_pi, c2p = q_forward(Q2, s, a_pi)
    _, a_next, logp_next, _, _ = pi_forward(P, s2, eps_s2)
    q1_t, _ = q_forward(T[1], s2, a_next)
    q2_t, _ = q_forward(T[2], s2, a_next)
    q1, c1 = q_forward(Q1, s, a)
    q2, c2 = q_forward(Q2, s, a)
    y = reward_scale * r + gamma * ((1 - d) * (np.minimum(q1_t, q2_t) - alpha * logp_next))  # :380-386
    q1_loss = 0.5 * np.mean((q1 - y) ** 2)
    q2_loss = 0.5 * np.mean((q2 - y) ** 2)
    prior = prior_log_prob(a_pi) if action_prior == 'normal' else 0.0
    pi_loss = np.mean(alpha * logp_pi - np.minimum(q1_pi, q2_pi) - prior)
    # gradients
    g_q1, _ = q_backward(Q1, c1, (q1 - y) / n)
    g_q2, _ = q_backward(Q2, c2, (q2 - y) / n)
    sel1 = q1_pi <= q2_pi                                           # tf.minimum grad -> x where x<=y
    _, dx1 = q_backward(Q1, c1p, np.where(sel1, -1.0 / n, 0.0), need_params=False)
    _, dx2 = q_backward(Q2, c2p, np.where(sel1, 0.0, -1.0 / n), need_params=False)
    O = s.shape[1]
    da = dx1[:, O:] + dx2[:, O:]
    if action_prior == 'normal':
        da = da + a_pi / n                                          # d/da of -mean(log N(a; 0, I))
    g_pi = pi_backward(P, cpi, np.full(n, alpha / n), da)
    g_alpha = -np.mean(logp_pi + target_entropy)                    # d/dlog_alpha of :437-438
    if grads_out is not None:
        grads_out.update(pi=g_pi, q1=g_q1, q2=g_q2, alpha=g_alpha)
    pi_gnorm = np.sqrt(sum(np.sum(g * g) for g in g_pi))
    q_gnorm = np.sqrt(sum(np.sum((0.5 * g) ** 2) for g in g_q1))     # grads of Q_loss wrt q1 vars (:431-432)
    # updates
    P = st.opt_pi.apply(list(P), g_pi)
    Q1 = st.opt_q1.apply(list(Q1), g_q1)
    Q2 = st.opt_q2.apply(list(Q2), g_q2)
    st.log_alpha = st.opt_a.apply([st.log_alpha], [np.array(g_alpha)])[0]
    st.params = list(P) + list(Q1) + list(Q2)
    st.target = [(1 - tau) * t + tau * p for t, p in zip(st.target, st.params)]   # :446-447
    pi_entropy = np.sum(np.log(std + 1e-8) + 0.5 * np.log(2 * np.pi * np.e), axis=-1)  # :341
    return {'sac_pi/pi_global_norm': pi_gnorm, 'sac_Q/q_global_norm': q_gnorm,
            'Q/q1_loss': q1_loss, 'sac_Q/q2_loss': q2_loss,
            'sac_Q/q1': np.mean(q1), 'sac_Q/q2': np.mean(q2), 'sac_pi/alpha': alpha,
            'sac_pi/pi_entropy': np.mean(pi_entropy), 'sac_pi/logp_pi': np.mean(logp_pi),
            'sac_pi/std': np.mean(logp_pi), 'pi_loss': pi_loss}


def actor_act(P, obs, eps):
    """``get_action_meta(obs)`` for rollouts (mopo.py:468-485): returns (pi, mu) tanh-squashed."""
    mu_t, a, _, _, _ = pi_forward(P, obs, eps)
    return a, mu_t


def flops_per_step(n, O, A, H=256):
    """Algorithmic GEMM FLOPs of one SAC step (forward + backward), batch n."""
    pi_f = O * H + H * H + 2 * H * A
    q_f = (O + A) * H + H * H + H
    fwd = 2 * pi_f + 6 * q_f
    bwd = 2 * pi_f + 2 * (2 * q_f) + 2 * q_f      # pi params+input; q1,q2 params+input; q*_pi input only
    return 2 * n * (fwd + bwd)
