"""Debug: f16x3 predict error per row vs the f64 oracle (which rows, what magnitudes)."""
import sys, os
import numpy as np
import shutil
if os.environ.get("SO"): shutil.copy(os.environ["SO"], "mopo_amd/libmopo_hip.so")
sys.path.insert(0, os.getcwd())
from oracle import bnn as obnn
from mopo_amd.bnn import BNN

def model(mats, E, H, dtype):
    return BNN({'name': 't', 'num_networks': E, 'num_elites': 5, 'separate_mean_var': True, 'obs_dim': 17,
                'act_dim': 6, 'hidden_dim': H, 'dtype': dtype}).set_params(mats)

E, H, B = 7, 200, 4099
rs = np.random.RandomState(E + H + B)
mats = obnn.to_mat_list(obnn.init_params(E, 17, 6, hidden=H, seed=3, inputs=rs.normal(size=(300, 23)) * 3))
p = obnn.from_mat_list(mats)
x = (rs.normal(size=(B, 23)) * 2).astype(np.float32)
rm, rv = obnn.forward(p, x, dtype=np.float64)
for dt in ('fp32', 'bf16x6', 'f16x3'):
    m, v = model(mats, E, H, dt).predict(x)
    em = np.abs(m - rm) / (1 + np.abs(rm))
    ev = np.abs(v - rv) / (1 + np.abs(rv))
    rowerr = np.maximum(em.max(axis=(0, 2)), ev.max(axis=(0, 2)))
    bad = np.argsort(-rowerr)[:6]
    print(dt, 'max', em.max(), ev.max(), 'rows>2e-5:', int((rowerr > 2e-5).sum()), 'worst rows', bad.tolist(),
          ['%.2e' % rowerr[b] for b in bad])
    if dt == 'f16x3':
        memb = np.maximum(em.max(axis=2), ev.max(axis=2))   # [E, B]
        print(' per member max', memb.max(axis=1))
        b = bad[0]
        print(' worst row members', memb[:, b], 'x', x[b])
        print(' rows by tile (16):', sorted(set((np.where(rowerr > 2e-5)[0] // 16).tolist()))[:40])
        print(' rows mod 64:', sorted(set((np.where(rowerr > 2e-5)[0] % 64).tolist()))[:64])

# --- numpy emulation of the f16x3 algorithm (per-row scale, per-layer-member weight scale)
def split16(v, s):
    vs = (v * s).astype(np.float32)
    h = vs.astype(np.float16)
    l = (vs - h.astype(np.float32)).astype(np.float16)
    return h.astype(np.float64), l.astype(np.float64)

def wsc(W):  # per member
    m = np.abs(W).reshape(W.shape[0], -1).max(1)
    ex = np.frexp(m)[1]
    return np.ldexp(1.0, 15 - ex)

def rsc(X):  # per row of [E,B,K] or [B,K]
    m = np.abs(X).max(-1, keepdims=True).astype(np.float32)
    ex = np.frexp(m)[1]
    return np.ldexp(1.0, 15 - ex).astype(np.float32)

def layer(X, W, b, act):
    # X [E,B,K] f32, W [E,K,N]
    sw = wsc(W)[:, None, None]
    w0, w1 = split16(W.astype(np.float32), sw.astype(np.float32))
    sx = rsc(X)
    x0, x1 = split16(X, sx)
    acc = x0 @ w0 + x0 @ w1 + x1 @ w0
    out = (acc / sw / sx).astype(np.float32) + b
    return (out * (1 / (1 + np.exp(-out)))).astype(np.float32) if act else out.astype(np.float32)

xs = ((x - p['mu']) / p['sigma']).astype(np.float32)
X = np.broadcast_to(xs, (E,) + xs.shape).astype(np.float32)
for l in range(4):
    X = layer(X, p['W'][l], p['b'][l], True)
mean = layer(X, p['W'][4], p['b'][4], False)
em = np.abs(mean - rm) / (1 + np.abs(rm))
print('numpy f16x3 emulation: mean max err', em.max())
m1, v1 = model(mats, E, H, 'f16x3').predict(x)
m2, v2 = model(mats, E, H, 'f16x3').predict(x)
print('determinism: identical?', np.array_equal(m1, m2), 'max diff', np.abs(m1 - m2).max())
