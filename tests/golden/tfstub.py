"""A torch-backed stand-in for the slice of the TensorFlow 1.14 API that the reference's graph code
calls on this path, so that the reference's OWN graph-building code can be executed here (TF is
not installed; nothing was denied).  TEST INFRASTRUCTURE ONLY: used by tests/golden/make_ref_vectors.py
in the build container to generate fixtures; never imported by mopo_amd/, tests or the GPU box.

What executes from the reference (loaded read-only by file path):
  * mopo/models/fc.py       FC.compute_output_tensor, FC._activations      (fc.py:15-22, 84-106)
  * mopo/models/utils.py    TensorStandardScaler.transform                 (utils.py:88-96)
  * mopo/models/bnn.py      BNN._compile_outputs (smv and joint head),     (bnn.py:631-675)
                            BNN._compile_losses                            (bnn.py:677-701)
  * mopo/algorithms/mopo.py MOPO._build (mlp, gaussian_likelihood, apply_squashing_func,
                            mlp_gaussian_policy, mlp_actor_critic, losses, optimizers, Polyak),
                            get_action_meta, _get_feed_dict, _do_training, _update_target
                            (mopo.py:204-485, 834-874)

What this module supplies is the TF1 primitive semantics those lines rely on, evaluated eagerly on
torch CPU tensors (f32 like the reference graph, or f64), with autograd standing in for
tf.gradients:
  * tf.layers.dense naming/reuse inside tf.variable_scope ('main/pi/dense_1/kernel:0', reuse=True
    returns the existing variable), the GLOBAL_VARIABLES creation order that mopo.py:32-33's
    get_vars() filters (including the Adam slot variables minimize() creates, which is why
    zip(get_vars('main'), get_vars('target')) pairs correctly by truncation);
  * tf.minimum / tf.maximum gradients to the first operand on ties (TF _MinimumGrad uses x <= y),
    tf.clip_by_value as minimum(maximum(t, lo), hi), tf.nn.softplus with Eigen's thresholds,
    tf.losses.mean_squared_error with SUM_BY_NONZERO_WEIGHTS;
  * tf.train.AdamOptimizer: TF1 ApplyAdam (lr_t = lr sqrt(1 - b2^t) / (1 - b1^t),
    m += (g - m)(1 - b1), v += (g^2 - v)(1 - b2), var -= lr_t m / (sqrt(v) + eps)), beta powers
    starting at b1, b2 and advanced after the update;
  * tf.assign(ref, expr) is recorded LAZILY: the coefficients of expr in each variable are read
    off autograd at build time and re-applied to the variables' current values when the op runs,
    so target_update (run after the training ops, mopo.py:852-853) sees the post-step weights as
    in the reference's graph;
  * tf.random_normal draws from a queue the caller fills (TF's Philox stream cannot be
    reproduced without TF), and records every draw.
Placeholders take their values from ``feeds`` (by placeholder name) at build time; Session.run
checks the feed_dict it is given against them.
"""
import contextlib
import sys
import types

import numpy as np
import torch


# ---------------------------------------------------------------------------- tensors and shapes
class Dim(int):
    @property
    def value(self):
        return int(self)


class Shape(tuple):
    def __new__(cls, dims):
        return tuple.__new__(cls, [Dim(d) for d in dims])

    def as_list(self):
        return [int(d) for d in self]


class T(torch.Tensor):
    """torch tensor whose .shape behaves like tf.TensorShape (.as_list(), dims with .value)."""

    @property
    def shape(self):
        return Shape(torch.Tensor.size(self))


def w(x):
    return x.as_subclass(T) if isinstance(x, torch.Tensor) and not isinstance(x, T) else x


def u(x):
    # identity: ops on T already dispatch to torch (T's default __torch_function__); an
    # as_subclass() alias of a variable would not be the leaf autograd differentiates against
    return x


class State:
    def __init__(self, dtype=torch.float32):
        self.dtype = dtype
        self.variables = []          # GLOBAL_VARIABLES, creation order
        self.by_name = {}
        self.scope = []              # [(name, reuse, counters)]
        self.feeds = {}
        self.noise = []              # queue for tf.random_normal
        self.noise_used = []
        self.init_values = {}        # variable name -> initial value (np array)
        self.missing_init = []
        self.optimizers = []


S = State()


def reset(dtype=torch.float32):
    global S
    S = State(dtype)
    return S


def _dtype(d):
    return S.dtype if d in (None, 'float32', 'float64') else d


class Var(T):
    """A graph variable: a leaf tensor with TF's variable name ('main/pi/dense/kernel:0')."""

    @property
    def name(self):
        return self.__dict__.get('_tf_name')


def _new_var(name, init):
    full = name + ':0'
    if full in S.init_values:
        val = np.asarray(S.init_values[full], np.float64)
        assert val.shape == tuple(np.shape(init)), (full, val.shape, np.shape(init))
    else:
        val = np.asarray(init, np.float64)
        S.missing_init.append(full)
    t = torch.tensor(val, dtype=S.dtype).as_subclass(Var).requires_grad_(True)
    t._tf_name = full
    S.variables.append(t)
    S.by_name[full] = t
    return t


def _scope_name():
    return '/'.join(s[0] for s in S.scope)


def _reuse():
    return any(s[1] for s in S.scope)


@contextlib.contextmanager
def variable_scope(name, reuse=None, default_name=None, **kw):
    S.scope.append((name, bool(reuse), {}))
    try:
        yield types.SimpleNamespace(name=_scope_name())
    finally:
        S.scope.pop()


def get_variable(name, shape=None, dtype=None, initializer=None, trainable=True, **kw):
    full = (_scope_name() + '/' if S.scope else '') + name
    if full + ':0' in S.by_name:
        if not _reuse():
            raise ValueError('Variable %s already exists' % full)
        return S.by_name[full + ':0']
    if isinstance(initializer, (int, float)):
        init = np.full(shape or (), float(initializer))
    elif callable(initializer):
        init = initializer(shape)
    else:
        init = np.zeros(shape)
    return _new_var(full, init)


def Variable(value, dtype=None, name='Variable', **kw):
    full = (_scope_name() + '/' if S.scope else '') + name
    return _new_var(full, np.asarray(value, np.float64))


def global_variables():
    return list(S.variables)


# ---------------------------------------------------------------------------- layers
def _layer_name(base):
    counters = S.scope[-1][2] if S.scope else S.__dict__.setdefault('_root_counters', {})
    n = counters.get(base, 0)
    counters[base] = n + 1
    return base if n == 0 else '%s_%d' % (base, n)


def _glorot(shape):
    lim = np.sqrt(6.0 / (shape[0] + shape[1]))
    return np.random.uniform(-lim, lim, size=shape)


def dense(x, units, activation=None, kernel_initializer=None, name=None, **kw):
    lname = name or _layer_name('dense')
    with variable_scope(lname, reuse=_reuse()):
        k = get_variable('kernel', shape=(int(x.shape[-1]), units), initializer=lambda s: _glorot(s))
        b = get_variable('bias', shape=(units,), initializer=0.0)
    y = w(torch.matmul(u(x), u(k)) + u(b))
    return activation(y) if activation is not None else y


# ---------------------------------------------------------------------------- ops
def _t(x):
    if isinstance(x, torch.Tensor):
        return x
    return torch.tensor(x, dtype=S.dtype).as_subclass(T)


def identity(x):
    return x


def relu(x):
    return w(torch.relu(u(x)))


def tanh(x):
    return w(torch.tanh(u(x)))


def sigmoid(x):
    return w(torch.sigmoid(u(x)))


def exp(x):
    return w(torch.exp(u(_t(x))))


def log(x):
    return w(torch.log(u(_t(x))))


def softplus(x):
    # Eigen scalar_softplus_op (TF 1.14 SoftplusOp): threshold = log(eps) + 2
    x = u(x)
    thr = float(np.log(np.finfo(np.float32 if x.dtype == torch.float32 else np.float64).eps) + 2)
    return w(torch.where(x > -thr, x, torch.where(x < thr, torch.exp(x), torch.log1p(torch.exp(x)))))


def softmax(x):
    return w(torch.softmax(u(x), -1))


def minimum(x, y):
    x, y = u(_t(x)), u(_t(y))
    return w(torch.where(x <= y, x, y))          # _MinimumGrad: x gets the gradient where x <= y


def maximum(x, y):
    x, y = u(_t(x)), u(_t(y))
    return w(torch.where(x >= y, x, y))          # _MaximumGrad: x where x >= y


def clip_by_value(t, lo, hi):
    return minimum(maximum(t, lo), hi)           # clip_ops.clip_by_value (TF 1.14)


def stop_gradient(x):
    return w(u(_t(x)).detach())


def reduce_sum(x, axis=None, keepdims=False):
    x = u(x)
    return w(x.sum() if axis is None else x.sum(dim=axis, keepdim=keepdims))


def reduce_mean(x, axis=None, keepdims=False):
    x = u(x)
    return w(x.mean() if axis is None else x.mean(dim=axis, keepdim=keepdims))


def square(x):
    return w(u(x) * u(x))


def squeeze(x, axis=None):
    return w(u(x).squeeze(axis))


def concat(values, axis):
    return w(torch.cat([u(v) for v in values], dim=axis))


def einsum(eq, *args):
    return w(torch.einsum(eq, *[u(a) for a in args]))


def matmul(a, b):
    return w(torch.matmul(u(a), u(b)))


def multiply(a, b, name=None):
    return w(u(_t(a)) * u(_t(b)))


def l2_loss(x):
    return w((u(x) ** 2).sum() / 2)


def add_n(xs):
    out = xs[0]
    for x in xs[1:]:
        out = out + x
    return out


def shape(x):
    return tuple(int(d) for d in torch.Tensor.size(u(x)))


def random_normal(shp, **kw):
    assert S.noise, 'tf.random_normal: noise queue empty'
    n = torch.as_tensor(S.noise.pop(0), dtype=S.dtype)
    assert tuple(n.shape) == tuple(shp), (tuple(n.shape), shp)
    S.noise_used.append(n.clone())
    return w(n)


def placeholder(dtype, shape=None, name=None):
    if name in S.feeds:
        return w(torch.as_tensor(S.feeds[name], dtype=S.dtype if dtype != 'int64' else torch.int64))
    return w(torch.zeros(1, dtype=S.dtype))


def mean_squared_error(labels, predictions, weights=1.0, **kw):
    # tf.losses.mean_squared_error, Reduction.SUM_BY_NONZERO_WEIGHTS
    lo = (u(predictions) - u(labels)) ** 2
    wt = torch.broadcast_to(torch.as_tensor(weights, dtype=lo.dtype), lo.shape)
    return w((lo * wt).sum() / (wt != 0).sum().to(lo.dtype))


# ---------------------------------------------------------------------------- ops to run later
class Op:
    def __init__(self, fn=None, deps=()):
        self.fn, self.deps = fn, list(deps)

    def run(self):
        for d in self.deps:
            _run_op(d)
        if self.fn is not None:
            self.fn()


def _run_op(x):
    if isinstance(x, Op):
        x.run()
    elif isinstance(x, (list, tuple)):
        for y in x:
            _run_op(y)


def group(*inputs, **kw):
    flat = []
    for i in inputs:
        flat.extend(i if isinstance(i, (list, tuple)) else [i])
    return Op(deps=flat)


def no_op():
    return Op()


def assign(ref, value):
    """Record ref <- sum_v c_v * v (the coefficients read off autograd now, applied at run time)."""
    vars_ = [v for v in S.variables if v.dtype.is_floating_point and v.requires_grad]
    val = u(value)
    if val.requires_grad:
        gs = torch.autograd.grad(val.sum(), vars_, allow_unused=True, retain_graph=True)
    else:
        gs = [None] * len(vars_)
    coef = []
    for v, g in zip(vars_, gs):
        if g is None or not bool((g != 0).any()):
            continue
        c = float(g.reshape(-1)[0])
        assert torch.allclose(g, torch.full_like(g, c)), 'assign: non-affine expression'
        coef.append((v, c))
    lin = sum(c * u(v).detach() for v, c in coef) if coef else 0
    assert torch.allclose(val.detach(), torch.as_tensor(lin, dtype=val.dtype).expand_as(val)), 'assign: not linear'

    def fn():
        with torch.no_grad():
            new = sum(c * u(v).detach().clone() for v, c in coef)
            u(ref).copy_(new)
    op = Op(fn)
    op.pairs = [(ref.name, v.name, c) for v, c in coef]
    return op


@contextlib.contextmanager
def control_dependencies(deps):
    yield


class Optimizer:
    pass


class AdamOptimizer(Optimizer):
    def __init__(self, learning_rate=1e-3, beta1=0.9, beta2=0.999, epsilon=1e-8, name='Adam'):
        self.lr, self.b1, self.b2, self.eps, self.name = learning_rate, beta1, beta2, epsilon, name
        self.grads = None
        self.beta_powers = None
        S.optimizers.append(self)

    def compute_gradients(self, loss, var_list):
        gs = torch.autograd.grad(u(loss), [u(v) for v in var_list], allow_unused=True, retain_graph=True)
        return [(None if g is None else g.detach(), v) for g, v in zip(gs, var_list)]

    def minimize(self, loss, var_list):
        gv = self.compute_gradients(loss, var_list)
        gv = [(g, v) for g, v in gv if g is not None]
        assert gv, 'No gradients provided for any variable'
        self.grads = gv
        # slots in creation order (Adam._create_slots: m then v per variable, beta powers first)
        with variable_scope(''):
            pass
        if self.beta_powers is None:
            b1p = _new_var(self._unique('beta1_power'), np.float64(self.b1))
            b2p = _new_var(self._unique('beta2_power'), np.float64(self.b2))
            self.beta_powers = (b1p, b2p)
        self.slots = []
        for g, v in gv:
            base = v.name[:-2]
            m = _new_var(base + '/' + self._slot('Adam'), np.zeros(tuple(v.shape)))
            vv = _new_var(base + '/' + self._slot('Adam_1'), np.zeros(tuple(v.shape)))
            self.slots.append((m, vv))

        def fn():
            b1p, b2p = self.beta_powers
            with torch.no_grad():
                lr_t = self.lr * torch.sqrt(1 - u(b2p)) / (1 - u(b1p))
                for (g, v), (m, vv) in zip(self.grads, self.slots):
                    u(m).add_((g - u(m)) * (1 - self.b1))
                    u(vv).add_((g * g - u(vv)) * (1 - self.b2))
                    u(v).sub_(lr_t * u(m) / (torch.sqrt(u(vv)) + self.eps))
                u(b1p).mul_(self.b1)
                u(b2p).mul_(self.b2)
        return Op(fn)

    def _unique(self, base):
        name, i = base, 0
        while name + ':0' in S.by_name:
            i += 1
            name = '%s_%d' % (base, i)
        return name

    def _slot(self, base):
        # slot names are '<var>/<optimizer name>' ('Adam', 'Adam_1'; 'alpha_optimizer', '..._1')
        if self.name == 'Adam':
            return base
        return self.name + base[4:]


def clip_by_global_norm(ts, clip_norm):
    gn = torch.sqrt(sum((u(t) ** 2).sum() for t in ts))
    scale = min(1.0, float(clip_norm) / float(gn)) if float(gn) > 0 else 1.0
    return [w(u(t) * scale) for t in ts], w(gn)


class Session:
    """Runs recorded ops; returns the eagerly computed fetch values (checks the feeds)."""

    def __init__(self):
        self.skip = set()

    def run(self, fetches, feed_dict=None):
        if feed_dict:
            for k, v in feed_dict.items():
                assert torch.allclose(u(k).double(), torch.as_tensor(np.asarray(v), dtype=torch.float64)), \
                    'Session.run: feed differs from the build-time placeholder value'
        return self._fetch(fetches)

    def _fetch(self, f):
        if isinstance(f, Op):
            if id(f) not in self.skip:
                f.run()
            return None
        if isinstance(f, dict):
            return {k: self._fetch(v) for k, v in f.items()}
        if isinstance(f, (list, tuple)):
            return [self._fetch(x) for x in f]
        if isinstance(f, torch.Tensor):
            return u(f).detach().numpy().copy()
        return f

    @contextlib.contextmanager
    def as_default(self):
        yield self


def global_variables_initializer():
    return Op()


def variables_initializer(vs):
    return Op()


# ---------------------------------------------------------------------------- module wiring
def install():
    """Put the stub in sys.modules as ``tensorflow`` (+ tensorflow.python.training.training_util)."""
    tf = types.ModuleType('tensorflow')
    for k in ('variable_scope', 'get_variable', 'Variable', 'global_variables', 'identity', 'tanh', 'sigmoid',
              'exp', 'log', 'minimum', 'maximum', 'clip_by_value', 'stop_gradient', 'reduce_sum', 'reduce_mean',
              'square', 'squeeze', 'concat', 'einsum', 'matmul', 'multiply', 'add_n', 'shape', 'random_normal',
              'placeholder', 'group', 'no_op', 'assign', 'control_dependencies', 'clip_by_global_norm',
              'Session', 'global_variables_initializer', 'variables_initializer'):
        setattr(tf, k, globals()[k])
    tf.float32, tf.float64, tf.int64, tf.int32 = 'float32', 'float64', 'int64', 'int32'
    tf.nn = types.SimpleNamespace(relu=relu, softplus=softplus, softmax=softmax, l2_loss=l2_loss, sigmoid=sigmoid)
    tf.layers = types.SimpleNamespace(dense=dense)
    tf.losses = types.SimpleNamespace(mean_squared_error=mean_squared_error)
    tf.train = types.SimpleNamespace(AdamOptimizer=AdamOptimizer, Optimizer=Optimizer)
    tf.truncated_normal_initializer = lambda stddev=1.0, **k: (lambda s: np.zeros(s))
    tf.constant_initializer = lambda v=0.0, **k: (lambda s: np.full(s, v))
    tf.contrib = types.SimpleNamespace(checkpoint=types.SimpleNamespace(Checkpointable=object))
    sys.modules['tensorflow'] = tf
    py = types.ModuleType('tensorflow.python')
    tr = types.ModuleType('tensorflow.python.training')
    tu = types.ModuleType('tensorflow.python.training.training_util')
    tu.get_or_create_global_step = lambda: _new_var('global_step', np.float64(0)) \
        if 'global_step:0' not in S.by_name else S.by_name['global_step:0']
    tu._increment_global_step = lambda n: Op()
    tr.training_util = tu
    py.training = tr
    tf.python = py
    sys.modules['tensorflow.python'] = py
    sys.modules['tensorflow.python.training'] = tr
    sys.modules['tensorflow.python.training.training_util'] = tu
    return tf
