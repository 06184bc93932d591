"""Per-domain termination functions (``mopo.static``), as device termination kinds.

Reference: mopo/static/__init__.py:7-25 builds ``{domain: StaticFns}``; the rules are
mopo/static/halfcheetah.py:6-11, walker2d.py:6-17, hopper.py:6-18, ant.py:6-17 (= antangle.py),
humanoid.py:7-15, and the never-done halfcheetahjump / halfcheetahvel / halfcheetahveljump /
point2denv / point2dwallenv / pendulum.  pendulum.py:9 returns float zeros, which the reference's own
rollout cannot negate (mopo.py:753 ``~term`` on float64 raises TypeError); here it is bool False.  On the accelerated path the
rule runs inside the FakeEnv kernels (``term_fn`` in csrc/internal.h) selected by ``term_kind``;
``termination_fn`` here is the same rule on torch tensors for callers that use it directly.
"""
import numpy as np

TERM_HALFCHEETAH, TERM_WALKER2D, TERM_HOPPER, TERM_ANT, TERM_HUMANOID = 0, 1, 2, 3, 4


class StaticFns:
    def __init__(self, domain, term_kind):
        self.domain, self.term_kind = domain, term_kind

    def termination_fn(self, obs, act, next_obs):
        import torch
        is_np = isinstance(next_obs, np.ndarray)
        x = torch.as_tensor(next_obs)
        assert len(obs.shape) == len(next_obs.shape) == len(act.shape) == 2
        if self.term_kind == TERM_WALKER2D:
            h, a = x[:, 0], x[:, 1]
            done = ~((h > 0.8) & (h < 2.0) & (a > -1.0) & (a < 1.0))
        elif self.term_kind == TERM_HOPPER:
            h, a = x[:, 0], x[:, 1]
            nd = torch.isfinite(x).all(-1) & (x[:, 1:] < 100).all(-1) & (h > .7) & (a.abs() < .2)
            done = ~nd
        elif self.term_kind == TERM_ANT:
            h = x[:, 0]
            done = ~(torch.isfinite(x).all(-1) & (h >= 0.2) & (h <= 1.0))
        elif self.term_kind == TERM_HUMANOID:
            z = x[:, 0]
            done = (z < 1.0) | (z > 2.0)
        else:
            done = torch.zeros(x.shape[0], dtype=torch.bool, device=x.device)
        done = done[:, None]
        return done.cpu().numpy() if is_np else done


static_fns = {
    'halfcheetah': StaticFns('halfcheetah', TERM_HALFCHEETAH),
    'walker2d': StaticFns('walker2d', TERM_WALKER2D),
    'hopper': StaticFns('hopper', TERM_HOPPER),
    'ant': StaticFns('ant', TERM_ANT),
    'antangle': StaticFns('antangle', TERM_ANT),
    'humanoid': StaticFns('humanoid', TERM_HUMANOID),
}
for _d in ('halfcheetahjump', 'halfcheetahvel', 'halfcheetahveljump', 'point2denv', 'point2dwallenv', 'pendulum'):
    static_fns[_d] = StaticFns(_d, TERM_HALFCHEETAH)


def term_kind_of(config):
    """Map a StaticFns-like object (ours, or the reference's class) to a device kind."""
    if hasattr(config, 'term_kind'):
        return config.term_kind
    mod = getattr(config, '__module__', '') or ''
    for name, fns in sorted(static_fns.items(), key=lambda kv: -len(kv[0])):   # longest suffix first
        if mod.endswith(name):
            return fns.term_kind
    raise ValueError('no device termination rule for %r (supported: %s)' % (config, list(static_fns)))
