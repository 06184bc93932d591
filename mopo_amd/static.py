"""Per-domain termination functions (``mopo.static``), as device termination kinds.

Reference: mopo/static/__init__.py:7-25 builds ``{domain: StaticFns}``; the rules are
mopo/static/halfcheetah.py:6-11, walker2d.py:6-17, hopper.py:6-18.  On the accelerated path the
rule runs inside the FakeEnv kernels (``term_fn`` in csrc/internal.h) selected by ``term_kind``;
``termination_fn`` here is the same rule on torch tensors for callers that use it directly.
"""
import numpy as np

TERM_HALFCHEETAH, TERM_WALKER2D, TERM_HOPPER = 0, 1, 2


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
        else:
            done = torch.zeros(x.shape[0], dtype=torch.bool, device=x.device)
        done = done[:, None]
        return done.cpu().numpy() if is_np else done


static_fns = {
    'halfcheetah': StaticFns('halfcheetah', TERM_HALFCHEETAH),
    'walker2d': StaticFns('walker2d', TERM_WALKER2D),
    'hopper': StaticFns('hopper', TERM_HOPPER),
}


def term_kind_of(config):
    """Map a StaticFns-like object (ours, or the reference's class) to a device kind."""
    if hasattr(config, 'term_kind'):
        return config.term_kind
    mod = getattr(config, '__module__', '') or ''
    for name, fns in static_fns.items():
        if mod.endswith(name):
            return fns.term_kind
    raise ValueError('no device termination rule for %r (supported: %s)' % (config, list(static_fns)))
