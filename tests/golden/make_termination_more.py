"""Termination fixtures for the domains beyond halfcheetah / walker2d / hopper, by EXECUTING the
reference's own ``mopo/static/<domain>.py`` ``StaticFns.termination_fn`` (numpy only).

Run in the build container only (needs /root/reference; nothing here runs on the GPU box):

    python tests/golden/make_termination_more.py

Output: tests/golden/termination_more.npz -- ``next_obs`` [n, 17] (f64) and ``done_<domain>`` per
domain, inputs and expected outputs only.  pendulum.py returns float zeros; stored as returned.
"""
import importlib.util
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = '/root/reference'
DOMAINS = ('ant', 'antangle', 'humanoid', 'halfcheetahjump', 'halfcheetahvel', 'halfcheetahveljump',
           'point2denv', 'point2dwallenv', 'pendulum')


def _static(domain):
    spec = importlib.util.spec_from_file_location('ref_static_' + domain,
                                                  os.path.join(REF, 'mopo/static/%s.py' % domain))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.StaticFns


def make_inputs(n=1024, O=17, seed=11):
    rs = np.random.RandomState(seed)
    nobs = rs.normal(size=(n, O))
    nobs[: n // 2, 0] = rs.uniform(-0.2, 1.4, size=n // 2)      # around ant's [0.2, 1.0]
    nobs[n // 2:, 0] = rs.uniform(0.6, 2.4, size=n - n // 2)     # around humanoid's [1.0, 2.0]
    # exact boundaries, their f64 neighbours, and non-finite entries in and out of column 0
    edge = [0.2, 1.0, 2.0, np.nextafter(0.2, 0), np.nextafter(0.2, 1), np.nextafter(1.0, 0),
            np.nextafter(1.0, 2), np.nextafter(2.0, 1), np.nextafter(2.0, 3), 0.0, -0.0]
    nobs[:len(edge), 0] = edge
    k = len(edge)
    nobs[k, 0] = np.nan; nobs[k + 1, 0] = np.inf; nobs[k + 2, 0] = -np.inf
    nobs[k + 3, 0] = 0.5; nobs[k + 3, 5] = np.nan
    nobs[k + 4, 0] = 1.5; nobs[k + 4, 16] = np.inf
    nobs[k + 5, 0] = 0.7; nobs[k + 5, 1] = -np.inf
    nobs[k + 6, 0] = np.float32(0.2)                               # f32-rounded boundary (> 0.2 in f64)
    nobs[k + 7, 0] = np.float32(1.0) + 0.0
    return nobs


def main():
    nobs = make_inputs()
    obs = np.zeros_like(nobs); act = np.zeros((len(nobs), 6))
    out = {'next_obs': nobs}
    for d in DOMAINS:
        out['done_' + d] = _static(d).termination_fn(obs, act, nobs)
    np.savez_compressed(os.path.join(HERE, 'termination_more.npz'), **out)
    print({d: int(np.asarray(out['done_' + d], bool).sum()) for d in DOMAINS})


if __name__ == '__main__':
    main()
