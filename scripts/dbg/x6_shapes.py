"""bf16x6 (and f16x3) ensemble predict vs the oracle over shapes: max scaled error per case."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle import bnn as obnn  # noqa: E402
from mopo_amd.bnn import BNN  # noqa: E402

for E in (7, 32):
    for H in (32, 64, 200):
        for f64 in (False, True):
            for dt in (sys.argv[1:] or ['bf16x6', 'f16x3', 'fp32']):
                rs = np.random.RandomState(E + H)
                p = obnn.init_params(E, 17, 6, hidden=H, seed=E * 7 + H)
                x = rs.normal(size=(300, 23)) * (3.0 if f64 else 1.0)
                if not f64:
                    x = x.astype(np.float32)
                m = BNN({'name': 't', 'num_networks': E, 'num_elites': 5, 'separate_mean_var': True, 'obs_dim': 17,
                         'act_dim': 6, 'hidden_dim': H, 'dtype': dt}).set_params(obnn.to_mat_list(p))
                mean, var = m.predict(x, factored=True)
                rm, rv = obnn.forward(p, np.asarray(x, np.float64), dtype=np.float64)
                err = np.abs(mean - rm) / (1 + np.abs(rm))
                print('E=%2d H=%3d f64=%d %-7s mean err %.3g  worst member %d' % (E, H, f64, dt, err.max(),
                                                                                int(err.max(axis=(1, 2)).argmax())),
                      flush=True)
