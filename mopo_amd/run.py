"""simple_run-style driver (simple_run/main.py:146-225) for the MI355X path.

    python -m mopo_amd.run --config examples.config.d4rl.halfcheetah_mixed \
        --data halfcheetah-medium-replay-v0.npz --model-dir models/ --epochs 10

``--data``: local qlearning_dataset arrays (d4rl downloads are unavailable offline).
``--model-dir``: directory holding '<model_name>.mat' (bnn.py:276-281); without it the ensemble
is trained from its initial weights to early stopping first (mopo.py:526-531).
``--ensemble-dtype`` / ``--actor-dtype``: the forward arithmetic (mopo_amd.bnn.DTYPES).
"""
import argparse
import json

from .bnn import DEFAULT_ENSEMBLE_DTYPE, DTYPES


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--config', required=True)
    p.add_argument('--data', required=True)
    p.add_argument('--model-dir', default=None)
    p.add_argument('--epochs', type=int, default=None)
    p.add_argument('--seed', type=int, default=88)                 # simple_run/base.py run_params
    p.add_argument('--ensemble-dtype', default=None, choices=DTYPES,
                   help='ensemble forward arithmetic (default: the config kwarg ensemble_dtype, else %s)'
                        % DEFAULT_ENSEMBLE_DTYPE)
    p.add_argument('--actor-dtype', default=None, choices=('fp32', 'bf16x6', 'f16x3'),
                   help='rollout policy forward (default: the ensemble dtype for fp32 and bf16x6, else f16x3)')
    a = p.parse_args(argv)
    from .config import DIMS, get_params
    from .loader import restore_pool
    from .mopo import from_config
    from .replay_pool import SimpleReplayPool
    from .static import static_fns
    params = get_params(a.config)
    obs_dim, act_dim = DIMS[params['domain']]
    pool = SimpleReplayPool(obs_dim=obs_dim, act_dim=act_dim, max_size=int(1e6))   # simple_run/base.py:267-272
    restore_pool(pool, a.data)
    over = {k: v for k, v in (('ensemble_dtype', a.ensemble_dtype), ('actor_dtype', a.actor_dtype)) if v}
    algo = from_config(params, pool, static_fns[params['domain']], model_load_dir=a.model_dir, seed=a.seed, **over)
    for diag in algo.train(a.epochs):
        print(json.dumps({k: float(v) for k, v in diag.items()}), flush=True)


if __name__ == '__main__':
    main()
