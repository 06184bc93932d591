"""simple_run-style driver (simple_run/main.py:146-225) for the MI355X path.

    python -m mopo_amd.run --config examples.config.d4rl.halfcheetah_mixed \
        --data halfcheetah-medium-replay-v0.npz --model-dir models/ --epochs 10

``--data``: local qlearning_dataset arrays (d4rl downloads are unavailable offline).
``--model-dir``: directory holding '<model_name>.mat' (bnn.py:276-281); without it the ensemble
keeps its initial weights (ensemble training is a later-round item).
"""
import argparse
import json


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--config', required=True)
    p.add_argument('--data', required=True)
    p.add_argument('--model-dir', default=None)
    p.add_argument('--epochs', type=int, default=None)
    p.add_argument('--seed', type=int, default=88)                 # simple_run/base.py run_params
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
    algo = from_config(params, pool, static_fns[params['domain']], model_load_dir=a.model_dir, seed=a.seed)
    for diag in algo.train(a.epochs):
        print(json.dumps({k: float(v) for k, v in diag.items()}), flush=True)


if __name__ == '__main__':
    main()
