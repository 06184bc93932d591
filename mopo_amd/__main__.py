"""``mopo`` console entry point (softlearning/scripts/console_scripts.py:51-93) for the MI355X path.

    python -m mopo_amd run_local examples.development \\
        --config=examples.config.d4rl.halfcheetah_mixed --gpus=1 --trial-gpus=1 --data=hc.npz
    python -m mopo_amd run_example_dry examples.development --config=examples.config.d4rl.halfcheetah_mixed

Mirrors the reference CLI (``run_local`` / ``run_example_dry`` / ``run_example_debug`` with the
examples/utils.py:90-290 flags) without ray/tune: ``run_local`` trains ``--num-samples`` seeds one
after the other in this process, each through ``mopo_amd.run`` (the simple_run-style driver).  The
ray resource flags (``--cpus``, ``--gpus``, ``--trial-*``, ``--resources*``, ``--with-server`` ...)
are accepted and ignored: one process drives one GPU here (multi-GPU is torchrun, see bench.py).
Offline additions: ``--data`` (local qlearning_dataset .npz: d4rl downloads are unavailable) --
or ``$D4RL_DATASET_DIR/<task>.npz`` named after the config's ``pool_load_path`` -- ``--model-dir``
(``<model_name>.mat``, bnn.py:276-281), ``--epochs`` and ``--ensemble-dtype`` / ``--actor-dtype``
(the forward arithmetic; default f16x3, held to the fp32 parity tolerances).  ``--config`` is any
importable module holding a ``params`` dict (examples/development/__init__.py:19-22), or one of the
restated D4RL config names when the reference's ``examples`` package is not installed.
"""
import argparse
import json
import os
import sys

from .bnn import DTYPES, default_ensemble_dtype

EXAMPLES = ('examples.development',)
COMMANDS = ('run_local', 'run_example_dry', 'run_example_debug')


def get_parser():
    """examples/utils.py:90-290 (the flags this path reads, plus the ray ones it accepts)."""
    p = argparse.ArgumentParser(prog='mopo')
    p.add_argument('--config', required=True)
    p.add_argument('--seed', type=int, default=88)            # simple_run/base.py run_params
    p.add_argument('--num-samples', type=int, default=1)
    p.add_argument('--checkpoint-frequency', type=int, default=None)
    p.add_argument('--checkpoint-at-end', type=str, default=None)
    p.add_argument('--data', default=None)
    p.add_argument('--model-dir', default=None)
    p.add_argument('--epochs', type=int, default=None)
    p.add_argument('--ensemble-dtype', default=None, choices=DTYPES)
    p.add_argument('--actor-dtype', default=None, choices=('fp32', 'bf16x6', 'f16x3'))
    for f in ('--cpus', '--gpus', '--trial-cpus', '--trial-extra-cpus', '--max-failures'):
        p.add_argument(f, type=int, default=None)
    for f in ('--trial-gpus', '--trial-extra-gpus'):
        p.add_argument(f, type=float, default=None)
    for f in ('--resources', '--resources-per-trial', '--include-webui', '--temp-dir', '--upload-dir',
              '--trial-name-template', '--restore', '--with-server', '--universe', '--domain', '--task',
              '--algorithm', '--exp-name', '--mode'):
        p.add_argument(f, type=str, default=None)
    return p


def resolve_data(args, params):
    """--data, else $D4RL_DATASET_DIR/<basename of pool_load_path>.npz (e.g. halfcheetah-medium-replay-v0)."""
    if args.data:
        return args.data
    root = os.environ.get('D4RL_DATASET_DIR')
    name = os.path.basename(params['kwargs']['pool_load_path'])
    if root and os.path.exists(os.path.join(root, name + '.npz')):
        return os.path.join(root, name + '.npz')
    raise SystemExit('mopo: no dataset for %s -- pass --data=<qlearning_dataset .npz> or set D4RL_DATASET_DIR '
                     '(d4rl downloads need the network)' % name)


def variant_spec(args):
    """The resolved experiment (the part of examples/development/base.py:get_variant_spec this path uses)."""
    from .config import get_params
    params = get_params(args.config)
    kw = params['kwargs']
    for k in ('ensemble_dtype', 'actor_dtype'):
        if getattr(args, k) is not None:
            kw[k] = getattr(args, k)
    kw.setdefault('ensemble_dtype', default_ensemble_dtype(kw.get('hidden_dim', 200)))
    seeds = [args.seed + i for i in range(max(args.num_samples, 1))]
    return {'algorithm_params': params, 'run_params': {'seeds': seeds, 'checkpoint_frequency': args.checkpoint_frequency},
            'model_dir': args.model_dir, 'epochs': args.epochs}


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if len(argv) < 2 or argv[0] not in COMMANDS:
        print('usage: python -m mopo_amd {%s} examples.development --config=<module> [flags]' % '|'.join(COMMANDS),
              file=sys.stderr)
        return 2
    cmd, example = argv[0], argv[1]
    if example not in EXAMPLES:
        print('mopo: unknown example %r (have: %s)' % (example, ', '.join(EXAMPLES)), file=sys.stderr)
        return 2
    args = get_parser().parse_args(argv[2:])
    spec = variant_spec(args)
    if cmd == 'run_example_dry':                              # instrument.py:173-202
        print(json.dumps(spec, indent=1, default=str))
        print('number of trials: %d' % len(spec['run_params']['seeds']))
        return 0
    from . import run
    data = resolve_data(args, spec['algorithm_params'])
    for seed in spec['run_params']['seeds']:                  # tune's num_samples, run sequentially
        rargv = ['--config', args.config, '--data', data, '--seed', str(seed)]
        if args.model_dir:
            rargv += ['--model-dir', args.model_dir]
        if args.epochs is not None:
            rargv += ['--epochs', str(args.epochs)]
        for k in ('ensemble_dtype', 'actor_dtype'):
            if getattr(args, k) is not None:
                rargv += ['--' + k.replace('_', '-'), getattr(args, k)]
        run.main(rargv)
    return 0


if __name__ == '__main__':
    sys.exit(main())
