"""Experiment configs: the reference's ``examples/config/...`` modules, or their restatement.

``get_params(name)`` follows examples/development/__init__.py:19-22 + base.py:221-257: the module
named by ``name`` is imported and its ``params`` dict read, then the MOPO algorithm defaults
(base.py:45-57 ``ALGORITHM_PARAMS_ADDITIONAL['MOPO']``) are deep-merged over it exactly as
``get_variant_spec_base`` does (``deep_update(params, ADDITIONAL)``: the additional kwargs win).
Keys the reference reads from elsewhere (``network_kwargs`` / ``hidden_dim`` / ``n_epochs``,
simple_run/base.py:44-67) are filled in underneath when the module does not set them.

A user's own module (any importable path holding ``params``) therefore works as in the reference.
When the module cannot be imported -- the reference's ``examples`` package is not installed here --
the D4RL names fall back to ``TASKS``, a restatement of examples/config/d4rl/*.py (base.py:1-28,
base_mopo.py:1-8, e.g. halfcheetah_mixed.py:3-14).
"""
import copy
import importlib

BASE = {
    'type': 'MOPO', 'universe': 'gym', 'log_dir': './ray_mopo/',
    'kwargs': {
        'epoch_length': 1000, 'train_every_n_steps': 1, 'n_train_repeat': 1, 'eval_render_mode': None,
        'eval_n_episodes': 10, 'eval_deterministic': True, 'discount': 0.99, 'tau': 5e-3, 'reward_scale': 1.0,
        'model_train_freq': 1000, 'model_retain_epochs': 5, 'rollout_batch_size': 50e3, 'deterministic': False,
        'num_networks': 7, 'num_elites': 5, 'real_ratio': 0.05, 'target_entropy': -3, 'max_model_t': None,
        # base_mopo.py
        'separate_mean_var': True, 'penalty_learned_var': True,
    },
}

# examples/development/base.py:45-57 (deep-merged OVER the config module's params)
ADDITIONAL = {'type': 'MOPO', 'kwargs': {
    'reparameterize': True, 'lr': 3e-4, 'target_update_interval': 1, 'tau': 5e-3, 'store_extra_policy_info': False,
    'action_prior': 'uniform', 'n_initial_exploration_steps': 5000}}

# simple_run/base.py:44-67: filled in UNDER the module's params (a module may override them)
DEFAULTS = {'kwargs': {'network_kwargs': {'hidden_sizes': [256, 256], 'activation': 'relu', 'output_activation': None},
                       'hidden_dim': 200, 'n_epochs': 1000}}

# (domain, task, exp_name, pool_load_path, pool_load_max_size, rollout_length, penalty_coeff)
TASKS = {
    'halfcheetah_mixed': ('halfcheetah', 'medium-replay-v0', 'halfcheetah_medium_replay',
                          'd4rl/halfcheetah-medium-replay-v0', 101000, 5, 1.0),
    'halfcheetah_medium': ('halfcheetah', 'medium-v0', 'halfcheetah_medium', 'd4rl/halfcheetah-medium-v0',
                           int(1e6), 1, 1.0),
    'halfcheetah_medium_expert': ('halfcheetah', 'medium-expert-v0', 'halfcheetah_medium_expert',
                                  'd4rl/halfcheetah-medium-expert-v0', 2 * 10 ** 6, 5, 5.0),
    'halfcheetah_random': ('halfcheetah', 'random-v0', 'halfcheetah_random', 'd4rl/halfcheetah-random-v0',
                           int(1e6), 5, 0.5),
    'walker2d_mixed': ('walker2d', 'medium-replay-v0', 'walker2d_medium_replay', 'd4rl/walker2d-medium-replay-v0',
                       100930, 1, 1.0),
    'walker2d_medium': ('walker2d', 'medium-v0', 'walker2d_medium', 'd4rl/walker2d-medium-v0', int(1e6), 5, 5.0),
    'walker2d_medium_expert': ('walker2d', 'medium-expert-v0', 'walker2d_medium_expert',
                               'd4rl/walker2d-medium-expert-v0', 2 * 10 ** 6, 1, 2.0),
    'walker2d_random': ('walker2d', 'random-v0', 'walker2d_random', 'd4rl/walker2d-random-v0', int(1e6), 1, 1.0),
    'hopper_mixed': ('hopper', 'medium-replay-v0', 'hopper_medium_replay', 'd4rl/hopper-mixed-v0', 200920, 5, 1.0),
    'hopper_medium': ('hopper', 'medium-v0', 'hopper_medium', 'd4rl/hopper-medium-v0', int(1e6), 5, 5.0),
    'hopper_medium_expert': ('hopper', 'medium-expert-v0', 'hopper_medium_expert', 'd4rl/hopper-medium-expert-v0',
                             2 * 10 ** 6, 5, 1.0),
    'hopper_random': ('hopper', 'random-v0', 'hopper_random', 'd4rl/hopper-random-v0', int(1e6), 5, 1.0),
}

DIMS = {'halfcheetah': (17, 6), 'walker2d': (17, 6), 'hopper': (11, 3)}


def deep_update(d, *updates):
    """softlearning/misc/utils.py deep_update: a copy of ``d`` with each update merged in recursively
    (nested dicts merge key by key, anything else is replaced)."""
    d = copy.deepcopy(d)
    for u in updates:
        for k, v in u.items():
            if isinstance(v, dict) and isinstance(d.get(k), dict):
                d[k] = deep_update(d[k], v)
            else:
                d[k] = copy.deepcopy(v)
    return d


def _restated(key):
    domain, task, exp, path, max_size, length, coeff = TASKS[key]
    p = copy.deepcopy(BASE)
    p.update({'domain': domain, 'task': task, 'exp_name': exp})
    p['kwargs'].update({'pool_load_path': path, 'pool_load_max_size': max_size, 'rollout_length': length,
                        'penalty_coeff': coeff})
    return p


def load_module_params(name, params_name='params'):
    """examples/development/__init__.py:19-22: ``importlib.import_module(name).params``; None when
    the module itself does not exist (an import error raised INSIDE an existing module propagates)."""
    try:
        module = importlib.import_module(name)
    except ModuleNotFoundError as e:
        # missing: the module itself or one of its parent packages; anything else came from its body
        if e.name is None or not (name == e.name or name.startswith(e.name + '.')):
            raise
        return None
    if not hasattr(module, params_name):
        raise AttributeError('config module %r has no %r dict' % (name, params_name))
    return copy.deepcopy(dict(getattr(module, params_name)))


def get_params(name):
    """The merged experiment dict MOPO is built from (see the module docstring)."""
    params = load_module_params(name) if '.' in name or name not in TASKS else None
    if params is None:
        key = name.split('.')[-1]
        if key not in TASKS:
            raise KeyError('config %r: no importable module of that name and not one of the restated '
                           'D4RL configs (%s)' % (name, sorted(TASKS)))
        params = _restated(key)
    for k in ('domain', 'task', 'exp_name'):
        if k not in params:
            raise KeyError('config %r: params has no %r' % (name, k))
    p = deep_update(DEFAULTS, params, ADDITIONAL)
    # softlearning/algorithms/utils.py:43-48: model_name = exp_name with '-' + '_smv' + '_1_0' (always set)
    p['kwargs']['model_name'] = (p['exp_name'].replace('_', '-') +
                                 ('_smv' if p['kwargs'].get('separate_mean_var') else '') + '_1_0')
    return p
