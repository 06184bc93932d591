"""The reference's experiment configs (``examples/config/d4rl/*.py``), as plain dicts.

Values follow examples/config/d4rl/base.py:1-28, base_mopo.py:1-8 and the per-task files
(e.g. halfcheetah_mixed.py:3-14); simple_run/base.py:44-67 supplies lr / tau / network_kwargs.
``get_params('halfcheetah_mixed')`` returns the merged kwargs MOPO is built from; a module path
in the reference's form ('examples.config.d4rl.halfcheetah_mixed') is accepted too.
"""
import copy

BASE = {
    'type': 'MOPO', 'universe': 'gym', 'log_dir': './ray_mopo/',
    'kwargs': {
        'epoch_length': 1000, 'train_every_n_steps': 1, 'n_train_repeat': 1, 'eval_render_mode': None,
        'eval_n_episodes': 10, 'eval_deterministic': True, 'discount': 0.99, 'tau': 5e-3, 'reward_scale': 1.0,
        'model_train_freq': 1000, 'model_retain_epochs': 5, 'rollout_batch_size': 50e3, 'deterministic': False,
        'num_networks': 7, 'num_elites': 5, 'real_ratio': 0.05, 'target_entropy': -3, 'max_model_t': None,
        # base_mopo.py
        'separate_mean_var': True, 'penalty_learned_var': True,
        # simple_run/base.py ALGORITHM_PARAMS_ADDITIONAL
        'reparameterize': True, 'lr': 3e-4, 'target_update_interval': 1, 'store_extra_policy_info': False,
        'action_prior': 'uniform', 'n_initial_exploration_steps': 5000,
        'network_kwargs': {'hidden_sizes': [256, 256], 'activation': 'relu', 'output_activation': None},
        'hidden_dim': 200, 'n_epochs': 1000,
    },
}

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


def get_params(name):
    key = name.split('.')[-1]
    if key not in TASKS:
        raise KeyError('unknown config %r (known: %s)' % (name, sorted(TASKS)))
    domain, task, exp, path, max_size, length, coeff = TASKS[key]
    p = copy.deepcopy(BASE)
    p.update({'domain': domain, 'task': task, 'exp_name': exp})
    p['kwargs'].update({'pool_load_path': path, 'pool_load_max_size': max_size, 'rollout_length': length,
                        'penalty_coeff': coeff})
    # softlearning/algorithms/utils.py:45-49: model_name = exp_name with '-' + '_smv' + '_1_0'
    p['kwargs']['model_name'] = exp.replace('_', '-') + ('_smv' if p['kwargs']['separate_mean_var'] else '') + '_1_0'
    return p
