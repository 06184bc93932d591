"""CPU: the ``mopo`` console mirror (softlearning/scripts/console_scripts.py, examples/utils.py flags)."""
import json
import subprocess
import sys

import pytest

from mopo_amd.__main__ import get_parser, main, resolve_data, variant_spec


def test_dry_run_resolves_the_reference_config(capsys):
    rc = main(['run_example_dry', 'examples.development', '--config=examples.config.d4rl.halfcheetah_mixed',
               '--gpus=1', '--trial-gpus=1', '--checkpoint-frequency=50', '--num-samples=2'])
    assert rc == 0
    out = capsys.readouterr().out
    spec = json.loads(out[:out.rindex('}') + 1])
    kw = spec['algorithm_params']['kwargs']
    # examples/config/d4rl/halfcheetah_mixed.py + base.py + base_mopo.py
    assert (kw['rollout_length'], kw['penalty_coeff'], kw['rollout_batch_size']) == (5, 1.0, 50e3)
    assert kw['pool_load_path'] == 'd4rl/halfcheetah-medium-replay-v0'
    assert spec['run_params']['seeds'] == [88, 89]
    assert 'number of trials: 2' in out


def test_ray_flags_are_accepted():
    a = get_parser().parse_args(['--config=examples.config.d4rl.walker2d_mixed', '--cpus=8', '--gpus=1',
                                 '--trial-gpus=0.5', '--resources={}', '--max-failures=3', '--with-server=False'])
    assert variant_spec(a)['algorithm_params']['domain'] == 'walker2d'


def test_unknown_command_and_missing_data(monkeypatch):
    assert main(['train', 'examples.development']) == 2
    assert main(['run_local', 'examples.nope', '--config=x']) == 2
    monkeypatch.delenv('D4RL_DATASET_DIR', raising=False)
    a = get_parser().parse_args(['--config=examples.config.d4rl.hopper_mixed'])
    with pytest.raises(SystemExit, match='no dataset'):
        resolve_data(a, variant_spec(a)['algorithm_params'])


def test_dataset_dir_lookup(tmp_path, monkeypatch):
    (tmp_path / 'hopper-mixed-v0.npz').write_bytes(b'')
    monkeypatch.setenv('D4RL_DATASET_DIR', str(tmp_path))
    a = get_parser().parse_args(['--config=examples.config.d4rl.hopper_mixed'])
    assert resolve_data(a, variant_spec(a)['algorithm_params']) == str(tmp_path / 'hopper-mixed-v0.npz')


def test_module_entry_point():
    r = subprocess.run([sys.executable, '-m', 'mopo_amd', 'run_example_dry', 'examples.development',
                        '--config=examples.config.d4rl.hopper_medium_expert'], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    assert '"penalty_coeff": 1.0' in r.stdout


def test_console_command_entry_points():
    """setup.py maps the `mopo` console command to mopo_amd.__main__:main (reference setup.py:14-18);
    bin/mopo runs it from a checkout."""
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = open(os.path.join(root, 'setup.py')).read()
    assert "'mopo=mopo_amd.__main__:main'" in src
    out = subprocess.run([sys.executable, os.path.join(root, 'bin', 'mopo'), 'run_example_dry', 'examples.development',
                          '--config=examples.config.d4rl.walker2d_mixed'], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert '"domain": "walker2d"' in out.stdout
