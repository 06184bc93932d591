"""GPU: the MOPO host loop (mopo.py:490-648 mirror) runs rollout + SAC epochs on the device path."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_mopo_two_epochs_from_config(tmp_path):
    from mopo_amd.config import get_params
    from mopo_amd.loader import restore_pool
    from mopo_amd.mopo import from_config
    from mopo_amd.replay_pool import SimpleReplayPool
    from mopo_amd.static import static_fns
    rs = np.random.RandomState(0)
    n = 5000
    obs = rs.normal(size=(n, 17)).astype(np.float32)
    np.savez(tmp_path / 'd.npz', observations=obs, actions=rs.uniform(-1, 1, (n, 6)).astype(np.float32),
             next_observations=obs + 0.1 * rs.normal(size=(n, 17)).astype(np.float32),
             rewards=rs.normal(size=n).astype(np.float32), terminals=np.zeros(n, bool))
    pool = SimpleReplayPool(obs_dim=17, act_dim=6, max_size=int(1e6))
    assert restore_pool(pool, str(tmp_path / 'd.npz')) == n and pool.size == n
    params = get_params('examples.config.d4rl.halfcheetah_mixed')
    assert params['kwargs']['model_name'] == 'halfcheetah-medium-replay_smv_1_0'
    algo = from_config(params, pool, static_fns['halfcheetah'], rollout_batch_size=2000, epoch_length=100,
                       model_train_freq=100)
    assert algo._model.dtype == 'f16x3'      # the product default (= bench.py's headline arithmetic)
    diags = list(algo.train(2))
    assert len(diags) == 2
    for d in diags:
        assert d['model/mean_rollout_length'] == 5.0
        assert all(np.isfinite(v) for v in d.values())
    # the dynamics model was trained first (mopo.py:526-531): random init -> to early stopping
    m = algo._model
    assert m._train_epochs >= 6 and d['model/val_loss'] == np.sort(m._holdout_losses)[:5].mean()
    assert len(m._model_inds) == 5
    # model pool sized as mopo.py:693-695: retain 5 x length 5 x 2000 x (100/100)
    assert algo._model_pool._max_size == 5 * 5 * 2000
    assert algo._model_pool.size == 2 * 5 * 2000
    assert algo._num_train_steps == 200


def test_mopo_from_user_config_module(tmp_path, monkeypatch):
    """A user's own config module (examples/development/__init__.py:19-22) drives MOPO: its
    rollout_length / penalty and an ensemble_dtype kwarg reach the rollout."""
    from mopo_amd.config import get_params
    from mopo_amd.mopo import from_config
    from mopo_amd.replay_pool import SimpleReplayPool
    from mopo_amd.static import static_fns
    (tmp_path / 'my_hc_cfg.py').write_text(
        "params = {'type': 'MOPO', 'universe': 'gym', 'domain': 'halfcheetah', 'task': 'mixed',\n"
        "          'exp_name': 'hc_user', 'kwargs': {'rollout_length': 2, 'penalty_coeff': 0.25,\n"
        "          'separate_mean_var': True, 'penalty_learned_var': True, 'num_networks': 7, 'num_elites': 5,\n"
        "          'real_ratio': 0.05, 'target_entropy': -3, 'model_retain_epochs': 5, 'ensemble_dtype': 'fp32'}}\n")
    monkeypatch.syspath_prepend(str(tmp_path))
    rs = np.random.RandomState(1)
    n = 3000
    obs = rs.normal(size=(n, 17)).astype(np.float32)
    pool = SimpleReplayPool(obs_dim=17, act_dim=6, max_size=n)
    pool.add_samples({'observations': obs, 'actions': rs.uniform(-1, 1, (n, 6)), 'rewards': rs.normal(size=(n, 1)),
                      'terminals': np.zeros((n, 1), bool), 'next_observations': obs + 0.1})
    params = get_params('my_hc_cfg')
    algo = from_config(params, pool, static_fns['halfcheetah'], rollout_batch_size=1000, epoch_length=20,
                       model_train_freq=20, max_model_t=5)
    assert algo._model.dtype == 'fp32' and algo.fake_env.penalty_coeff == 0.25
    d = next(algo.train(1))
    assert d['model/mean_rollout_length'] == 2.0 and algo._model_pool.size == 2000


def test_reallocate_model_pool_vs_oracle():
    """MOPO._reallocate_model_pool (mopo.py:689-711) over a rollout-length ramp: the device pool's
    size after every epoch equals the oracle's, and the rows carried into a resized pool (also out of
    a wrapped ring) are bit-identical to the oracle pool's; a shrink below the live row count trips
    the reference's size assert (mopo.py:710) in both."""
    from types import SimpleNamespace
    from mopo_amd.mopo import MOPO
    from oracle import rollout as orl
    O, A = 5, 2
    rs = np.random.RandomState(3)
    stub = SimpleNamespace(_obs_dim=O, _act_dim=A, _rollout_batch_size=40, _epoch_length=10,
                           _model_train_freq=5, _model_retain_epochs=2, _rollout_schedule=[1, 4, 1, 4])
    opool = None
    for epoch, n_add in zip(range(9), [50, 70, 200, 30, 300, 10, 400, 5, 90]):
        stub._epoch = epoch
        MOPO._set_rollout_length(stub)
        if epoch == 6:  # grow out of a wrapped ring: the schedule's max length rises to 6
            stub._rollout_schedule = [0, 1, 1, 6]
            MOPO._set_rollout_length(stub)
        MOPO._reallocate_model_pool(stub)
        opool = orl.reallocate(opool, O, A, stub._rollout_batch_size, stub._epoch_length, stub._model_train_freq,
                               stub._rollout_length, stub._model_retain_epochs)
        assert stub._model_pool._max_size == opool._max_size, epoch
        assert stub._model_pool.size == opool.size, epoch
        got = stub._model_pool.return_all_samples(as_numpy=True)
        ref = opool.return_all_samples()
        for k in ref:
            np.testing.assert_array_equal(got[k].reshape(ref[k].shape), ref[k], err_msg='%s epoch %d' % (k, epoch))
        smp = {'observations': rs.normal(size=(n_add, O)).astype(np.float32),
               'actions': rs.uniform(-1, 1, size=(n_add, A)).astype(np.float32),
               'next_observations': rs.normal(size=(n_add, O)).astype(np.float32),
               'rewards': rs.normal(size=(n_add, 1)).astype(np.float32),
               'terminals': rs.uniform(size=(n_add, 1)) < 0.2}
        stub._model_pool.add_samples(smp)
        opool.add_samples(smp)
    stub._rollout_schedule = [0, 1, 1, 1]
    MOPO._set_rollout_length(stub)
    with pytest.raises(AssertionError):
        MOPO._reallocate_model_pool(stub)
    with pytest.raises(AssertionError):
        orl.reallocate(opool, O, A, stub._rollout_batch_size, stub._epoch_length, stub._model_train_freq,
                       stub._rollout_length, stub._model_retain_epochs)


def test_mopo_rollouts_every_model_train_freq_steps():
    """model_train_freq < epoch_length (mopo.py:554-563): a rollout at timesteps 0, 40, 80 of a 100-step
    epoch, the SAC steps of the timesteps in between (n_train_repeat 2), each rollout under its own
    Philox key; target_update_interval 2 runs through the same loop."""
    import torch
    from mopo_amd.mopo import MOPO
    from mopo_amd.replay_pool import SimpleReplayPool
    from mopo_amd.static import static_fns
    rs = np.random.RandomState(2)
    n = 3000
    obs = rs.normal(size=(n, 17)).astype(np.float32)
    pool = SimpleReplayPool(obs_dim=17, act_dim=6, max_size=n)
    pool.add_samples({'observations': obs, 'actions': rs.uniform(-1, 1, (n, 6)), 'rewards': rs.normal(size=(n, 1)),
                      'terminals': np.zeros((n, 1), bool), 'next_observations': obs + 0.1})
    algo = MOPO(pool, static_fns['halfcheetah'], 17, 6, rollout_batch_size=500, rollout_length=1, epoch_length=100,
                model_train_freq=40, n_train_repeat=2, target_update_interval=2, separate_mean_var=True,
                penalty_coeff=1.0, penalty_learned_var=True, real_ratio=0.05, target_entropy=-3, max_model_t=3)
    seen = []
    orig = algo._rollout_model

    def spy(*a, **k):
        seen.append((algo._epoch, k.get('rollout_key')))
        return orig(*a, **k)
    algo._rollout_model = spy
    d = list(algo.train(2))
    assert seen == [(0, 0), (0, 1), (0, 2), (1, 3), (1, 4), (1, 5)]
    # mopo.py:689-711: rollouts per epoch = 500 * 100 / 40, retained 20 epochs, rollout length 1
    assert algo._model_pool._max_size == 20 * int(1 * 500 * 100 / 40)
    assert algo._model_pool.size == 6 * 500
    assert algo._num_train_steps == 2 * 100 * 2 and d[-1]['train-steps'] == 400
    assert all(np.isfinite(v) for v in d[-1].values())
    rows = algo._model_pool.fields['observations'][:algo._model_pool.size].reshape(6, 500, 17)
    assert not torch.equal(rows[0], rows[1])          # distinct start-row draws per rollout


def test_mopo_real_ratio_one_skips_rollouts():
    """real_ratio = 1.0 (mopo.py:554): no model rollout and no model pool; SAC trains on env rows only."""
    from mopo_amd.mopo import MOPO
    from mopo_amd.replay_pool import SimpleReplayPool
    from mopo_amd.static import static_fns
    rs = np.random.RandomState(3)
    n = 2000
    obs = rs.normal(size=(n, 17)).astype(np.float32)
    pool = SimpleReplayPool(obs_dim=17, act_dim=6, max_size=n)
    pool.add_samples({'observations': obs, 'actions': rs.uniform(-1, 1, (n, 6)), 'rewards': rs.normal(size=(n, 1)),
                      'terminals': np.zeros((n, 1), bool), 'next_observations': obs + 0.1})
    algo = MOPO(pool, static_fns['halfcheetah'], 17, 6, rollout_batch_size=500, rollout_length=1, epoch_length=50,
                model_train_freq=25, separate_mean_var=True, real_ratio=1.0, target_entropy=-3, max_model_t=3)
    calls = []
    orig = algo._rollout_model
    algo._rollout_model = lambda *a, **k: calls.append(k) or orig(*a, **k)
    d = list(algo.train(1))
    assert calls == [] and not hasattr(algo, '_model_pool')
    assert algo._num_train_steps == 50 and all(np.isfinite(v) for v in d[-1].values())
