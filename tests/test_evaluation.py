"""Evaluation rollouts and perf/NormalizedReturn (rl_algorithm.py:258-304, samplers/utils.py:36-92,
mopo.py:115-123, 575-629).  The environment is a synthetic gym-API object (no MuJoCo in this image):
the host metrics are checked against hand computation on CPU; on the GPU the device policy's
deterministic actions are checked against the oracle actor, and a MOPO epoch with an evaluation
environment against a host re-run of the same episodes with the oracle's tanh(mu)."""
import numpy as np
import pytest

from mopo_amd import evaluation as ev


class ToyEnv:
    """17-d state, 6-d action; episode e (counted over resets) ends after 8 + 3 (e % 4) steps."""

    def __init__(self, seed=0):
        self.rs = np.random.RandomState(seed)
        self.n_resets = 0

    def reset(self):
        self.len = 8 + 3 * (self.n_resets % 4)
        self.n_resets += 1
        self.t = 0
        self.s = self.rs.normal(size=17).astype(np.float32)
        return self.s.copy()

    def step(self, a):
        a = np.asarray(a, np.float64)
        self.t += 1
        s = 0.9 * self.s + 0.1 * np.concatenate([a, a, a[:5]])
        r = float(a.sum() - 0.01 * np.sum(s ** 2))
        self.s = s.astype(np.float32)
        return self.s.copy(), r, self.t >= self.len, {'t': self.t}


class HostPolicy:
    def __init__(self, fn):
        self.fn = fn

    def actions(self, obs):
        return self.fn(obs)


def test_env_name_and_ref_scores():
    assert ev.env_name_of('halfcheetah-medium-replay_smv_1_0') == 'halfcheetah-medium-replay-v0'
    assert ev.env_name_of('hopper-medium_1_0') == 'hopper-medium-v0'
    assert ev.ref_scores('walker2d-medium-expert_smv_1_0') == (1.629008, 4592.3)
    assert ev.ref_scores('not-a-task_1_0') == (0.0, 0.0)


def test_rollout_and_metrics_by_hand():
    env = ToyEnv()
    paths = ev.evaluation_paths(env, HostPolicy(lambda o: np.full((o.shape[0], 6), 0.5)), 5, 12)
    lengths = [len(p['rewards']) for p in paths]
    assert lengths == [8, 11, 12, 12, 8]          # 14 and 17-step episodes cut at path_length
    assert paths[0]['observations'].shape == (8, 17) and paths[0]['actions'].shape == (8, 6)
    assert paths[0]['terminals'][-1, 0] and not paths[2]['terminals'][-1, 0]
    np.testing.assert_array_equal(paths[1]['observations'][1:], paths[1]['next_observations'][:-1])
    m = ev.evaluate_rollouts(paths)
    rets = [p['rewards'].sum() for p in paths]
    assert list(m) == ['return-average', 'return-min', 'return-max', 'return-std', 'episode-length-avg',
                       'episode-length-min', 'episode-length-max', 'episode-length-std']
    assert m['return-average'] == pytest.approx(np.mean(rets)) and m['return-std'] == pytest.approx(np.std(rets))
    assert (m['episode-length-min'], m['episode-length-max']) == (8, 12)
    perf = ev.perf_metrics(m, -280.178953, 12135.0)
    assert perf['perf/NormalizedReturn'] == pytest.approx((np.mean(rets) + 280.178953) / (12135.0 + 280.178953))
    assert 'perf/NormalizedReturn' not in ev.perf_metrics(m, 0.0, 0.0)
    assert ev.evaluation_paths(env, None, 0, 10) == []


def _flat_to_list(flat, O, A, H):
    from oracle import sac as osac
    out, o = [], 0
    for shp in osac.param_shapes(O, A, H):
        n = int(np.prod(shp))
        out.append(np.asarray(flat[o:o + n], np.float64).reshape(shp))
        o += n
    return out


@pytest.mark.gpu
def test_device_policy_deterministic_vs_oracle():
    import torch
    from oracle import sac as osac
    O, A, H = 17, 6, 256
    P = osac.init_params(O, A, H, seed=5)
    P[5] = np.linspace(-0.5, 0.5, A)
    flat = torch.from_numpy(np.concatenate([p.ravel() for p in P]).astype(np.float32)).cuda()
    obs = np.random.RandomState(1).normal(size=(37, O)).astype(np.float32)
    got = ev.DevicePolicy(flat, O, A, H).actions(obs)
    mu_ref = osac.actor_act(osac.split(P)[0], obs.astype(np.float64), np.zeros((37, A)))[1]
    assert np.abs(got - mu_ref).max() < 2e-6
    stoch = ev.DevicePolicy(flat, O, A, H, deterministic=False).actions(obs)
    assert np.abs(stoch - mu_ref).max() > 1e-3 and np.all(np.abs(stoch) <= 1)


@pytest.mark.gpu
def test_mopo_epoch_with_evaluation_environment():
    from oracle import sac as osac
    from mopo_amd.config import get_params
    from mopo_amd.mopo import from_config
    from mopo_amd.replay_pool import SimpleReplayPool
    from mopo_amd.static import static_fns
    rs = np.random.RandomState(0)
    n = 3000
    obs = rs.normal(size=(n, 17)).astype(np.float32)
    pool = SimpleReplayPool(obs_dim=17, act_dim=6, max_size=n)
    pool.add_samples({'observations': obs, 'actions': rs.uniform(-1, 1, (n, 6)).astype(np.float32),
                      'next_observations': obs + 0.1 * rs.normal(size=(n, 17)).astype(np.float32),
                      'rewards': rs.normal(size=(n, 1)).astype(np.float32), 'terminals': np.zeros((n, 1), bool)})
    algo = from_config(get_params('examples.config.d4rl.halfcheetah_mixed'), pool, static_fns['halfcheetah'],
                       rollout_batch_size=1000, epoch_length=50, model_train_freq=50, max_model_t=None,
                       evaluation_environment=ToyEnv(seed=3), eval_n_episodes=4, max_path_length=12)
    d = next(iter(algo.train(1)))
    # host re-run: same env seed, the trained policy's tanh(mu) from the oracle
    flat = algo._sac.get_params()[0].cpu().numpy()
    Ppi = osac.split(_flat_to_list(flat, 17, 6, 256))[0]
    pol = HostPolicy(lambda o: osac.actor_act(Ppi, o.astype(np.float64), np.zeros((o.shape[0], 6)))[1])
    ref = ev.evaluate_rollouts(ev.evaluation_paths(ToyEnv(seed=3), pol, 4, 12))
    for k, v in ref.items():
        assert d['evaluation/' + k] == pytest.approx(v, rel=1e-5, abs=1e-5), k
    assert d['perf/AverageReturn'] == d['evaluation/return-average']
    assert d['perf/AverageLength'] == d['evaluation/episode-length-avg']
    assert d['perf/NormalizedReturn'] == pytest.approx((ref['return-average'] + 280.178953) / (12135.0 + 280.178953),
                                                       rel=1e-5)
    assert 'times/evaluation_paths' in d
