"""FakeEnv: the model environment stepped by MOPO rollouts, on the MI355X.

Mirrors ``FakeEnv`` (mopo/models/fake_env.py:4-131): same constructor, same ``step`` signature
and return ``(next_obs, penalized_rewards, terminals, info)`` with the same info keys.  The whole
step (ensemble forward + residual + sampling + elite gather + penalty + termination) runs in
``mopo_fakeenv_step`` (csrc/bnn.hip + csrc/fakeenv.hip).

RNG: ``rng='numpy'`` (default) consumes numpy's global legacy stream exactly like the reference
-- ``np.random.normal(size=(E, B, D))`` then ``model.random_inds(B)`` -- so results match the
reference for the same seed; only the selected member's noise is shipped to the device.
numpy inputs return numpy outputs; torch CUDA inputs return torch CUDA outputs.
"""
import numpy as np

from . import _lib as L
from .static import term_kind_of


class FakeEnv:
    def __init__(self, model, config, penalty_coeff=0., penalty_learned_var=False,
                 penalty_learned_var_random=False):
        self.model = model
        self.config = config
        self.penalty_coeff = penalty_coeff
        self.penalty_learned_var = penalty_learned_var
        self.penalty_learned_var_random = penalty_learned_var_random
        self.term_kind = term_kind_of(config)

    def step(self, obs, act, deterministic=False, noise=None, model_inds=None, stream=None):
        import torch
        assert len(obs.shape) == len(act.shape)                              # fake_env.py:38
        is_np = isinstance(obs, np.ndarray)
        single = len(obs.shape) == 1
        if single:
            obs, act = obs[None], act[None]
        dev = torch.device('cuda')
        to = (lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)) if is_np else (lambda x: x.contiguous())
        o = to(obs)
        if o.dtype not in (torch.float32, torch.float64):
            o = o.float()
        a = to(act).float().contiguous()
        B = o.shape[0]
        E, O, D = self.model.num_nets, self.model.obs_dim, self.model.obs_dim + 1
        noise_sel = inds = None
        if not deterministic:
            # the reference's RNG order (fake_env.py:72 then 77 -> bnn.py:343)
            if noise is None:
                noise = np.random.normal(size=(E, B, D))
            if model_inds is None:
                model_inds = self.model.random_inds(B)
            mi = np.asarray(model_inds, np.int64) if not torch.is_tensor(model_inds) else model_inds
            if torch.is_tensor(noise):
                noise_sel = noise[torch.as_tensor(mi, device=noise.device), torch.arange(B, device=noise.device)]
                noise_sel = noise_sel.to(dev, torch.float64).contiguous()
            else:
                noise_sel = torch.from_numpy(np.ascontiguousarray(noise[mi, np.arange(B)], np.float64)).to(dev)
            inds = torch.as_tensor(mi, dtype=torch.int64).to(dev)
        f64 = dict(dtype=torch.float64, device=dev)
        f32 = dict(dtype=torch.float32, device=dev)
        out = {
            'next_obs': torch.empty((B, O), **f64), 'rew': torch.empty((B,), **f64),
            'term': torch.empty((B,), dtype=torch.uint8, device=dev), 'penalty': torch.empty((B,), **f32),
            'unpen': torch.empty((B,), **f64), 'imean': torch.empty((B, D + 1), **f32),
            'istd': torch.empty((B, D + 1), **f32), 'logp': torch.empty((B,), **f64),
            'dev': torch.empty((B,), **f32), 'emean': torch.empty((E, B, D), **f32),
            'evar': torch.empty((E, B, D), **f32)}
        args = L.FakeEnvArgs(
            d_obs=L.ptr(o), obs_f64=int(o.dtype == torch.float64), d_act=L.ptr(a), B=B,
            d_noise_sel=L.ptr(noise_sel), d_model_inds=L.ptr(inds), deterministic=int(bool(deterministic)),
            penalty_coeff=float(self.penalty_coeff), penalty_learned_var=int(bool(self.penalty_learned_var)),
            term_kind=self.term_kind, d_next_obs=L.ptr(out['next_obs']), d_rewards=L.ptr(out['rew']),
            d_terminals=L.ptr(out['term']), d_penalty=L.ptr(out['penalty']), d_unpenalized=L.ptr(out['unpen']),
            d_info_mean=L.ptr(out['imean']), d_info_std=L.ptr(out['istd']), d_log_prob=L.ptr(out['logp']),
            d_dev=L.ptr(out['dev']), d_ens_mean=L.ptr(out['emean']), d_ens_var=L.ptr(out['evar']))
        L.check(L.lib().mopo_fakeenv_step(self.model.handle, args, L.stream_ptr(stream)))
        next_obs = out['next_obs']
        rew = out['rew'][:, None]
        term = out['term'].bool()[:, None]
        pen = out['penalty'][:, None] if self.penalty_coeff != 0 else None
        unpen = out['unpen'][:, None]
        info = {'mean': out['imean'], 'std': out['istd'], 'log_prob': out['logp'], 'dev': out['dev'],
                'unpenalized_rewards': unpen, 'penalty': pen, 'penalized_rewards': rew}
        if is_np:
            cv = lambda t: None if t is None else t.cpu().numpy()
            next_obs, rew, term = cv(next_obs), cv(rew), cv(term)
            info = {k: cv(v) for k, v in info.items()}
        if single:  # fake_env.py:121-127
            next_obs, rew, term = next_obs[0], rew[0], term[0]
            info['mean'], info['std'] = info['mean'][0], info['std'][0]
            info['unpenalized_rewards'], info['penalized_rewards'] = info['unpenalized_rewards'][0], info['penalized_rewards'][0]
        return next_obs, rew, term, info

    def close(self):
        pass
