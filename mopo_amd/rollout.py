"""Fused model rollout: ``MOPO._rollout_model`` (mopo/algorithms/mopo.py:723-765) on one GPU.

``ModelRollout.run`` launches the whole horizon (actor -> ensemble -> FakeEnv post -> compaction
-> pool append, csrc/rollout.hip) on the current stream with no host synchronisation; the
transitions land in a device ``SimpleReplayPool`` in the reference's order.  Two RNG modes:

* ``perf`` (default): Philox on the device (start rows, policy noise, member choice, obs noise).
* ``parity``: every stream injected -- start rows, TF policy noise ``eps_act`` and the numpy
  FakeEnv draws (the selected member's noise and the member index per row), so the result can be
  compared to the reference for identical inputs.
"""
import ctypes as C
import os

import numpy as np

from . import _lib as L


def hidden_pair(H):
    """The two hidden widths of the policy / Q MLPs (mopo.py:275-280, 311-325: ``hidden_sizes``): an int
    H means [H, H]."""
    if isinstance(H, (int, np.integer)):
        return int(H), int(H)
    hs = [int(x) for x in H]
    if len(hs) != 2 or min(hs) < 1:
        raise NotImplementedError('policy / Q hidden_sizes must be two widths [H1, H2] (got %r)' % (H,))
    return hs[0], hs[1]


def device_hidden(H):
    """The square width the device kernels run a [H1, H2] network at: max(H1, H2) rounded up to 16.
    A narrower layer is embedded with zero weights and biases, which is exact for the relu MLPs: a
    padded unit is relu(0) = 0 forward, its relu mask is off backward, so its weights' gradients, Adam
    moments and updates stay exactly 0 (and the Polyak average of zeros is 0)."""
    h1, h2 = hidden_pair(H)
    return (max(h1, h2) + 15) // 16 * 16


def sac_param_shapes(O, A, H=256):
    """Creation order of get_vars('main') (mopo.py:32-33, 298-324): pi, q1, q2 in TF [in,out] layout;
    ``H`` an int or [H1, H2]."""
    h1, h2 = hidden_pair(H)
    pi = [(O, h1), (h1,), (h1, h2), (h2,), (h2, A), (A,), (h2, A), (A,)]
    q = [(O + A, h1), (h1,), (h1, h2), (h2,), (h2, 1), (1,)]
    return pi + q + q


def init_sac_params(O, A, H=256, seed=2):
    """tf.layers.dense defaults: glorot_uniform kernels, zero biases; returns a flat float32 array in
    the [H1, H2] network's own layout."""
    rng = np.random.RandomState(seed)
    parts = []
    for shp in sac_param_shapes(O, A, H):
        if len(shp) == 2:
            lim = np.sqrt(6.0 / (shp[0] + shp[1]))
            parts.append(rng.uniform(-lim, lim, size=shp).astype(np.float32).ravel())
        else:
            parts.append(np.zeros(shp, np.float32))
    flat = np.concatenate(parts)
    if hidden_pair(H)[0] == hidden_pair(H)[1]:
        assert flat.size == L.lib().mopo_sac_param_count(O, A, hidden_pair(H)[0])
    return flat


def sac_pad_index(O, A, H):
    """Positions of a [H1, H2] network's flat parameters inside the flat layout of the square
    device_hidden(H) network (each tensor's [:rows, :cols] corner); None when H is already square."""
    h1, h2 = hidden_pair(H)
    hd = device_hidden(H)
    if h1 == h2 == hd:
        return None
    idx, off = [], 0
    for ls, ds in zip(sac_param_shapes(O, A, (h1, h2)), sac_param_shapes(O, A, hd)):
        if len(ls) == 2:
            idx.append((off + np.arange(ls[0])[:, None] * ds[1] + np.arange(ls[1])[None, :]).ravel())
        else:
            idx.append(off + np.arange(ls[0]))
        off += int(np.prod(ds))
    return np.concatenate(idx).astype(np.int64)


def split_params(flat, O, A, H=256):
    out, off = [], 0
    for shp in sac_param_shapes(O, A, H):
        n = int(np.prod(shp))
        out.append(flat[off:off + n].reshape(shp))
        off += n
    return out


_ACTOR_DTYPES = {'fp32': 0, 'bf16x6': 3, 'f16x3': 4}


def default_actor_dtype(ensemble_dtype):
    """The rollout policy's arithmetic for an ensemble dtype: the exact-operand forms beside the exact-operand
    ensembles -- f32 MFMA beside fp32, the exact bf16x6 split beside bf16x6 -- so the whole rollout computes on
    the reference's f32 operands; else the f16x3 actor (~22-bit operands on the f16 MFMA, held to the fp32
    actor tolerances) beside the reduced-operand ensembles (f16x3, bf16x3, bf16)."""
    return ensemble_dtype if ensemble_dtype in ('fp32', 'bf16x6') else 'f16x3'


class ModelRollout:
    """Owns the rollout workspace for up to ``max_batch`` rows x ``max_horizon`` steps."""

    def __init__(self, model, max_batch, max_horizon=32):
        self.model = model
        self.max_batch, self.max_horizon = int(max_batch), int(max_horizon)
        h = C.c_void_p()
        L.check(L.lib().mopo_rollout_create(C.byref(h), model.handle, self.max_batch, self.max_horizon))
        self._h = h

    def __del__(self):
        h = getattr(self, '_h', None)
        if h is not None and h.value:
            L.lib().mopo_rollout_destroy(h)
            self._h = None

    def run(self, env_obs, pi_params, pool, batch_size, horizon, term_kind, penalty_coeff, elites,
            seed=0, epoch=0, pi_hidden=256, start_idx=None, eps_act=None, eps_obs=None, model_inds=None,
            staged=False, uid_offset=0, stream=None, step_desc=None, step_hook=None, penalty_learned_var=True,
            deterministic=False, rollout_random=False, act_uniform=None, actor_dtype=None):
        """Returns the device int64[horizon] tensor of rows added per step (steps_added).
        ``step_desc(i)`` / ``step_hook(i, steps)``: per-step staging (see mopo_rollout_run_staged_steps).
        ``penalty_learned_var`` / ``deterministic``: FakeEnv's modes (fake_env.py:69-110; every D4RL
        config uses the learned-var penalty, not deterministic); ``rollout_random``: uniform actions
        (mopo.py:736-738), ``act_uniform`` [horizon, B, A] injects them in parity mode.
        ``actor_dtype``: 'fp32', 'bf16x6' or 'f16x3' policy forward (default: default_actor_dtype)."""
        import torch
        dev = env_obs.device
        B = int(batch_size)
        # every steps[i], i < horizon, is stored by the rollout's advance kernels when B > 0 (no fill launch);
        # the elites' device copy is kept while they stay the same (no H2D copy per rollout)
        legacy = os.environ.get('MOPO_ROLLOUT_FILL') == '1'                       # A/B knob: the old launches
        alloc = torch.empty if (B > 0 and int(horizon) > 0 and not legacy) else torch.zeros
        steps = alloc(max(horizon, 1), dtype=torch.int64, device=dev)
        ekey = (tuple(int(e) for e in np.asarray(elites).ravel()), str(dev))
        if getattr(self, '_elites', (None, None))[0] != ekey or legacy:
            self._elites = (ekey, torch.as_tensor(np.asarray(elites, np.int32)).to(dev))
        el = self._elites[1]
        keep = [steps, el]

        def dptr(x, dt):
            if x is None:
                return None
            t = torch.as_tensor(x).to(dev, dt).contiguous()
            keep.append(t)
            return L.ptr(t)

        args = L.RolloutArgs(
            d_env_obs=L.ptr(env_obs), env_size=int(env_obs.shape[0]), d_start_idx=dptr(start_idx, torch.int64),
            d_pi_params=pi_params if isinstance(pi_params, int) else L.ptr(pi_params), pi_hidden=int(pi_hidden), d_elites=L.ptr(el), n_elites=int(el.numel()),
            B=B, horizon=int(horizon), penalty_coeff=float(penalty_coeff), term_kind=int(term_kind),
            seed=int(seed) & (2 ** 64 - 1), epoch=int(epoch), uid_offset=int(uid_offset),
            d_eps_act=dptr(eps_act, torch.float32), d_eps_obs=dptr(eps_obs, torch.float64),
            d_model_inds=dptr(model_inds, torch.int32), d_steps=L.ptr(steps),
            penalty_learned_var=int(bool(penalty_learned_var)), deterministic=int(bool(deterministic)),
            rollout_random=int(bool(rollout_random)), d_act_uniform=dptr(act_uniform, torch.float32),
            actor_dtype=_ACTOR_DTYPES[actor_dtype or default_actor_dtype(self.model.dtype)])
        if step_hook is not None:
            # one call per horizon step into the staging block step_hook(i) names; step_hook(i, steps)
            # is then called after step i is enqueued (multi-GPU: gather step i while i + 1 computes)
            for i in range(int(horizon)):
                L.check(L.lib().mopo_rollout_run_staged_steps(self._h, args, step_desc(i), i, i + 1,
                                                              L.stream_ptr(stream)))
                step_hook(i, steps)
            self._keepalive = keep
            return steps[:horizon]
        desc = pool.desc() if not isinstance(pool, L.PoolDesc) else pool
        fn = L.lib().mopo_rollout_run_staged if staged else L.lib().mopo_rollout_run
        L.check(fn(self._h, args, desc, L.stream_ptr(stream)))
        self._keepalive = keep
        return steps[:horizon]
