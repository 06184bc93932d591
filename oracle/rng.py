"""Oracle: the perf-mode random streams of the fused rollout, restated in numpy.
TEST INFRASTRUCTURE ONLY.

The reference draws every rollout random number from numpy's global MT19937 (start rows
``flexible_replay_pool.py:87``, policy noise ``mopo.py:306``, observation noise ``fake_env.py:72``,
member choice ``bnn.py:343``); parity mode injects exactly those draws.  Perf mode replaces them with
counter-based Philox4x32-10 streams keyed by the global row id, so that any row can be recomputed
on its own.  This module restates those device streams (``mopo_amd/csrc/common.h`` philox /
box_muller, ``rollout.hip`` rollout_start_kernel and rollout_post_kernel, ``actor.hip``
actor_noise and the member choice) so that sampled rows of a full-size perf-mode rollout can be
checked against the oracle.  Philox itself is pinned by the Random123 known-answer vectors
(tests/test_oracle.py); the streams' layout is pinned by the GPU test that replays them.

Counter = {uid lo, uid hi ^ (block << 20), step, stream}; key = {seed lo, seed hi}.  A rollout of
epoch ``ep`` draws its start rows at step ``ep * 4096`` and horizon step ``i`` at ``ep * 4096 + 1 + i``.
"""
import numpy as np

RNG_START, RNG_ACT, RNG_OBS_NOISE, RNG_MODEL = 1, 2, 3, 4
_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = 0x9E3779B9, 0xBB67AE85
_LO = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Philox4x32-10 on uint32 arrays (broadcast); returns the four output words as uint32 arrays."""
    c = [np.asarray(x, np.uint64) & _LO for x in (c0, c1, c2, c3)]
    c = np.broadcast_arrays(*c)
    c = [x.copy() for x in c]
    k0, k1 = int(k0) & 0xFFFFFFFF, int(k1) & 0xFFFFFFFF
    for _ in range(10):
        p0 = _M0 * c[0]
        p1 = _M1 * c[2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & _LO
        hi1, lo1 = p1 >> np.uint64(32), p1 & _LO
        c = [hi1 ^ c[1] ^ np.uint64(k0), lo1, hi0 ^ c[3] ^ np.uint64(k1), lo0]
        k0 = (k0 + _W0) & 0xFFFFFFFF
        k1 = (k1 + _W1) & 0xFFFFFFFF
    return [x.astype(np.uint32) for x in c]


def _words(uid, seed, step, stream, block=0):
    uid = np.asarray(uid, np.int64).astype(np.uint64)
    hi = (uid >> np.uint64(32)) ^ (np.uint64(block) << np.uint64(20))
    return philox4x32_10(uid & _LO, hi, np.uint64(step), np.uint64(stream), seed & 0xFFFFFFFF,
                         (seed >> 32) & 0xFFFFFFFF)


def box_muller(a, b):
    """common.h box_muller in float32: two normals from two uint32 words."""
    f = np.float32
    u1 = (a.astype(f) + f(1.0)) * f(2.3283064e-10)
    u2 = b.astype(f) * f(2.3283064e-10)
    r = np.sqrt(f(-2.0) * np.log(u1))
    t = f(6.2831853) * u2
    return r * np.cos(t), r * np.sin(t)


def _normals(uid, seed, step, stream, n):
    """n normals per row: block j supplies normals 4j..4j+3 (x,y -> 0,1; z,w -> 2,3)."""
    out = np.empty((len(uid), 4 * ((n + 3) // 4)), np.float32)
    for blk in range((n + 3) // 4):
        x, y, z, w = _words(uid, seed, step, stream, blk)
        out[:, 4 * blk], out[:, 4 * blk + 1] = box_muller(x, y)
        out[:, 4 * blk + 2], out[:, 4 * blk + 3] = box_muller(z, w)
    return out[:, :n]


def start_rows(uid, seed, step, env_size):
    """rollout_start_kernel: perf mode of env_pool.random_indices(B)."""
    x = _words(uid, seed, step, RNG_START)[0]
    return ((x.astype(np.uint64) * np.uint64(env_size)) >> np.uint64(32)).astype(np.int64)


def act_noise(uid, seed, step, A):
    """actor_noise: the policy's N(0, 1) draw per action dim (mopo.py:306)."""
    return _normals(uid, seed, step, RNG_ACT, A)


def obs_noise(uid, seed, step, D):
    """rollout_post_kernel: the observation-noise normal per output dim (fake_env.py:72)."""
    return _normals(uid, seed, step, RNG_OBS_NOISE, D)


def model_choice(uid, seed, step, elites):
    """actor_kernel member selection: perf mode of np.random.choice(elites, B) (bnn.py:343)."""
    x = _words(uid, seed, step, RNG_MODEL)[0]
    elites = np.asarray(elites, np.int32)
    return elites[((x.astype(np.uint64) * np.uint64(len(elites))) >> np.uint64(32)).astype(np.int64)]


# ---- the SAC step's perf-mode streams (csrc/sac_rows.h gather_elem / head_noise), keyed by the device
# step counter ``it`` (0 for a fresh handle, +1 per step) and the call's seed (MOPO: seed + 7919 * epoch)
RNG_SAC = 5


def _sac_words(r, seed, c1, c2, stream):
    return philox4x32_10(np.asarray(r, np.uint64), c1, c2, stream, seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)


def sac_batch_indices(n, n_env, env_size, model_size, seed, it):
    """_training_batch (mopo.py:801-821) in perf mode: row r < n_env indexes the env pool, the rest the
    model pool, uniform over the pool's live size: counter {r, it lo, it hi, RNG_SAC}."""
    r = np.arange(n, dtype=np.uint64)
    x = _sac_words(r, seed, np.uint64(it & 0xFFFFFFFF), np.uint64((it >> 32) & 0xFFFFFFFF), RNG_SAC)[0]
    size = np.where(r < n_env, env_size, model_size).astype(np.uint64)
    return ((x.astype(np.uint64) * size) >> np.uint64(32)).astype(np.int64)


def sac_noise(n, A, seed, it, nxt):
    """The policy noise of the SAC step (mopo.py:306) for pi(s) (nxt 0) / pi(s') (nxt 1): action j of row r
    from the Philox block j // 4 with counter {r | nxt << 31, it ^ (block << 24), it hi, RNG_SAC + 16};
    actions 4b, 4b+1 from words (x, y), 4b+2, 4b+3 from (z, w)."""
    r = np.arange(n, dtype=np.uint64) | (np.uint64(nxt) << np.uint64(31))
    out = np.empty((n, 4 * ((A + 3) // 4)), np.float32)
    for blk in range((A + 3) // 4):
        x, y, z, w = _sac_words(r, seed, np.uint64((it & 0xFFFFFFFF) ^ (blk << 24)),
                                np.uint64((it >> 32) & 0xFFFFFFFF), RNG_SAC + 16)
        out[:, 4 * blk], out[:, 4 * blk + 1] = box_muller(x, y)
        out[:, 4 * blk + 2], out[:, 4 * blk + 3] = box_muller(z, w)
    return out[:, :A]
