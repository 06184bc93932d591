"""mopo_amd: MI355X-native MOPO model-rollout + SAC-update hot path.

Host side mirrors the reference interfaces (construct_model / BNN.predict, FakeEnv.step,
SimpleReplayPool, MOPO._rollout_model / _do_training); compute runs in libmopo_hip.so
(hand-written HIP for gfx950, C ABI in include/mopo_hip.h).
"""
from ._lib import lib, MopoError  # noqa: F401

__all__ = ['lib', 'MopoError']
