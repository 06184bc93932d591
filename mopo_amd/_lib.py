"""ctypes binding of libmopo_hip.so (the C ABI declared in include/mopo_hip.h).

The product path always goes through this library; if it is missing the import fails loudly
(there is no CPU fallback).  Build it with ``make -C mopo_amd/csrc -j8`` or
``python -c "import __graft_entry__ as g; g.build()"``.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, 'libmopo_hip.so')

c_void_p, c_int, c_i64, c_u64, c_u32, c_float, c_double = (
    C.c_void_p, C.c_int, C.c_int64, C.c_uint64, C.c_uint32, C.c_float, C.c_double)


class FakeEnvArgs(C.Structure):
    _fields_ = [('d_obs', c_void_p), ('obs_f64', c_int), ('d_act', c_void_p), ('B', c_i64),
                ('d_noise_sel', c_void_p), ('d_model_inds', c_void_p), ('deterministic', c_int),
                ('penalty_coeff', c_float), ('penalty_learned_var', c_int), ('term_kind', c_int),
                ('d_next_obs', c_void_p), ('d_rewards', c_void_p), ('d_terminals', c_void_p),
                ('d_penalty', c_void_p), ('d_unpenalized', c_void_p), ('d_info_mean', c_void_p),
                ('d_info_std', c_void_p), ('d_log_prob', c_void_p), ('d_dev', c_void_p),
                ('d_ens_mean', c_void_p), ('d_ens_var', c_void_p)]


class PoolDesc(C.Structure):
    _fields_ = [('d_obs', c_void_p), ('d_act', c_void_p), ('d_rew', c_void_p), ('d_term', c_void_p),
                ('d_next_obs', c_void_p), ('d_state', c_void_p), ('max_size', c_i64)]


class RolloutArgs(C.Structure):
    _fields_ = [('d_env_obs', c_void_p), ('env_size', c_i64), ('d_start_idx', c_void_p),
                ('d_pi_params', c_void_p), ('pi_hidden', c_int), ('d_elites', c_void_p),
                ('n_elites', c_int), ('B', c_i64), ('horizon', c_int), ('penalty_coeff', c_float),
                ('term_kind', c_int), ('seed', c_u64), ('epoch', c_u32), ('uid_offset', c_i64),
                ('d_eps_act', c_void_p), ('d_eps_obs', c_void_p), ('d_model_inds', c_void_p),
                ('d_steps', c_void_p), ('penalty_learned_var', c_int), ('deterministic', c_int),
                ('rollout_random', c_int), ('d_act_uniform', c_void_p), ('actor_dtype', c_int)]


# name -> (restype, argtypes); every symbol declared in include/mopo_hip.h
SIGNATURES = {
    'mopo_last_error': (C.c_char_p, []),
    'mopo_version': (c_int, []),
    'mopo_bnn_create': (c_int, [C.POINTER(c_void_p), c_int, c_int, c_int, c_int, c_int, c_int]),
    'mopo_bnn_destroy': (c_int, [c_void_p]),
    'mopo_bnn_set_params': (c_int, [c_void_p, C.POINTER(c_void_p), c_int]),
    'mopo_bnn_predict': (c_int, [c_void_p, c_void_p, c_int, c_i64, c_void_p, c_void_p, c_void_p]),
    'mopo_bnn_packed_bytes': (c_i64, [c_void_p]),
    'mopo_bnn_packed_copy': (c_int, [c_void_p, c_int, c_void_p, c_i64, c_void_p]),
    'mopo_fakeenv_step': (c_int, [c_void_p, C.POINTER(FakeEnvArgs), c_void_p]),
    'mopo_sac_param_count': (c_i64, [c_int, c_int, c_int]),
    'mopo_actor_forward': (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_i64, c_void_p,
                                   c_u64, c_u32, c_void_p, c_void_p, c_void_p]),
    'mopo_actor_forward_dtype': (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_i64, c_void_p,
                                         c_u64, c_u32, c_void_p, c_void_p, c_int, c_void_p]),
    'mopo_pool_add': (c_int, [C.POINTER(PoolDesc), c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                              c_void_p, c_i64, c_void_p]),
    'mopo_pool_gather': (c_int, [C.POINTER(PoolDesc), c_int, c_int, c_void_p, c_i64, c_void_p, c_void_p,
                                 c_void_p, c_void_p, c_void_p, c_i64, c_void_p]),
    'mopo_pool_random_indices': (c_int, [C.POINTER(PoolDesc), c_i64, c_u64, c_u32, c_void_p, c_void_p]),
    'mopo_pool_staged_block_bytes': (c_i64, [c_int, c_int, c_i64]),
    'mopo_pool_add_blocks': (c_int, [C.POINTER(PoolDesc), c_int, c_int, c_void_p, c_i64, c_int, c_i64, c_void_p,
                                     c_void_p]),
    'mopo_rollout_run_staged_steps': (c_int, [c_void_p, C.POINTER(RolloutArgs), C.POINTER(PoolDesc), c_int, c_int,
                                              c_void_p]),
    'mopo_bnn_train_create': (c_int, [C.POINTER(c_void_p), c_int, c_int, c_int, c_int, c_int, c_int, C.c_float]),
    'mopo_bnn_train_destroy': (c_int, [c_void_p]),
    'mopo_bnn_train_set_params': (c_int, [c_void_p, C.POINTER(c_void_p)]),
    'mopo_bnn_train_get_params': (c_int, [c_void_p, C.POINTER(c_void_p)]),
    'mopo_bnn_format_samples': (c_int, [C.POINTER(PoolDesc), c_int, c_int, c_void_p, c_i64, c_void_p, c_void_p,
                                        c_void_p]),
    'mopo_bnn_train_fit_scaler': (c_int, [c_void_p, c_void_p, c_i64, c_void_p]),
    'mopo_bnn_train_epoch': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_i64, c_int, c_void_p]),
    'mopo_bnn_train_eval_mse': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    'mopo_bnn_train_shuffle': (c_int, [c_void_p, c_void_p, c_void_p, c_i64, c_void_p]),
    'mopo_bnn_train_shuffle_async': (c_int, [c_void_p, c_void_p, c_void_p, c_i64, c_void_p, c_void_p]),
    'mopo_bnn_train_snapshot': (c_int, [c_void_p, c_int, c_void_p]),
    'mopo_bnn_train_snapshot_members': (c_int, [c_void_p, c_void_p, c_int, c_void_p]),
    'mopo_bnn_train_restore': (c_int, [c_void_p, c_void_p]),
    'mopo_bnn_train_logs': (c_int, [c_void_p, c_void_p, c_int]),
    'mopo_bnn_train_tile_lists': (c_int, [c_int, c_int, c_int, c_int, c_void_p, c_i64]),
    'mopo_bnn_train_debug_stamps': (c_int, [c_void_p, c_i64]),
    'mopo_rollout_create': (c_int, [C.POINTER(c_void_p), c_void_p, c_i64, c_int]),
    'mopo_rollout_destroy': (c_int, [c_void_p]),
    'mopo_rollout_run': (c_int, [c_void_p, C.POINTER(RolloutArgs), C.POINTER(PoolDesc), c_void_p]),
    'mopo_rollout_run_staged': (c_int, [c_void_p, C.POINTER(RolloutArgs), C.POINTER(PoolDesc), c_void_p]),
    'mopo_rollout_profile': (c_int, [c_void_p, c_int]),
    'mopo_rollout_profile_read': (c_int, [c_void_p, c_void_p, c_void_p, c_int]),
    'mopo_sac_create': (c_int, [C.POINTER(c_void_p), c_int, c_int, c_int, c_int, c_int, c_void_p, c_float,
                                c_float, c_float, c_float, c_float, c_float]),
    'mopo_sac_destroy': (c_int, [c_void_p]),
    'mopo_sac_buffers': (c_int, [c_void_p] + [C.POINTER(c_void_p)] * 6 + [C.POINTER(c_i64)]),
    'mopo_sac_step': (c_int, [c_void_p, C.POINTER(PoolDesc), C.POINTER(PoolDesc), c_int, c_u64, c_void_p,
                              c_void_p, c_void_p, c_void_p]),
    'mopo_sac_set_graph': (c_int, [c_void_p, c_int]),
    'mopo_sac_check': (c_int, [c_void_p, C.POINTER(c_int)]),
    'mopo_sac_inject_timeout': (c_int, [c_void_p]),
    'mopo_sac_set_target_schedule': (c_int, [c_void_p, c_i64, c_i64, c_i64, c_void_p]),
    'mopo_sac_set_action_prior': (c_int, [c_void_p, c_int]),
    'mopo_sac_copy': (c_int, [c_void_p, c_int, c_int, c_void_p, c_i64, c_void_p]),
    'mopo_sac_debug_stamps': (c_int, [c_void_p, c_void_p, c_i64]),
    'mopo_mt_create': (c_int, [C.POINTER(c_void_p), c_u32]),
    'mopo_mt_destroy': (c_int, [c_void_p]),
    'mopo_mt_seed': (c_int, [c_void_p, c_u32]),
    'mopo_mt_set_state': (c_int, [c_void_p, c_void_p, c_int, c_int, c_double]),
    'mopo_mt_get_state': (c_int, [c_void_p, c_void_p, C.POINTER(c_int), C.POINTER(c_int),
                                  C.POINTER(c_double)]),
    'mopo_mt_normal': (c_int, [c_void_p, c_void_p, c_i64]),
    'mopo_mt_randint': (c_int, [c_void_p, c_void_p, c_i64, c_i64, c_i64]),
    'mopo_mt_random_sample': (c_int, [c_void_p, c_void_p, c_i64]),
    'mopo_mt_randint_i32': (c_int, [c_void_p, c_void_p, c_i64, c_i64, c_i64]),
}

_lib = None


def lib():
    """Load libmopo_hip.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError('libmopo_hip.so not built at %s (run make -C mopo_amd/csrc)' % LIB_PATH)
        # torch ships its own libamdhip64.so.7; load it first so the library binds to that one HIP
        # runtime (same soname) instead of pulling /opt/rocm's copy into the process beside it.
        import torch  # noqa: F401
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _lib = L
    return _lib


class MopoError(RuntimeError):
    pass


def check(rc):
    if rc != 0:
        raise MopoError(lib().mopo_last_error().decode())
    return rc


def ptr(t):
    """Device/host pointer of a torch tensor or numpy array (None -> NULL)."""
    if t is None:
        return None
    if hasattr(t, 'data_ptr'):
        return t.data_ptr()
    return t.ctypes.data


def stream_ptr(stream=None):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream
