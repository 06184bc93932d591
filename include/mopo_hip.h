/*
 * libmopo_hip — MI355X (gfx950) C ABI for the MOPO model-rollout + SAC-update hot path.
 *
 * Plain C types only (pointers, sizes); no torch types.  All array pointers named d_* are
 * DEVICE pointers owned by the caller (the library borrows them for the duration of the call);
 * h_* are host pointers.  `stream` is a hipStream_t passed as void* (NULL = default stream).
 * Every entry point returns 0 on success and -1 on error; mopo_last_error() returns a
 * thread-local message.  One handle = one stream at a time (not re-entrant), matching the
 * reference's single Python thread driving one tf.Session.
 *
 * Reference interfaces replaced (xionghuichen/mopo @ v0):
 *   mopo_bnn_*        construct_model / BNN.finalize / BNN.load_params / BNN.predict
 *                     (mopo/models/constructor.py:7-43, mopo/models/bnn.py:166-281, 508-546)
 *   mopo_fakeenv_step FakeEnv.step (mopo/models/fake_env.py:37-131) + termination_fn
 *                     (mopo/static/{halfcheetah,walker2d,hopper}.py)
 *   mopo_actor_forward MOPO.get_action_meta (mopo/algorithms/mopo.py:468-485, 298-308)
 *   mopo_rollout_*    MOPO._rollout_model (mopo/algorithms/mopo.py:723-765) writing into
 *                     SimpleReplayPool.add_samples (softlearning/replay_pools/flexible_replay_pool.py:57-83)
 *   mopo_pool_gather  FlexibleReplayPool.random_batch / batch_by_indices (flexible_replay_pool.py:85-135)
 *   mopo_sac_*        MOPO._do_training / _update_target (mopo/algorithms/mopo.py:834-853,
 *                     graph mopo.py:204-466); SAC API sac.py:26-47
 *   mopo_bnn_train_*  BNN.train (mopo/models/bnn.py:369-503; loss :226-249, 677-701; Adam
 *                     constructor.py:41), format_samples_for_training (constructor.py:46-57),
 *                     caller MOPO._train_model (mopo/algorithms/mopo.py:713-721)
 *   mopo_mt_*         numpy legacy RandomState (MT19937) as used by fake_env.py:72,
 *                     bnn.py:343, flexible_replay_pool.py:87
 */
#ifndef MOPO_HIP_H
#define MOPO_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- errors / info ------------------------------------------------------------------ */
const char* mopo_last_error(void);
int mopo_version(void);

/* ---- probabilistic ensemble (BNN) ---------------------------------------------------- */
typedef struct mopo_bnn_s* mopo_bnn_t;

/* E members, obs_dim O, act_dim A, hidden H (4 swish layers), D = O+1 outputs.
 * smv=1: separate mean / var heads (bnn.py:656-675); smv=0: joint 2D head (bnn.py:644-655).
 * dtype: 0 = fp32 (exact-f32 MFMA 16x16x4);
 *        1 = bf16 weights/activations, f32 accumulate (~8 significand bits; the C3 config);
 *        2 = "bf16x3": every f32 operand split into 2 bf16 parts, 3 bf16 products per f32 product
 *            (~17 significand bits), f32 accumulate;
 *        3 = "bf16x6": 3 bf16 parts, 6 bf16 products per f32 product, f32 accumulate (~22-bit
 *            operands, held to the fp32 parity tolerances);
 *        4 = "f16x3": every f32 operand as 2 fp16 parts under power-of-two scales (per weight block,
 *            per activation row), 3 f16 products per f32 product, f32 accumulate (~22-bit operands,
 *            held to the fp32 parity tolerances; MOPO's default and the bench headline).
 * Limits: obs_dim + act_dim <= 32 (one or two 16-wide input k-groups); hidden 32, 64, 200 or 400 (any
 * width with the same number of 16-wide blocks); the bf16 kinds need 2 (obs_dim + 1) <= 48 head
 * slots; E <= 256. */
int mopo_bnn_create(mopo_bnn_t* out, int E, int obs_dim, int act_dim, int hidden, int smv, int dtype);
int mopo_bnn_destroy(mopo_bnn_t h);
/* The reference .mat layout, keys '0'..'15' (bnn.py:224-225, 588-592): mu[1,IN], sigma[1,IN],
 * (W[E,in,out], b[E,1,out]) x 5 mean layers, (Wv[E,H,D], bv[E,1,D]) if smv, maxlv[1,D], minlv[1,D].
 * n_arrays = 16 (smv) or 14; all host float32, C order. */
int mopo_bnn_set_params(mopo_bnn_t h, const float* const* h_arrays, int n_arrays);
/* BNN.predict(inputs, factored=True): d_inputs [B, O+A] (f32 if inputs_f64==0 else f64)
 * -> d_mean, d_var [E, B, D] f32. */
int mopo_bnn_predict(mopo_bnn_t h, const void* d_inputs, int inputs_f64, int64_t B,
                     float* d_mean, float* d_var, void* stream);
/* The handle's packed device parameters (weights in the kernels' fragment layout, biases, scaler,
 * log-var bounds, f16x3 scales) as one opaque byte image: packed_bytes() is its size (-1 before
 * set_params); packed_copy(to_handle=0) writes it to d_buf, to_handle=1 loads it from d_buf into a
 * handle of the same shapes and dtype that already had set_params called.  Multi-GPU: rank 0's image
 * is broadcast device-to-device (no host round trip or repack) -- no reference counterpart. */
int64_t mopo_bnn_packed_bytes(mopo_bnn_t h);
int mopo_bnn_packed_copy(mopo_bnn_t h, int to_handle, void* d_buf, int64_t nbytes, void* stream);

/* ---- FakeEnv.step ------------------------------------------------------------------- */
/* termination rules of mopo/static/<domain>.py: NONE covers halfcheetah{,jump,vel,veljump}, point2denv,
 * point2dwallenv and pendulum (never done); ANT covers ant.py / antangle.py; HUMANOID humanoid.py */
enum { MOPO_TERM_NONE = 0, MOPO_TERM_HALFCHEETAH = 0, MOPO_TERM_WALKER2D = 1, MOPO_TERM_HOPPER = 2,
       MOPO_TERM_ANT = 3, MOPO_TERM_HUMANOID = 4, MOPO_TERM_KINDS = 5 };

typedef struct {
  const void* d_obs;        /* [B, O], f64 if obs_f64 else f32 */
  int obs_f64;
  const float* d_act;       /* [B, A] f32 */
  int64_t B;
  const double* d_noise_sel; /* [B, D] f64: the standard normals of fake_env.py:72 for the SELECTED
                               member of each row, noise[model_inds[b], b]; unused if deterministic */
  const int64_t* d_model_inds; /* [B] member index per row (bnn.py:343); unused if deterministic */
  int deterministic;        /* fake_env.py:69-70,84-86 */
  float penalty_coeff;      /* fake_env.py:97,115 */
  int penalty_learned_var;  /* 1: max_e ||std_e||  0: max_e ||mean_e - mean|| (fake_env.py:98-110) */
  int term_kind;            /* MOPO_TERM_* */
  /* outputs (device) */
  double* d_next_obs;       /* [B, O] f64; must not alias d_obs */
  double* d_rewards;        /* [B] penalized rewards f64 */
  uint8_t* d_terminals;     /* [B] */
  float* d_penalty;         /* [B] f32, may be NULL */
  double* d_unpenalized;    /* [B] f64, may be NULL */
  float* d_info_mean;       /* [B, D+1] f32 (model mean with terminal column), may be NULL */
  float* d_info_std;        /* [B, D+1] f32, may be NULL */
  double* d_log_prob;       /* [B] f64, may be NULL */
  float* d_dev;             /* [B] f32, may be NULL */
  float* d_ens_mean;        /* workspace / output [E, B, D] f32 (required) */
  float* d_ens_var;         /* workspace / output [E, B, D] f32 (required) */
} mopo_fakeenv_args;

int mopo_fakeenv_step(mopo_bnn_t h, const mopo_fakeenv_args* a, void* stream);

/* ---- policy (actor) --------------------------------------------------------------------
 * SAC parameters are one flat f32 buffer in reference creation order (mopo.py:32-33, 298-324):
 *   pi: W1[O,Hp] b1[Hp] W2[Hp,Hp] b2[Hp] Wmu[Hp,A] bmu[A] Wls[Hp,A] bls[A]
 *   q1: W1[O+A,Hp] b1 W2[Hp,Hp] b2 W3[Hp,1] b3[1]      q2: same
 * mopo_sac_param_count() gives the total; the pi block starts at offset 0. */
int64_t mopo_sac_param_count(int obs_dim, int act_dim, int hidden);

/* get_action_meta(obs): act = tanh(mu + eps*exp(clip(log_std))) (mopo.py:298-308, 286-296).
 * d_eps [B, A] f32 injected normals, or NULL to draw Philox normals from (seed, step). */
int mopo_actor_forward(const float* d_pi_params, int obs_dim, int act_dim, int hidden,
                       const void* d_obs, int obs_f64, int64_t B, const float* d_eps,
                       uint64_t seed, uint32_t step, float* d_act, float* d_mu, void* stream);
/* The same with the arithmetic chosen: dtype 0 = fp32 (f32 MFMA), 3 = bf16x6 (f32 operands split exactly into
 * 3 bf16 parts, 6 bf16 MFMA products), 4 = f16x3 (f32 operands as 2 fp16 parts under power-of-two scales,
 * 3 f16 MFMA products, ~22-bit operands); hidden 32 or 256 for the split forms. */
int mopo_actor_forward_dtype(const float* d_pi_params, int obs_dim, int act_dim, int hidden,
                             const void* d_obs, int obs_f64, int64_t B, const float* d_eps,
                             uint64_t seed, uint32_t step, float* d_act, float* d_mu, int dtype, void* stream);

/* ---- device-resident SimpleReplayPool ---------------------------------------------------
 * SoA fields (simple_replay_pool.py:48-70), all caller-owned device arrays of max_size rows:
 * observations f32[O], actions f32[A], rewards f32[1], terminals u8[1], next_observations f32[O].
 * d_state = int64[2] {pointer, size} on the device. */
typedef struct {
  float* d_obs;
  float* d_act;
  float* d_rew;
  uint8_t* d_term;
  float* d_next_obs;
  int64_t* d_state;
  int64_t max_size;
} mopo_pool_desc;

/* add_samples with device arrays of n rows (flexible_replay_pool.py:57-83). */
int mopo_pool_add(const mopo_pool_desc* pool, int obs_dim, int act_dim, const float* d_obs,
                  const float* d_act, const float* d_rew, const uint8_t* d_term,
                  const float* d_next_obs, int64_t n, void* stream);
/* batch_by_indices: d_idx int64[n] -> dst rows (dst_* arrays of n rows, any may be NULL).
 * dst_row_offset lets two gathers (env + model pool, mopo.py:809-816) fill one batch. */
int mopo_pool_gather(const mopo_pool_desc* pool, int obs_dim, int act_dim, const int64_t* d_idx,
                     int64_t n, float* dst_obs, float* dst_act, float* dst_rew, float* dst_term,
                     float* dst_next_obs, int64_t dst_row_offset, void* stream);
/* uniform random indices in [0, size) from Philox (perf mode of random_indices). */
int mopo_pool_random_indices(const mopo_pool_desc* pool, int64_t n, uint64_t seed, uint32_t step,
                             int64_t* d_idx, void* stream);

/* Multi-GPU staging: a block of B staged rows laid out obs f32[B][O] | act f32[B][A] | rew f32[B] |
 * next_obs f32[B][O] | term u8[B] (a pool descriptor over it has max_size B, no state).  add_blocks
 * appends the first d_counts[b] rows of each block b = 0..n_blocks-1 in that order (the all-gathered
 * per-step blocks, step-major then rank-major) and advances ptr/size on the device (no host sync). */
int64_t mopo_pool_staged_block_bytes(int obs_dim, int act_dim, int64_t B);
int mopo_pool_add_blocks(const mopo_pool_desc* pool, int obs_dim, int act_dim, const uint8_t* d_blocks,
                         int64_t block_stride, int n_blocks, int64_t B, const int64_t* d_counts, void* stream);

/* ---- ensemble training (BNN.train, bnn.py:369-503) -------------------------------------
 * Training state of an smv ensemble (E members, 4 swish layers of width H, mean + log-var heads).
 * The host drives the loop (holdout split, bootstrap indices, early stopping, elites: bnn.py:369-503)
 * with numpy's stream; these calls are its device parts.  lr: tf.train.AdamOptimizer (1e-3,
 * constructor.py:41).  max_batch: minibatch rows per member (256, mopo.py:529); max_eval: rows of
 * one mse evaluation (holdout <= 1000, bnn.py:392). */
typedef struct mopo_bnn_train_s* mopo_bnn_train_t;
int mopo_bnn_train_create(mopo_bnn_train_t* out, int E, int obs_dim, int act_dim, int hidden, int max_batch,
                          int max_eval, float lr);
int mopo_bnn_train_destroy(mopo_bnn_train_t h);
/* The 16 .mat arrays (smv layout, as mopo_bnn_set_params; host f32).  set resets the optimizer. */
int mopo_bnn_train_set_params(mopo_bnn_train_t h, const float* const* h_arrays);
int mopo_bnn_train_get_params(mopo_bnn_train_t h, float* const* h_arrays);
/* format_samples_for_training (constructor.py:46-57) of pool rows d_rows[n] (NULL: rows 0..n-1):
 * d_inputs [n, O+A] = [obs | act], d_targets [n, O+1] = [rew | next_obs - obs]. */
int mopo_bnn_format_samples(const mopo_pool_desc* pool, int obs_dim, int act_dim, const int64_t* d_rows,
                            int64_t n, float* d_inputs, float* d_targets, void* stream);
/* TensorStandardScaler.fit (utils.py:69-86) on d_inputs [n, O+A]. */
int mopo_bnn_train_fit_scaler(mopo_bnn_train_t h, const float* d_inputs, int64_t n, void* stream);
/* One epoch of minibatch Adam steps (bnn.py:425-432): minibatch b of member e is rows
 * d_idxs[e * n_idx + b * batch .. +batch) (int32) of d_inputs / d_targets; the last one may be partial. */
int mopo_bnn_train_epoch(mopo_bnn_train_t h, const float* d_inputs, const float* d_targets, const int32_t* d_idxs,
                         int64_t n_idx, int batch, void* stream);
/* _compile_losses(inc_var_loss=False) (bnn.py:677-701) per member over rows d_rows[e * n + r]
 * (NULL: rows 0..n-1 for every member, the tiled holdout set) -> d_losses[E] f32. */
int mopo_bnn_train_eval_mse(mopo_bnn_train_t h, const float* d_inputs, const float* d_targets,
                            const int32_t* d_rows, int n, float* d_losses, void* stream);
/* shuffle_rows (bnn.py:385-387): d_idxs[e] <- d_idxs[e][argsort(d_keys[e])], keys f64 [E, n]
 * (the np.random.uniform draws). */
int mopo_bnn_train_shuffle(mopo_bnn_train_t h, int32_t* d_idxs, const double* d_keys, int64_t n, void* stream);
/* The same shuffle with the order (the key sort) computed on order_stream, which may run beside the
 * epoch's steps; only the apply to d_idxs is queued on stream, behind the order. */
int mopo_bnn_train_shuffle_async(mopo_bnn_train_t h, int32_t* d_idxs, const double* d_keys, int64_t n,
                                 void* order_stream, void* stream);
/* _save_state(member) / _set_state (bnn.py:264-285). */
int mopo_bnn_train_snapshot(mopo_bnn_train_t h, int member, void* stream);
/* _save_state for several members in one launch (the members whose holdout loss improved this epoch). */
int mopo_bnn_train_snapshot_members(mopo_bnn_train_t h, const int* h_members, int n, void* stream);
int mopo_bnn_train_restore(mopo_bnn_train_t h, void* stream);
/* h_logs[0] = data term of the last minibatch's training loss. */
int mopo_bnn_train_logs(mopo_bnn_train_t h, float* h_logs, int n);
/* Host only (no device call): the per-XCD tile lists of the training step's weight-gradient launch.
 * Writes 8 lists of `per` packed tiles (layer | member << 3 | tile row << 7 | tile column << 12, -1 padded)
 * followed by the 8 list lengths into out (8 per + 8 ints; out may be NULL) and returns per (< 0: error).
 * No reference counterpart: a layout detail of bnn.py:425-432's minibatch op on this device. */
int mopo_bnn_train_tile_lists(int E, int obs_dim, int act_dim, int hidden, int32_t* out, int64_t cap);
/* Diagnostic builds only (MOPO_TRAIN_STAMPS=1; otherwise returns -1): the rows launch's
 * per-workgroup phase stamps of the last step, [block][8] (bnn_train.hip mopo_bnn_train_debug_stamps). */
int mopo_bnn_train_debug_stamps(uint64_t* h_out, int64_t n);

/* ---- fused model rollout (MOPO._rollout_model) ----------------------------------------- */
typedef struct mopo_rollout_s* mopo_rollout_t;

typedef struct {
  /* env pool observations (start states) */
  const float* d_env_obs;   /* [env_size, O] f32 */
  int64_t env_size;
  const int64_t* d_start_idx; /* [B] injected start rows (flexible_replay_pool.py:87) or NULL */
  const float* d_pi_params; /* flat SAC params (pi block used) */
  int pi_hidden;
  const int32_t* d_elites;  /* [n_elites] member ids (bnn.py:337-339) */
  int n_elites;
  int64_t B;                /* rollout_batch_size */
  int horizon;              /* rollout_length */
  float penalty_coeff;
  int term_kind;
  uint64_t seed;            /* Philox key (perf mode) */
  uint32_t epoch;           /* mixed into the Philox counter */
  int64_t uid_offset;       /* global id of this rank's first row (Philox counter; multi-GPU shards) */
  /* parity mode (all NULL in perf mode): per-step injected streams, step i uses rows [0, B_i) */
  const float* d_eps_act;   /* [horizon, B, A] f32 */
  const double* d_eps_obs;  /* [horizon, B, D] f64: the noise of the SELECTED member per row */
  const int32_t* d_model_inds; /* [horizon, B] member per row */
  /* outputs */
  int64_t* d_steps;         /* [horizon] rows added per step (mopo.py:748) */
  /* FakeEnv / rollout modes (fake_env.py:37-131, mopo.py:734-738) */
  int penalty_learned_var;  /* 1: max_e ||std_e|| over all D dims (every D4RL config, fake_env.py:110)
                               0: max_e ||mean_e - mean over members|| over the obs dims (fake_env.py:98-108) */
  int deterministic;        /* 1: no sampling; next state = mean over ALL members of the means (fake_env.py:69-70,
                               84-86); the selection streams are unused */
  int rollout_random;       /* 1: actions ~ U(-1, 1) instead of the policy's (mopo.py:736-738) */
  const float* d_act_uniform; /* parity mode with rollout_random: [horizon, B, A] injected uniforms, or NULL */
  int actor_dtype;          /* policy forward arithmetic: 0 fp32, 3 bf16x6, 4 f16x3 (mopo_actor_forward_dtype) */
} mopo_rollout_args;

int mopo_rollout_create(mopo_rollout_t* out, mopo_bnn_t bnn, int64_t max_batch, int max_horizon);
int mopo_rollout_destroy(mopo_rollout_t h);
/* Runs the whole horizon on `stream` without host synchronisation; transitions are appended
 * to `pool` in the reference's order (step-major, order-preserving non-terminal compaction). */
int mopo_rollout_run(mopo_rollout_t h, const mopo_rollout_args* a, const mopo_pool_desc* pool,
                     void* stream);
/* Rollout that writes its transitions to a caller staging buffer instead of a pool:
 * staging rows [horizon][B] (step i rows [0, steps[i]) valid) - the per-rank leg of the
 * multi-GPU all-gather path. */
int mopo_rollout_run_staged(mopo_rollout_t h, const mopo_rollout_args* a,
                            const mopo_pool_desc* staging, void* stream);

/* Live kernel timing (hipEvents on the launch stream around every launch, per kernel class:
 * 0 start-gather, 1 actor, 2 ensemble forward, 3 FakeEnv post, 4 compaction, 5 pointer advance).
 * profile_read synchronises the recorded events, returns summed ms and launch counts for the
 * runs since the last read, and clears them. */
/* Steps [step_begin, step_end) of one staged rollout (the first call starts at 0; later calls continue
 * where the previous one stopped).  Rows of step i go to staging rows (i - step_begin) * B, so with one
 * call per step each step fills its own staging block -- the multi-GPU path gathers step i while step
 * i + 1 computes.  d_steps[i] receives the rows of step i. */
int mopo_rollout_run_staged_steps(mopo_rollout_t h, const mopo_rollout_args* a, const mopo_pool_desc* staging,
                                  int step_begin, int step_end, void* stream);
int mopo_rollout_profile(mopo_rollout_t h, int enable);
int mopo_rollout_profile_read(mopo_rollout_t h, double* ms, int64_t* launches, int n);

/* ---- SAC update (MOPO._do_training + _update_target) ------------------------------------
 * h_params: initial flat parameters (mopo_sac_param_count floats, layout above); target = copy
 * (target_init, mopo.py:449-450); log_alpha initial value (mopo.py:357-360); Adam lr / gamma / tau /
 * reward_scale / target_entropy as MOPO.__init__ (mopo.py:56-61, 171-174).  batch = 256 in the
 * reference (sampler batch_size), of which n_env rows come from the env pool (int(256*real_ratio),
 * mopo.py:801-816). */
typedef struct mopo_sac_s* mopo_sac_t;
int mopo_sac_create(mopo_sac_t* out, int obs_dim, int act_dim, int hidden, int batch, int n_env,
                    const float* h_params, float log_alpha, float lr, float gamma, float tau,
                    float reward_scale, float target_entropy);
int mopo_sac_destroy(mopo_sac_t h);
/* device buffers owned by the handle: params [n_params + 1] (last = log_alpha), target, Adam m/v,
 * grads (same layout; grads[n_params] = d alpha_loss / d log_alpha), logs[16]:
 * 0 q1_loss 1 q2_loss 2 mean q1 3 mean q2 4 alpha 5 pi_entropy 6 logp_pi 7 pi_global_norm
 * 8 q_global_norm 9 policy_loss  (the fetches of mopo.py:453-463; values of the last step) */
int mopo_sac_buffers(mopo_sac_t h, float** d_params, float** d_target, float** d_adam_m, float** d_adam_v,
                     float** d_grads, float** d_logs, int64_t* n_params);
/* Run n_steps grad steps (batch gather from env_pool/model_pool + update + Polyak) on `stream`.
 * Perf mode (all injected pointers NULL): Philox batch indices / policy noise; the step sequence is
 * captured once into a hipGraph and replayed.  Parity mode (n_steps = 1): d_idx[batch] int64 rows
 * (first n_env from the env pool), d_eps_s / d_eps_n [batch, act_dim] policy noise for pi(s), pi(s'). */
int mopo_sac_step(mopo_sac_t h, const mopo_pool_desc* env_pool, const mopo_pool_desc* model_pool,
                  int n_steps, uint64_t seed, const int64_t* d_idx, const float* d_eps_s,
                  const float* d_eps_n, void* stream);
int mopo_sac_set_graph(mopo_sac_t h, int enable);
/* Synchronises the device and reads the fused step's sticky hand-off timeout word (no reference
 * counterpart: the reference's TF session has no in-launch hand-offs).  A bounded wait that gave up
 * makes every later step hold its parameter / Adam / target updates and write NaN logs; this call
 * reports it (*timed_out = 1, returns -1 with mopo_last_error() set) and clears the word. */
int mopo_sac_check(mopo_sac_t h, int* timed_out);
/* Fault injection for tests: sets the timeout word as a give-up would. */
int mopo_sac_inject_timeout(mopo_sac_t h);
/* Target-network schedule (mopo.py:834-845 `if iteration % target_update_interval == 0:
 * _update_target()`, iteration = the epoch-local timestep of mopo.py:545-571, shared by the
 * n_train_repeat steps of a timestep, :790-795): the step whose device step counter is c updates the
 * targets iff ((c - base) / n_train_repeat) % interval == 0.  Enqueued on `stream` (it orders with
 * mopo_sac_step); the default {0, 1, 1} updates on every step. */
int mopo_sac_set_target_schedule(mopo_sac_t h, int64_t base, int64_t n_train_repeat, int64_t interval, void* stream);

/* softlearning SAC's action_prior (softlearning/algorithms/sac.py:42, 285-289): 0 'uniform' (MOPO's own
 * graph, mopo.py:364; the default), 1 'normal' -- the policy loss subtracts the standard-normal log-prob
 * of the policy's action. */
int mopo_sac_set_action_prior(mopo_sac_t h, int normal);
/* device<->device copy of a handle buffer (which: 0 params, 1 target, 2 adam_m, 3 adam_v, 4 grads,
 * 5 logs); to_handle=1 writes the handle's buffer from d_buf (e.g. loading a checkpoint). */
int mopo_sac_copy(mopo_sac_t h, int which, int to_handle, void* d_buf, int64_t count, void* stream);
/* Diagnostic builds only (MOPO_SAC_STAMPS=1; otherwise returns -1): per-workgroup phase timestamps
 * (s_memrealtime, 100 MHz) of the last step's five launches, u64 [launch][block][8]. */
int mopo_sac_debug_stamps(mopo_sac_t h, uint64_t* h_out, int64_t n);

/* ---- numpy legacy RandomState replica (host) ------------------------------------------ */
typedef struct mopo_mt_s* mopo_mt_t;
int mopo_mt_create(mopo_mt_t* out, uint32_t seed);
int mopo_mt_destroy(mopo_mt_t h);
int mopo_mt_seed(mopo_mt_t h, uint32_t seed);
/* state exchange with numpy.random.get_state()/set_state() */
int mopo_mt_set_state(mopo_mt_t h, const uint32_t* key624, int pos, int has_gauss, double gauss);
int mopo_mt_get_state(mopo_mt_t h, uint32_t* key624, int* pos, int* has_gauss, double* gauss);
int mopo_mt_normal(mopo_mt_t h, double* h_out, int64_t n);                  /* legacy_gauss */
int mopo_mt_randint(mopo_mt_t h, int64_t* h_out, int64_t n, int64_t low, int64_t high); /* randint(low, high, n) */
int mopo_mt_random_sample(mopo_mt_t h, double* h_out, int64_t n);
/* randint(low, high, n) written as int32 (BNN.train's bootstrap indices, bnn.py:402) */
int mopo_mt_randint_i32(mopo_mt_t h, int32_t* h_out, int64_t n, int64_t low, int64_t high);

#ifdef __cplusplus
}
#endif
#endif
