// Fused model rollout: MOPO._rollout_model (mopo/algorithms/mopo.py:723-765) on the device.
//
// Per horizon step (all launched back-to-back on one stream, no host synchronisation; the live
// row count, pool pointer and size stay on the device):
//   actor_kernel      get_action_meta (mopo.py:734) + obs/act half of the pool row + member pick
//   bnn_fwd ROLLOUT   ensemble forward; per row keeps only the selected member's mean/std and the
//                     max-over-members aleatoric norm (fake_env.py:66-81, 110) -> no [E,B,D] in HBM
//   rollout_post      sample, reward penalty, termination, next_obs/rew/term half of the pool row
//                     (fake_env.py:72, 90-115; mopo.py:750-751)
//   rollout_compact   order-preserving non-terminal compaction  obs = next_obs[~term] (mopo.py:753-758)
//   step_advance      steps_added / pool pointer & size (mopo.py:748; flexible_replay_pool.py:45-48)
#include "actor.h"

#include <vector>

namespace mopo {

enum { KC_START = 0, KC_ACTOR, KC_BNN, KC_POST, KC_COMPACT, KC_ADVANCE, KC_N };

struct Rollout {
  // optional live kernel timing: hipEvents recorded around every launch, per kernel class
  bool profile = false;
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> ev;
  std::vector<hipEvent_t> pool_ev;
  size_t ev_used = 0;
  Bnn* bnn = nullptr;
  int64_t Bmax = 0;
  int Hmax = 0;
  void* mem = nullptr;
  double* obs[2];
  int64_t* uid[2];
  float* act;
  float* wpk = nullptr;  // policy weights, fragment-major (pack_actor), repacked every run
  int wpk_hp = 0, wpk_f16 = 0;
  uint32_t* pen;
  int32_t* sel;
  float* xs;        // [B][32] the ensemble's scaled input rows (written by the actor)
  float* mean_sel;
  float* std_sel;
  float* mean_all = nullptr;  // [E][Bmax][D], allocated on first use (mean-distance penalty / deterministic)
  uint8_t* keep;
  int* blockcnt;
  int* cnt;  // [0] live rows this step, [1] survivors, [2 + k] rows of part k (split rollout)
  static constexpr int MAXSPLIT = 4;
  hipStream_t sp[MAXSPLIT] = {};        // streams of parts 1.. of the split rollout (run_impl)
  hipEvent_t ev_fork[MAXSPLIT] = {}, ev_join[MAXSPLIT] = {};
  // horizon state carried between step-range calls (mopo_rollout_run_staged_steps)
  int oc = 0, uc = 0, next_step = 0;
};

constexpr int PB = 256;  // rows per block in post / compact

// scoped hipEvent pair on the launch stream (only when profiling is enabled)
struct KTimer {
  Rollout* h; hipStream_t s; size_t idx = (size_t)-1;
  KTimer(Rollout* h_, int cls, hipStream_t s_) : h(h_), s(s_) {
    if (!h->profile) return;
    if (h->ev_used == h->ev.size()) {
      hipEvent_t a, b;
      // timing-only events: without the system-scope fence an event record does not write back and
      // invalidate the caches between launches (which made every timed ensemble launch ~10 % slower)
      if (hipEventCreateWithFlags(&a, hipEventDisableSystemFence) != hipSuccess ||
          hipEventCreateWithFlags(&b, hipEventDisableSystemFence) != hipSuccess) return;
      h->ev.push_back({cls, {a, b}});
    }
    idx = h->ev_used++;
    h->ev[idx].first = cls;
    (void)hipEventRecord(h->ev[idx].second.first, s);
  }
  ~KTimer() {
    if (idx != (size_t)-1) (void)hipEventRecord(h->ev[idx].second.second, s);
  }
};

// Start states (mopo.py:740-741): a block's 64 rows draw their source rows first (one thread each), then the
// block copies the 64 x O observations element-wise, so the f64 stores of consecutive threads are contiguous
// (one thread per row, each storing its 136-B row, took 26 us per 100k rows)
constexpr int START_ROWS = 64, START_TPB = 256;
__global__ __launch_bounds__(START_TPB) void rollout_start_kernel(const float* env_obs, int64_t env_size,
                                                                  const int64_t* idx_in, int O, int64_t B,
                                                                  uint64_t seed, uint32_t step, int64_t uid_offset,
                                                                  double* obs, int64_t* uid, int* cnt, int nsplit,
                                                                  int64_t bpart) {
  __shared__ int64_t srcs[START_ROWS];
  const int64_t r0 = blockIdx.x * (int64_t)START_ROWS;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    cnt[0] = (int)B;
    for (int k = 0; k < nsplit; ++k)  // split rollout: part k = rows [k bpart, min((k + 1) bpart, B))
      cnt[2 + k] = (int)(k + 1 < nsplit ? bpart : B - (int64_t)k * bpart);
  }
  if (threadIdx.x < START_ROWS && r0 + threadIdx.x < B) {
    const int64_t row = r0 + threadIdx.x;
    const int64_t u = uid_offset + row;
    int64_t src;
    if (idx_in) {
      src = idx_in[row];
    } else {  // perf mode of np.random.randint(0, size, B) (flexible_replay_pool.py:87)
      u32x4 c{(uint32_t)u, (uint32_t)((uint64_t)u >> 32), step, RNG_START};
      u32x4 r = philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
      src = (int64_t)(((uint64_t)r.x * (uint64_t)env_size) >> 32);
    }
    srcs[threadIdx.x] = src;
    uid[row] = u;
  }
  __syncthreads();
  const int nr = (int)(B - r0 < START_ROWS ? B - r0 : START_ROWS);
  for (int i = threadIdx.x; i < nr * O; i += START_TPB) {
    const int r = i / O, k = i - r * O;
    obs[(r0 + r) * O + k] = (double)env_obs[srcs[r] * O + k];
  }
}

struct PostArgs {
  int O;
  const int* cnt;
  const double* obs;        // current obs f64 [B][O]
  const int64_t* uid;
  const float* mean_sel;    // [B][D]
  const float* std_sel;
  const uint32_t* pen;
  const double* eps;        // injected [B][D] or NULL
  uint64_t seed; uint32_t step;
  float coeff;
  int term_kind;
  double* obs_next;         // [B][O]
  uint8_t* keep;
  int* blockcnt;
  mopo_pool_desc pool;
  int64_t stage_base;       // >= 0: staged layout
  int64_t pool_off;         // pool layout: rows go to (state[0] + pool_off + row) % max_size
  // every member's mean [E][all_stride][D] (the ensemble's mean_all), for the mean-distance penalty
  // (pen_dist, fake_env.py:98-108) and deterministic steps (det, fake_env.py:69-70, 84-86)
  const float* mean_all;
  int E;
  int64_t all_stride;
  int pen_dist, det;
};

// FakeEnv post-processing of one horizon step (fake_env.py:66-115) for POST_RPB rows per block, one
// 32-lane group per row and one lane per output dim d < D = O + 1: every load and store of the row's
// D values is contiguous across its lanes, and each lane draws only its own normal (Philox block
// d / 4, Box-Muller pair (d % 4) / 2: the same numbers the per-row order gives).  The row's next
// observation is assembled in LDS for the termination function.  With compaction, the kept rows of
// each PB-row chunk are counted into blockcnt (zeroed before the launch).
constexpr int POST_RPB = 8;
__global__ __launch_bounds__(256) void rollout_post_kernel(const PostArgs a) {
  __shared__ double srow[POST_RPB][33];
  __shared__ int kept[POST_RPB];
  const int tid = threadIdx.x, sub = tid & 31, rl = tid >> 5;
  const int64_t row = (int64_t)blockIdx.x * POST_RPB + rl;
  const int O = a.O, D = O + 1;
  const int64_t count = *a.cnt;
  const bool live = row < count;
  const bool on = live && sub < D;
  double s = 0.0;
  // member e's mean of this lane's dim after the residual add, in f32 as the reference's in-place
  // ensemble_model_means[:, :, 1:] += obs (fake_env.py:66)
  const double ob = on && sub >= 1 ? a.obs[row * O + sub - 1] : 0.0;
  auto member_mean = [&](int e) {
    const float m = a.mean_all[((int64_t)e * a.all_stride + row) * D + sub];
    return sub >= 1 ? (float)((double)m + ob) : m;
  };
  float pen_d = 0.f;
  if (a.pen_dist) {  // max_e || mean_e - mean_e' mean_e' || over the obs dims (fake_env.py:98-108)
    float sum = 0.f;
    if (on && sub >= 1)
      for (int e = 0; e < a.E; ++e) sum += member_mean(e);
    const float avg = sum / (float)a.E;                           // np.mean(axis=0), f32
    for (int e = 0; e < a.E; ++e) {
      const float dd = on && sub >= 1 ? member_mean(e) - avg : 0.f;
      float q = dd * dd;
#pragma unroll
      for (int o = 16; o >= 1; o >>= 1) q += __shfl_xor(q, o);       // the row's 32-lane group
      pen_d = fmaxf(pen_d, sqrtf(q));
    }
  }
  if (on && a.det) {  // samples = mean over ALL members of the means (fake_env.py:69-70, 84-86)
    float acc = 0.f;
    for (int e = 0; e < a.E; ++e) acc += member_mean(e);
    s = (double)(acc / (float)a.E);
    srow[rl][sub] = s;
  } else if (on) {
    float m = a.mean_sel[row * D + sub];
    if (sub >= 1) m = (float)((double)m + ob);                      // fake_env.py:66
    double e;
    if (a.eps) {
      e = a.eps[row * D + sub];
    } else {  // Philox normal `sub` of the row's stream (perf mode of fake_env.py:72)
      const int64_t u = a.uid[row];
      u32x4 c{(uint32_t)u, (uint32_t)((uint64_t)u >> 32) ^ ((uint32_t)(sub >> 2) << 20), a.step, RNG_OBS_NOISE};
      u32x4 r = philox(c, (uint32_t)a.seed, (uint32_t)(a.seed >> 32));
      float z0, z1;
      if (sub & 2) box_muller(r.z, r.w, z0, z1);
      else box_muller(r.x, r.y, z0, z1);
      e = (double)((sub & 1) ? z1 : z0);
    }
    s = (double)m + e * (double)a.std_sel[row * D + sub];          // fake_env.py:72
    srow[rl][sub] = s;
  }
  __syncthreads();
  const int64_t pos = a.stage_base >= 0 ? a.stage_base + row
                                        : (a.pool.d_state[0] + a.pool_off + row) % a.pool.max_size;
  if (on && sub >= 1) {                                            // next_obs = samples[:, 1:] (:90)
    a.obs_next[row * O + sub - 1] = s;
    a.pool.d_next_obs[pos * O + sub - 1] = (float)s;
  }
  if (sub == 0) {
    bool keep = false;
    if (live) {
      const bool term = term_fn(a.term_kind, &srow[rl][1], O);     // fake_env.py:91
      const float pen = a.pen_dist ? pen_d : __uint_as_float(a.pen[row]);
      const double pr = a.coeff != 0.f ? s - (double)a.coeff * (double)pen : s;   // fake_env.py:115
      a.pool.d_rew[pos] = (float)pr;                               // rewards = samples[:, :1] - c * penalty
      a.pool.d_term[pos] = term ? 1 : 0;
      keep = !term;
      if (a.keep) a.keep[row] = keep ? 1 : 0;
    }
    kept[rl] = keep ? 1 : 0;
  }
  if (a.blockcnt) {
    __syncthreads();
    if (tid == 0) {
      int t = 0;
#pragma unroll
      for (int i = 0; i < POST_RPB; ++i) t += kept[i];
      if (t) atomicAdd(a.blockcnt + (int64_t)blockIdx.x * POST_RPB / PB, t);  // PB % POST_RPB == 0
    }
  }
}

// The same post-processing for the common case (sampled steps, max-aleatoric penalty: neither pen_dist
// nor det) with one thread per (row, dim): POSTF_ROWS rows of D lanes each, packed back to back (the
// 32-lane groups above leave 14 of 32 lanes idle at D = 18).  Each row's pool position is computed once
// (its 64-bit modulo by one lane); values and draws are the ones rollout_post_kernel makes.
constexpr int POSTF_ROWS = 16, POSTF_MAXD = 64;   // PB % POSTF_ROWS == 0: a block's rows share one chunk
__global__ __launch_bounds__(1024) void rollout_post_flat_kernel(const PostArgs a) {
  __shared__ double srow[POSTF_ROWS][POSTF_MAXD];
  __shared__ int64_t spos[POSTF_ROWS];
  __shared__ int kept[POSTF_ROWS];
  const int tid = threadIdx.x;
  const int O = a.O, D = O + 1;
  const int64_t r0 = (int64_t)blockIdx.x * POSTF_ROWS;
  const int64_t count = *a.cnt;
  if (tid < POSTF_ROWS) {
    const int64_t row = r0 + tid;
    spos[tid] = a.stage_base >= 0 ? a.stage_base + row : (a.pool.d_state[0] + a.pool_off + row) % a.pool.max_size;
  }
  const int rl = tid / D, sub = tid - rl * D;
  const int64_t row = r0 + rl;
  const bool on = rl < POSTF_ROWS && row < count;
  double s = 0.0;
  if (on) {
    float m = a.mean_sel[row * D + sub];
    if (sub >= 1) m = (float)((double)m + a.obs[row * O + sub - 1]);    // fake_env.py:66
    double e;
    if (a.eps) {
      e = a.eps[row * D + sub];
    } else {  // Philox normal `sub` of the row's stream (perf mode of fake_env.py:72)
      const int64_t u = a.uid[row];
      u32x4 c{(uint32_t)u, (uint32_t)((uint64_t)u >> 32) ^ ((uint32_t)(sub >> 2) << 20), a.step, RNG_OBS_NOISE};
      u32x4 r = philox(c, (uint32_t)a.seed, (uint32_t)(a.seed >> 32));
      float z0, z1;
      if (sub & 2) box_muller(r.z, r.w, z0, z1);
      else box_muller(r.x, r.y, z0, z1);
      e = (double)((sub & 1) ? z1 : z0);
    }
    s = (double)m + e * (double)a.std_sel[row * D + sub];              // fake_env.py:72
    srow[rl][sub] = s;
  }
  __syncthreads();
  if (on && sub >= 1) {                                                // next_obs = samples[:, 1:] (:90)
    a.obs_next[row * O + sub - 1] = s;
    a.pool.d_next_obs[spos[rl] * O + sub - 1] = (float)s;
  }
  if (tid < POSTF_ROWS) {
    const int64_t rr = r0 + tid;
    bool keep = false;
    if (rr < count) {
      const bool term = term_fn(a.term_kind, &srow[tid][1], O);        // fake_env.py:91
      const double s0 = srow[tid][0];
      const float pen = __uint_as_float(a.pen[rr]);
      const double pr = a.coeff != 0.f ? s0 - (double)a.coeff * (double)pen : s0;   // fake_env.py:115
      const int64_t pos = spos[tid];
      a.pool.d_rew[pos] = (float)pr;
      a.pool.d_term[pos] = term ? 1 : 0;
      keep = !term;
      if (a.keep) a.keep[rr] = keep ? 1 : 0;
    }
    kept[tid] = keep ? 1 : 0;
  }
  if (a.blockcnt) {
    __syncthreads();
    if (tid == 0) {
      int t = 0;
#pragma unroll
      for (int i = 0; i < POSTF_ROWS; ++i) t += kept[i];
      if (t) atomicAdd(a.blockcnt + r0 / PB, t);
    }
  }
}

// MOPO_POST_FLAT=0 (A/B): the 32-lane-per-row post kernel for every step
static int post_flat() {
  static const int v = [] {
    const char* e = std::getenv("MOPO_POST_FLAT");
    return e ? std::atoi(e) : 1;
  }();
  return v;
}

__global__ __launch_bounds__(PB) void rollout_compact_kernel(int O, const int* blockcnt, const uint8_t* keepf,
                                                             const int* cnt, const double* obs_src,
                                                             double* obs_dst, const int64_t* uid_src,
                                                             int64_t* uid_dst, int* survivors) {
  __shared__ int red[PB];
  __shared__ int woff[PB / 64 + 1];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  int part = 0;
  for (int j = tid; j < (int)blockIdx.x; j += PB) part += blockcnt[j];
  red[tid] = part;
  __syncthreads();
  for (int st = PB / 2; st > 0; st >>= 1) {
    if (tid < st) red[tid] += red[tid + st];
    __syncthreads();
  }
  const int base = red[0];
  const int64_t row = blockIdx.x * (int64_t)PB + tid;
  const int64_t count = *cnt;
  const bool keep = row < count && keepf[row];
  const unsigned long long bal = __ballot(keep);
  const int pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0));
  if (lane == 0) woff[wid] = __popcll(bal);
  __syncthreads();
  if (tid == 0) {
    int acc = 0;
    for (int w = 0; w < PB / 64; ++w) { int c = woff[w]; woff[w] = acc; acc += c; }
    woff[PB / 64] = acc;
  }
  __syncthreads();
  if (keep) {
    const int64_t pos = base + woff[wid] + pre;
    for (int k = 0; k < O; ++k) obs_dst[pos * O + k] = obs_src[row * O + k];
    uid_dst[pos] = uid_src[row];
  }
  if (blockIdx.x == gridDim.x - 1 && tid == 0) *survivors = base + woff[PB / 64];
}

__global__ void step_advance_kernel(int* cnt, int64_t* steps, int i, int compacted, int64_t* pool_state,
                                    int64_t max_size) {
  const int64_t n = cnt[0];
  steps[i] = n;
  if (pool_state) {
    pool_state[0] = (pool_state[0] + n) % max_size;
    pool_state[1] = min(pool_state[1] + n, max_size);
  }
  if (compacted) cnt[0] = cnt[1];
}

// Steps [i0, i1) without compaction (halfcheetah): every step keeps all cnt[0] rows, so step i's
// rows went to pool_off = (i - i0) * n and one advance covers the whole range (staged: no pool).
__global__ void steps_advance_kernel(const int* cnt, int64_t* steps, int i0, int i1, int64_t* pool_state,
                                     int64_t max_size) {
  const int64_t n = cnt[0];
  for (int i = i0; i < i1; ++i) steps[i] = n;
  if (!pool_state) return;
  const int64_t tot = n * (i1 - i0);
  pool_state[0] = (pool_state[0] + tot) % max_size;
  pool_state[1] = min(pool_state[1] + tot, max_size);
}

static int split_parts() {  // MOPO_ROLLOUT_SPLIT=<parts> (0 or 1: one stream); default 2
  static const int v = [] {
    const char* e = std::getenv("MOPO_ROLLOUT_SPLIT");
    const int n = e ? std::atoi(e) : 2;
    return n < 1 ? 1 : (n > Rollout::MAXSPLIT ? Rollout::MAXSPLIT : n);
  }();
  return v;
}

// Horizon steps [i0, i1) of one rollout.  i0 == 0 draws the start states and repacks the policy;
// later ranges continue from the state the previous call left (obs ping-pong, live counts).  Staged
// rows of step i go to rows (i - i0) * B of the staging descriptor.
static int run_impl(Rollout* h, const mopo_rollout_args* a, const mopo_pool_desc* p, bool staged, int i0, int i1,
                    hipStream_t s) {
  MOPO_REQUIRE(a && p, "rollout: NULL argument");
  MOPO_REQUIRE(a->B >= 0 && a->B <= h->Bmax, "rollout: B exceeds the handle's max_batch");
  MOPO_REQUIRE(a->horizon >= 0 && a->horizon <= h->Hmax, "rollout: horizon exceeds max_horizon");
  MOPO_REQUIRE(a->term_kind >= 0 && a->term_kind < MOPO_TERM_KINDS, "rollout: unknown term_kind");
  MOPO_REQUIRE(a->d_env_obs && a->env_size > 0, "rollout: empty env pool");
  MOPO_REQUIRE(a->d_pi_params, "rollout: NULL policy params");
  MOPO_REQUIRE(a->d_model_inds || (a->d_elites && a->n_elites > 0), "rollout: elites required");
  MOPO_REQUIRE(p->d_obs && p->d_act && p->d_rew && p->d_term && p->d_next_obs, "rollout: NULL pool field");
  MOPO_REQUIRE(staged || p->d_state, "rollout: pool state required");
  MOPO_REQUIRE(a->d_steps, "rollout: d_steps output required");
  MOPO_REQUIRE(0 <= i0 && i0 <= i1 && i1 <= a->horizon, "rollout: bad step range");
  MOPO_REQUIRE(i0 == 0 || i0 == h->next_step, "rollout: step ranges must continue the previous call");
  MOPO_REQUIRE(!staged || p->max_size >= (int64_t)(i1 - i0) * a->B, "rollout: staging buffer too small");
  if (a->B == 0 || a->horizon == 0 || i0 == i1) return 0;
  Bnn* bnn = h->bnn;
  const int O = bnn->O, A = bnn->A, D = O + 1;
  const int64_t B = a->B;
  const int nblk = ceil_div((int)B, PB);
  const uint32_t step0 = a->epoch * 4096u;
  // live rows are compacted between steps (mopo.py:758); a one-step rollout never needs it: its
  // rows, terminal or not, all enter the pool (mopo.py:750-751) and no next step reads them
  const bool compact = a->term_kind != MOPO_TERM_HALFCHEETAH && a->horizon > 1;
  // no compaction, pool layout: positions advance by B per step and one launch advances the pool
  const bool batched_advance = !compact && !staged;
  // Split rollout (pool or staged layout): with no compaction the rows never interact, so two halves run their own
  // actor -> ensemble -> post chains on two streams; each half's kernels fill the CUs the other
  // half's launch tails and small kernels leave idle.  Identical results (rows, Philox streams and
  // pool positions do not depend on the split).  Off while profiling per kernel.
  // (a one-step rollout gains nothing from it: measured 150 -> 137M transitions/s for C3)
  const int nsplit = !compact && !h->profile && a->horizon > 1 ? std::min<int>(split_parts(), (int)(B / 2048)) : 1;
  const bool split = nsplit > 1;
  const int64_t bpart = !split ? B
                       : (B / nsplit + 63) / 64 * 64;   // equal parts (unequal halves measured slower)
  if (i0 == 0) {
    h->oc = 0;
    h->uc = 0;
    KTimer t(h, KC_START, s);
    hipLaunchKernelGGL(rollout_start_kernel, dim3((unsigned)((B + START_ROWS - 1) / START_ROWS)), dim3(START_TPB), 0, s,
                       a->d_env_obs, a->env_size,
                       a->d_start_idx, O, B, a->seed, step0, a->uid_offset, h->obs[0], h->uid[0], h->cnt, nsplit,
                       bpart);
  }
  if (i0 == 0) {
    MOPO_HIP(hipGetLastError());
    MOPO_REQUIRE(a->actor_dtype == DT_FP32 || a->actor_dtype == DT_F16X3 || a->actor_dtype == DT_BF16X6,
                 "rollout: actor_dtype must be 0 (fp32), 3 (bf16x6) or 4 (f16x3)");
    const int f16 = a->actor_dtype == DT_F16X3 ? 1 : (a->actor_dtype == DT_BF16X6 ? 2 : 0);   // pack_actor's split
    if (!h->wpk || h->wpk_hp != a->pi_hidden || h->wpk_f16 != f16) {
      if (h->wpk) (void)hipFree(h->wpk);
      MOPO_HIP(hipMalloc(&h->wpk, actor_packed_floats(O, a->pi_hidden, f16) * sizeof(float)));
      h->wpk_hp = a->pi_hidden;
      h->wpk_f16 = f16;
    }
    KTimer t(h, KC_START, s);
    if (pack_actor(a->d_pi_params, O, A, a->pi_hidden, h->wpk, s, f16)) return -1;
  }
  // every member's mean per row is needed by the mean-distance penalty and by deterministic steps
  const bool det = a->deterministic != 0;
  const bool pen_dist = a->penalty_learned_var == 0 && a->penalty_coeff != 0.f;
  const bool need_all = det || pen_dist;
  if (need_all && !h->mean_all)
    MOPO_HIP(hipMalloc(&h->mean_all, (size_t)bnn->E * h->Bmax * D * sizeof(float)));
  MOPO_REQUIRE(!a->rollout_random || a->d_act_uniform || !a->d_eps_act,
               "rollout: parity mode with rollout_random needs the injected uniforms (d_act_uniform)");
  int oc = h->oc, uc = h->uc;
  // one horizon step for rows [off, off + n) of the batch (live count in *cnt) on stream ss
  auto step_rows = [&](int i, int64_t off, int64_t n, int* cnt, hipStream_t ss, hipEvent_t after_actor) -> int {
    const uint32_t st = step0 + 1 + i;
    ActorArgs aa{};
    aa.P = a->d_pi_params; aa.Wpk = h->wpk; aa.O = O; aa.A = A; aa.Hp = a->pi_hidden;
    aa.obs = h->obs[oc] + off * O; aa.obs_f64 = 1; aa.B = n; aa.d_count = cnt;
    aa.eps = a->d_eps_act ? a->d_eps_act + ((int64_t)i * B + off) * A : nullptr;
    aa.seed = a->seed; aa.step = st; aa.d_uid = h->uid[uc] + off;
    aa.act = h->act + off * A;
    aa.pool_obs = p->d_obs; aa.pool_act = p->d_act; aa.pool_state = p->d_state; aa.pool_max = p->max_size;
    aa.stage_base = staged ? (int64_t)(i - i0) * B + off : -1;
    aa.pool_off = batched_advance ? (int64_t)(i - i0) * B + off : 0;
    aa.pen_zero = h->pen + off;
    aa.sel_out = det ? nullptr : h->sel + off;
    aa.sel_in = a->d_model_inds ? a->d_model_inds + (int64_t)i * B + off : nullptr;
    aa.rand_act = a->rollout_random;
    aa.dtype = a->actor_dtype;
    aa.alone = !split;
    aa.act_uni = a->d_act_uniform ? a->d_act_uniform + ((int64_t)i * B + off) * A : nullptr;
    aa.elites = a->d_elites; aa.n_elites = a->n_elites;
    aa.xs = h->xs + off * XS_STRIDE; aa.xs_mu = bnn->dev.mu; aa.xs_sigma = bnn->dev.sigma; aa.xs_in = bnn->dev.IN;
    {
      KTimer t(h, KC_ACTOR, ss);
      if (launch_actor(aa, ss)) return -1;
    }
    if (after_actor) MOPO_HIP(hipEventRecord(after_actor, ss));

    FwdArgs f{};
    f.in = FwdIn{h->obs[oc] + off * O, 1, O, h->act + off * A, 0, A};
    f.B = n; f.d_count = cnt; f.xs = h->xs + off * XS_STRIDE;
    f.pen_bits = h->pen + off; f.sel = det ? nullptr : h->sel + off; f.mean_sel = h->mean_sel + off * D;
    f.std_sel = h->std_sel + off * D;
    f.mean_all = need_all ? h->mean_all + off * D : nullptr;
    f.all_stride = h->Bmax;
    {
      KTimer t(h, KC_BNN, ss);
      if (launch_bnn_fwd(bnn, FWD_ROLLOUT, f, ss)) return -1;
    }

    PostArgs pa{};
    pa.O = O; pa.cnt = cnt; pa.obs = h->obs[oc] + off * O; pa.uid = h->uid[uc] + off;
    pa.mean_sel = h->mean_sel + off * D; pa.std_sel = h->std_sel + off * D; pa.pen = h->pen + off;
    pa.eps = a->d_eps_obs ? a->d_eps_obs + ((int64_t)i * B + off) * D : nullptr;
    pa.seed = a->seed; pa.step = st; pa.coeff = a->penalty_coeff; pa.term_kind = a->term_kind;
    pa.obs_next = h->obs[oc ^ 1] + off * O; pa.keep = compact ? h->keep : nullptr;
    pa.blockcnt = compact ? h->blockcnt : nullptr;
    pa.pool = *p; pa.stage_base = staged ? (int64_t)(i - i0) * B + off : -1;
    pa.pool_off = batched_advance ? (int64_t)(i - i0) * B + off : 0;
    pa.mean_all = f.mean_all; pa.E = bnn->E; pa.all_stride = h->Bmax; pa.pen_dist = pen_dist; pa.det = det;
    {
      KTimer t(h, KC_POST, ss);
      // with compaction the post kernel adds each block's kept rows into its PB-row chunk count
      if (compact) MOPO_HIP(hipMemsetAsync(h->blockcnt, 0, (size_t)nblk * sizeof(int), ss));
      if (post_flat() && !pen_dist && !det && D <= POSTF_MAXD)
        hipLaunchKernelGGL(rollout_post_flat_kernel, dim3(ceil_div((int)n, POSTF_ROWS)),
                           dim3((POSTF_ROWS * D + 63) / 64 * 64), 0, ss, pa);
      else
        hipLaunchKernelGGL(rollout_post_kernel, dim3(ceil_div((int)n, POST_RPB)), dim3(256), 0, ss, pa);
    }
    MOPO_HIP(hipGetLastError());
    return 0;
  };
  if (split) {
    for (int k = 1; k < nsplit; ++k)
      if (!h->sp[k]) {
        MOPO_HIP(hipStreamCreateWithFlags(&h->sp[k], hipStreamNonBlocking));
        // device-scope events (no system-scope cache write-back / invalidate at each record: the parts only
        // hand device memory to each other)
        MOPO_HIP(hipEventCreateWithFlags(&h->ev_fork[k], hipEventDisableTiming | hipEventDisableSystemFence));
        MOPO_HIP(hipEventCreateWithFlags(&h->ev_join[k], hipEventDisableTiming | hipEventDisableSystemFence));
      }
    // part k starts once part k - 1's first actor is done: the chains run offset by about one actor
    // launch instead of in lockstep, so their ensemble tails do not coincide
    for (int i = i0; i < i1; ++i) {
      for (int k = 0; k < nsplit; ++k) {
        hipStream_t ss = k == 0 ? s : h->sp[k];
        if (i == i0 && k > 0) MOPO_HIP(hipStreamWaitEvent(ss, h->ev_fork[k], 0));
        const int64_t off = k * bpart, n = k + 1 < nsplit ? bpart : B - off;
        if (step_rows(i, off, n, h->cnt + 2 + k, ss, i == i0 && k + 1 < nsplit ? h->ev_fork[k + 1] : nullptr))
          return -1;
      }
      oc ^= 1;
    }
    for (int k = 1; k < nsplit; ++k) {
      MOPO_HIP(hipEventRecord(h->ev_join[k], h->sp[k]));
      MOPO_HIP(hipStreamWaitEvent(s, h->ev_join[k], 0));
    }
    KTimer t(h, KC_ADVANCE, s);
    hipLaunchKernelGGL(steps_advance_kernel, dim3(1), dim3(1), 0, s, h->cnt, a->d_steps, i0, i1,
                       staged ? nullptr : p->d_state, p->max_size);
    MOPO_HIP(hipGetLastError());
  } else {
    for (int i = i0; i < i1; ++i) {
      if (step_rows(i, 0, B, h->cnt, s, nullptr)) return -1;
      if (compact) {
        KTimer t(h, KC_COMPACT, s);
        hipLaunchKernelGGL(rollout_compact_kernel, dim3(nblk), dim3(PB), 0, s, O, h->blockcnt, h->keep, h->cnt,
                           h->obs[oc ^ 1], h->obs[oc], h->uid[uc], h->uid[uc ^ 1], h->cnt + 1);
        MOPO_HIP(hipGetLastError());
        uc ^= 1;
      } else {
        oc ^= 1;
      }
      if (batched_advance) {
        if (i + 1 == i1) {
          KTimer t(h, KC_ADVANCE, s);
          hipLaunchKernelGGL(steps_advance_kernel, dim3(1), dim3(1), 0, s, h->cnt, a->d_steps, i0, i1, p->d_state,
                             p->max_size);
        }
      } else {
        KTimer t(h, KC_ADVANCE, s);
        hipLaunchKernelGGL(step_advance_kernel, dim3(1), dim3(1), 0, s, h->cnt, a->d_steps, i, compact ? 1 : 0,
                           staged ? nullptr : p->d_state, p->max_size);
      }
      MOPO_HIP(hipGetLastError());
    }
  }
  h->oc = oc;
  h->uc = uc;
  h->next_step = i1;
  return 0;
}

}  // namespace mopo

using namespace mopo;

extern "C" int mopo_rollout_create(mopo_rollout_t* out, mopo_bnn_t bnn, int64_t max_batch, int max_horizon) {
  MOPO_REQUIRE(out && bnn, "mopo_rollout_create: NULL argument");
  MOPO_REQUIRE(max_batch > 0 && max_batch < (1LL << 30), "mopo_rollout_create: bad max_batch");
  Bnn* b = reinterpret_cast<Bnn*>(bnn);
  MOPO_REQUIRE(b->O + 1 <= 32, "mopo_rollout_create: obs_dim must be < 32");
  Rollout* h = new Rollout();
  h->bnn = b; h->Bmax = max_batch; h->Hmax = max_horizon;
  const int O = b->O, A = b->A, D = O + 1;
  const int64_t B = max_batch;
  const int nblk = ceil_div((int)B, PB);
  size_t sz[] = {(size_t)B * O * 8, (size_t)B * O * 8, (size_t)B * 8, (size_t)B * 8, (size_t)B * A * 4,
                 (size_t)B * 4,     (size_t)B * 4,     (size_t)B * D * 4, (size_t)B * D * 4, (size_t)B,
                 (size_t)nblk * 4,  32,                (size_t)B * XS_STRIDE * 4};
  size_t off[13], tot = 0;
  for (int i = 0; i < 13; ++i) { off[i] = tot; tot += (sz[i] + 255) & ~(size_t)255; }
  if (hipMalloc(&h->mem, tot) != hipSuccess) { delete h; return fail("mopo_rollout_create: out of device memory"); }
  char* m = (char*)h->mem;
  h->obs[0] = (double*)(m + off[0]); h->obs[1] = (double*)(m + off[1]);
  h->uid[0] = (int64_t*)(m + off[2]); h->uid[1] = (int64_t*)(m + off[3]);
  h->act = (float*)(m + off[4]); h->pen = (uint32_t*)(m + off[5]); h->sel = (int32_t*)(m + off[6]);
  h->mean_sel = (float*)(m + off[7]); h->std_sel = (float*)(m + off[8]); h->keep = (uint8_t*)(m + off[9]);
  h->blockcnt = (int*)(m + off[10]); h->cnt = (int*)(m + off[11]); h->xs = (float*)(m + off[12]);
  *out = reinterpret_cast<mopo_rollout_t>(h);
  return 0;
}

extern "C" int mopo_rollout_profile(mopo_rollout_t hh, int enable) {
  Rollout* h = reinterpret_cast<Rollout*>(hh);
  MOPO_REQUIRE(h, "mopo_rollout_profile: NULL handle");
  h->profile = enable != 0;
  h->ev_used = 0;
  return 0;
}

extern "C" int mopo_rollout_profile_read(mopo_rollout_t hh, double* ms, int64_t* launches, int n) {
  Rollout* h = reinterpret_cast<Rollout*>(hh);
  MOPO_REQUIRE(h && ms && launches, "mopo_rollout_profile_read: NULL argument");
  for (int i = 0; i < n; ++i) { ms[i] = 0.0; launches[i] = 0; }
  for (size_t i = 0; i < h->ev_used; ++i) {
    auto& e = h->ev[i];
    MOPO_HIP(hipEventSynchronize(e.second.second));
    float t = 0.f;
    MOPO_HIP(hipEventElapsedTime(&t, e.second.first, e.second.second));
    if (e.first < n) { ms[e.first] += t; launches[e.first] += 1; }
  }
  h->ev_used = 0;
  return 0;
}

extern "C" int mopo_rollout_destroy(mopo_rollout_t hh) {
  Rollout* h = reinterpret_cast<Rollout*>(hh);
  if (!h) return 0;
  for (auto& e : h->ev) { (void)hipEventDestroy(e.second.first); (void)hipEventDestroy(e.second.second); }
  for (int k = 0; k < Rollout::MAXSPLIT; ++k) {
    if (h->ev_fork[k]) (void)hipEventDestroy(h->ev_fork[k]);
    if (h->ev_join[k]) (void)hipEventDestroy(h->ev_join[k]);
    if (h->sp[k]) (void)hipStreamDestroy(h->sp[k]);
  }
  if (h->mem) (void)hipFree(h->mem);
  if (h->wpk) (void)hipFree(h->wpk);
  if (h->mean_all) (void)hipFree(h->mean_all);
  delete h;
  return 0;
}

extern "C" int mopo_rollout_run(mopo_rollout_t hh, const mopo_rollout_args* a, const mopo_pool_desc* p,
                                void* stream) {
  Rollout* h = reinterpret_cast<Rollout*>(hh);
  MOPO_REQUIRE(h, "mopo_rollout_run: NULL handle");
  MOPO_REQUIRE(a, "mopo_rollout_run: NULL args");
  return run_impl(h, a, p, false, 0, a->horizon, (hipStream_t)stream);
}

extern "C" int mopo_rollout_run_staged(mopo_rollout_t hh, const mopo_rollout_args* a, const mopo_pool_desc* p,
                                       void* stream) {
  Rollout* h = reinterpret_cast<Rollout*>(hh);
  MOPO_REQUIRE(h, "mopo_rollout_run_staged: NULL handle");
  MOPO_REQUIRE(a, "mopo_rollout_run_staged: NULL args");
  return run_impl(h, a, p, true, 0, a->horizon, (hipStream_t)stream);
}

extern "C" int mopo_rollout_run_staged_steps(mopo_rollout_t hh, const mopo_rollout_args* a, const mopo_pool_desc* p,
                                             int step_begin, int step_end, void* stream) {
  Rollout* h = reinterpret_cast<Rollout*>(hh);
  MOPO_REQUIRE(h && a, "mopo_rollout_run_staged_steps: NULL argument");
  return run_impl(h, a, p, true, step_begin, step_end, (hipStream_t)stream);
}
