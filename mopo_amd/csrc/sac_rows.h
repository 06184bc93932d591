// Row-block kernels of the SAC step (sac.hip): the forward of all eight MLP instances and the critics'
// first-layer backward, each as ONE launch whose workgroups own 16 batch rows x 64 columns of a
// 256-wide layer, with every cross-column reduction the next stage needs (output layers, the policy
// head, the critics' action gradient) carried as per-block PARTIAL dot products that the consumer
// sums in a fixed order (bit-reproducible, no atomics, no in-launch hand-off).
//
//   F1  sac_fwd_kernel<false>: pi(s), pi(s'), Q1(s,a), Q2(s,a): layer 1 (recomputed per block from the
//       <= 31 inputs) + layer 2 + the partial dots of the block's 64 outputs with the output layer
//       ([W_mean | W_log_std] for the policy, W3 for a critic)                   (mopo.py:298-324)
//   F2  sac_fwd_kernel<true>: Q1/Q2(s, pi(s)) with the main critics, Qt1/Qt2(s', pi(s')) with the
//       targets; the prologue sums pi's partials of its 16 rows into the squashed-Gaussian head
//       (action, log-prob, noise: mopo.py:282-308) -- the action is the critic's layer-1 input; the
//       main critics' blocks also emit their share of d Q / d action (dq = 1) for the policy backward
//   B1  sac_dh1_kernel: dh1 = (dq (x) W3 * (h2 > 0)) W2^T * (h1 > 0) for Q1/Q2(s,a), the prologue forming
//       each row's dq from the critics' partials (the TD target y, mopo.py:380-404); the policy's
//       row-local backward chain (policy_rows_block, from F2's partials with the min-Q selection,
//       mopo.py:367-377); the step control (lr_t, beta powers, target-update flag: mopo.py:407-447); and
//       the gather of the next step's batch
// The weight gradients and the batch loss tail follow in one more launch (sac_wgrad.h).
#pragma once
#include "gemm_group.h"

namespace mopo {

// ---- SAC batch gather (_training_batch, mopo.py:801-821): rows [0, n_env) from the env pool, rest
// from the model pool; each index uniform over the pool's live size (Philox) unless injected.  One
// thread per (row, field column): every thread derives its row's source index itself (the Philox
// draw is cheap), so the work is two dependent memory latencies (pool size + counter, then the field)
// with no barrier.  Run by sac_gather_kernel (sac.hip) and by the gather blocks of sac_dh1_kernel.
struct Batch {
  float *sa, *xpi, *xn, *rew, *term;  // [s, a], [s, pi(s)], [s', pi(s')], r, done
  int64_t* idx;                       // [n] sampled rows
};

struct GatherArgs {
  mopo_pool_desc env, mod;
  int n, n_env, O, A;                // n: batch rows
  const int64_t* idx_in;             // injected rows or NULL (Philox draw)
  uint64_t seed;
  const int64_t* iter;
  int iter_add;                      // the step the batch is for: *iter + iter_add (B1 gathers the next step's)
  Batch out;
};

// field c of batch row r (obs | act | next_obs | rew | term)
static __device__ __forceinline__ void gather_elem(const GatherArgs& g, int r, int c) {
  const int O = g.O, A = g.A, W = O + A;
  const bool fe = r < g.n_env;
  const mopo_pool_desc& p = fe ? g.env : g.mod;
  int64_t src;
  if (g.idx_in) {
    src = g.idx_in[r];
  } else {
    const uint64_t size = (uint64_t)p.d_state[1];
    const int64_t it = *g.iter + g.iter_add;
    u32x4 cc{(uint32_t)r, (uint32_t)it, (uint32_t)((uint64_t)it >> 32), RNG_SAC};
    u32x4 q = philox(cc, (uint32_t)g.seed, (uint32_t)(g.seed >> 32));
    src = (int64_t)(((uint64_t)q.x * size) >> 32);
  }
  const Batch& b = g.out;
  if (c == 0) b.idx[r] = src;
  if (c < O) {
    const float v = p.d_obs[src * O + c];
    b.sa[r * W + c] = v;
    b.xpi[r * W + c] = v;
  } else if (c < O + A) {
    b.sa[r * W + c] = p.d_act[src * A + (c - O)];
  } else if (c < 2 * O + A) {
    b.xn[r * W + (c - O - A)] = p.d_next_obs[src * O + (c - O - A)];
  } else if (c == 2 * O + A) {
    b.rew[r] = p.d_rew[src];
  } else {
    b.term[r] = (float)p.d_term[src];
  }
}

// ---- the policy's row-local backward chain (mopo.py:337-377 through the critics at (s, pi(s))), run by
// the policy-row blocks of sac_dh1_kernel: block (rb, cq) owns batch rows [16 rb, 16 rb + 16) and
// columns [128 cq, 128 cq + 128) of the policy's first hidden layer.
//   dx_a   = -1/n d Q_sel(s, pi) / d action                            (Q_sel = the smaller critic per row)
//            -- the sum of the per-column-block partials sac_fwd_kernel<true> wrote (dq = 1), of the
//            critic tf.minimum selects (mopo.py:367-377; its gradient goes to x where x <= y)
//   dhead  = squashed-Gaussian head backward (mean, log_std; alpha / n on the log-prob)
//   dh2p   = (dhead_mu Wm^T + dhead_ls Wl^T) * (h2p > 0)               (all H columns, in LDS)
//   dh1p   = dh2p W2p^T * (h1p > 0)                                     (this block's columns, MFMA)
// Every quantity before dh1p is row-local, so each column block recomputes it (cheap: ncq partials
// per action, K = 2A per dh2p value) and only cq == 0 stores dhead and dh2p, which the policy weight
// gradients of the next launch read with dh1p.
constexpr int OPW = 16;              // floats per (column block, row) record of the policy's output partials
constexpr int DPW = 8;               // ... of the action-gradient partials (A <= 8); a critic's is 1 float
constexpr int EPW = 8;               // row stride of the step's policy-noise records eps_out (A <= 8)
constexpr int MAX_NCQ = 4;           // column blocks of 64 (H <= 256)
constexpr int DH2_TILES = 4;         // dh2p column tiles per wave (H <= 256 over >= 4 waves)

// Row-block-exclusive layouts of everything F2 hands to B1 (so the fused F2 + B1 launch, sac_f2b1_kernel, can
// hand it over in-launch): every 128-B line holds ONE 16-row block's values, so no workgroup ever caches a line
// of a row block whose producers have not finished.  Per-row records are strided by ns = n rounded up to 16.
static __device__ __forceinline__ int rows_ns(int n) { return (n + 15) & ~15; }
// a critic's output-layer partial of (column block cq, row r): [nrb][ncq][16]
static __device__ __forceinline__ int qp_idx(int cq, int r, int ncq) { return ((r >> 4) * ncq + cq) * 16 + (r & 15); }
// a head's log-prob of row r: [nrb][32] (the second half of each 128-B line unused)
static __device__ __forceinline__ int lp_idx(int r) { return (r >> 4) * 32 + (r & 15); }
// a store the fused launch hands over in-launch: write-through (sc1), drained before the row block's counter add
template <bool SC1>
static __device__ __forceinline__ void hstore(float* p, float v) {
  if constexpr (SC1) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}

// ---- in-launch hand-off of the fused F2 + B1 launch (cdna_hip_programming.md Guideline 16, R1 form): the
// producer's payload stores are write-through, every wave drains them, the workgroup barrier, then ONE lane's
// agent-scope add to its row block's counter; the consumer polls that word (one lane, relaxed), then ONE agent
// acquire, the drain and the workgroup barrier before the plain loads of the handed-off rows.  A consumer only
// ever waits on producers with lower workgroup ids (all of them are dispatched first), and every spin is bounded:
// on a give-up it sets the sticky timeout word, which the loss tail turns into NaN logs.
constexpr unsigned SAC_SPIN_LIMIT = 1u << 19;
#ifndef MOPO_SAC_LDOFF
#define MOPO_SAC_LDOFF 1   // the forward blocks' W1 / W2 operand loads at plain offsets (bounds by the range)
#endif
#ifndef MOPO_SAC_LDOFF2
#define MOPO_SAC_LDOFF2 0  // the same for step 7's, B1's critic and policy-row W2 loads (H a multiple of 64):
                           // 37.3-37.9 vs 37.0-37.2 us/step with the forward blocks' alone (same box), so off
#endif
constexpr int SYNC_STRIDE = 32;      // one counter per 128-B line: counter c at sync[c * SYNC_STRIDE]
#ifndef MOPO_SAC_B1_LATE
// 1: in the F1 + F2 + B1 launch a B1 block waits for its row block's F1 blocks before issuing ANY operand
// (its loads then do not compete with F1's); 0: it prefetches the weights first -- measured 37.9-38.0 vs
// 39.6-39.9 us/step for 1 (profiles/r05_sac_ab_fused.txt): the prefetch matters more than F1's slowdown
#define MOPO_SAC_B1_LATE 0
#endif
constexpr bool B1_LATE = MOPO_SAC_B1_LATE != 0;
// the counters of one row block rb: sync[(SYNC_N rb + class) SYNC_STRIDE]; the timeout word after the last
// F1 blocks: pi(s), pi(s'), Q(s, a); F2: main / target critics; B1: step control + gather, critic dh1, policy rows
enum { SYNC_PI_S = 0, SYNC_PI_N = 1, SYNC_Q_SA = 2, SYNC_F2_MAIN = 3, SYNC_F2_TGT = 4, SYNC_B1_CTL = 5, SYNC_B1_Q = 6,
       SYNC_B1_PI = 7, SYNC_N = 8 };
// global words after the per-row-block counters (x SYNC_STRIDE): the sticky timeout word (set by a give-up, read
// and cleared by the host: mopo_sac_check)
enum { SYNC_TMO = 0, SYNC_GLOBAL = 1 };
static __device__ __forceinline__ unsigned* sync_at(unsigned* sync, int rb, int c) {
  return sync + (SYNC_N * rb + c) * SYNC_STRIDE;
}
#ifndef MOPO_SAC_FUSE_ACQ
#define MOPO_SAC_FUSE_ACQ 1          // the consumer's agent acquire after the poll (A/B knob)
#endif
static __device__ __forceinline__ void handoff_signal(unsigned* cnt) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the same wait over ONE class of every row block (lane r of wave 0 polls row block r's counter, nrb <= 64)
static __device__ __forceinline__ void handoff_wait_rows(unsigned* sync, int nrb, int cls, unsigned target,
                                                         unsigned* tmo) {
  if (threadIdx.x < 64) {
    const int r = threadIdx.x;
    unsigned spins = 0;
    while (true) {
      const unsigned v = r < nrb ? __hip_atomic_load(sync + (SYNC_N * r + cls) * SYNC_STRIDE, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT) : target;
      if (__all(v >= target)) break;
      __builtin_amdgcn_s_sleep(2);
      if (++spins > SAC_SPIN_LIMIT) {
        if (r == 0) __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
#if MOPO_SAC_FUSE_ACQ
    if (r == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
#endif
  }
  __syncthreads();
}

static __device__ __forceinline__ void handoff_wait(unsigned* cnt, unsigned target, unsigned* tmo) {
  if (threadIdx.x == 0) {
    unsigned spins = 0;
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > SAC_SPIN_LIMIT) {
        __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
#if MOPO_SAC_FUSE_ACQ
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  }
  __syncthreads();
}

struct PolicyRows {
  int n, O, A, H, ncq;
  const float* dapart[2];            // Q1 / Q2 at (s, pi(s)): [ncq][n][DPW] partials of dh1 W1[O:]^T (dq = 1)
  // Q1 / Q2(s, pi) = b3 + the critics' forward partials [ncq][n]: the min-Q selection
  const float* qpart[2]; const float* b3[2];
  const float* head_s;               // [n][2A] mean | raw log_std
  const float* eps_s; int lde;       // [n][lde]: F1's draws (EPW) or the injected noise (A)
  const float* log_alpha;
  const float* Wm; const float* Wl;  // [H][A]
  const float* h2p; const float* h1p;// [n][H]
  const float* W2p;                  // [H][H]
  float* dhead; float* dh2p; float* dh1p;
  int prior;                         // 1: action_prior 'normal' (softlearning sac.py:285-289): + a / n on d L / d a
};


// Latency layout: every global operand of the chain is loaded in ONE burst of unconditional
// (range-checked) loads at the start -- the action-gradient partials and head inputs, Wm / Wl / h2p at
// this thread's dh2p column, this wave's W2p operands of the dh1p tile and the h1p mask -- so the
// block pays one memory latency, then computes.
// S: >= 16 (H + 4) floats of LDS; hs: >= 3 * 128 floats.  Blocks of 4 or 8 waves (64 or 128 dh1p
// columns).  H % 16 == 0, H <= 256 (one dh2p column per thread), A <= 8.
// FZ >= 1 (fused launches): the operands of earlier launches are issued first, then the block waits for its
// row block's F2 producers (sync class SYNC_F2_MAIN >= 2 ncq) and loads what they handed over; FZ = 2 (F1 +
// F2 + B1): the pi(s) activations (h1p, h2p) are loaded after the row block's pi(s) blocks of F1 are done.
template <int FZ = 0>
static __device__ __forceinline__ void policy_rows_block(const PolicyRows& c, int x, float* S, float* hs,
                                                         const Stamps& st, unsigned* sync = nullptr,
                                                         int nrb = 0) {
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = c.H, A = c.A, HS = H + 4, n = c.n;
  const int pcols = 16 * (int)(blockDim.x >> 6);   // dh1p columns of the block: one 16-wide tile per wave
  const int ncq = (H + pcols - 1) / pcols;
  const int rb = x / ncq, cq = x % ncq, r0 = rb * 16;
  const int li = lane & 15, lk = lane >> 4;
  // ---- the burst: head inputs, Wm / Wl / h2p at this thread's dh2p column, this wave's W2p operands of
  //      the dh1p tile and the h1p mask, the critics' partials
  const int hr = tid >> 3, hj = tid & 7, hrow = r0 + hr;
  const bool hon = tid < 128 && hj < A && hrow < n;
  const int ns = rows_ns(n);
  float mu, raw, ep;
  float qv[2][MAX_NCQ];                // Q1 / Q2(s, pi) partials of this thread's row: the chain's first link
  float dap[2][MAX_NCQ];
  auto handed = [&]() {                // what F2 wrote: head, critic partials, action-gradient partials
    const auto dh = rsrc(c.head_s, (int64_t)n * 2 * A), de = rsrc(c.eps_s, (int64_t)n * c.lde);
    mu = bload(dh, hon ? hrow * 2 * A + hj : -1);
    raw = bload(dh, hon ? hrow * 2 * A + A + hj : -1);
    ep = bload(de, hon ? hrow * c.lde + hj : -1);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const auto dq = rsrc(c.qpart[i], (int64_t)c.ncq * ns);
      const auto dp = rsrc(c.dapart[i], (int64_t)c.ncq * ns * DPW);
#pragma unroll
      for (int q = 0; q < MAX_NCQ; ++q) {
        qv[i][q] = bload(dq, (hon && q < c.ncq) ? qp_idx(q, hrow, c.ncq) : -1);
        dap[i][q] = bload(dp, (hon && q < c.ncq) ? (q * ns + hrow) * DPW + hj : -1);
      }
    }
  };
  if constexpr (FZ == 0) handed();
  if constexpr (FZ >= 2 && B1_LATE)   // F1's pi(s) blocks of this row block first, then every operand
    handoff_wait(sync_at(sync, rb, SYNC_PI_S), (unsigned)c.ncq, sync + SYNC_N * nrb * SYNC_STRIDE);
  const float la = *c.log_alpha;
  float b3v[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) b3v[i] = *c.b3[i];
  // dh2p tiles of this wave: 16 columns each, tiles w, w + nw, ... (at most DH2_TILES)
  const int nw = (int)(blockDim.x >> 6), nt2 = (H + 15) >> 4;
  const auto dwm = rsrc(c.Wm, (int64_t)H * A), dwl = rsrc(c.Wl, (int64_t)H * A), dh2 = rsrc(c.h2p, (int64_t)n * H);
  float wb[DH2_TILES][4], h2v[DH2_TILES][4];   // B(k, c) = k < 8 ? Wm[c][k] : Wl[c][k - 8]; lane k = 4 s + lk
#pragma unroll
  for (int q = 0; q < DH2_TILES; ++q) {
    const int c2 = (w + q * nw) * 16 + li;
    const bool on = w + q * nw < nt2 && c2 < H;
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      const int k = 4 * (s2 & 1) + lk;
      wb[q][s2] = bload(s2 < 2 ? dwm : dwl, (on && k < A) ? c2 * A + k : -1);
    }
  }
  auto f1_loads = [&]() {             // F1's pi(s) activations at this thread's dh2p columns
#pragma unroll
    for (int q = 0; q < DH2_TILES; ++q) {
      const int c2 = (w + q * nw) * 16 + li;
      const bool on = w + q * nw < nt2 && c2 < H;
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) h2v[q][s2] = bload(dh2, on ? (r0 + 4 * lk + s2) * H + c2 : -1);  // rows >= n: 0
    }
  };
  if constexpr (FZ < 2 || B1_LATE) f1_loads();
  const int j0 = cq * pcols + w * 16, col = j0 + li;
  const bool tile_on = j0 < H;
  const auto dw2 = rsrc(c.W2p, (int64_t)H * H);
  const int boff = (tile_on ? col : 0) * H;
  f32x4 bq[16];                       // B(k, j) = W2p[j][k]: lane (li, lk) contracts k = 64 lk + 4 t + u
  if (MOPO_SAC_LDOFF2 && (H & 63) == 0) {
    // k < H exactly when 64 lk < H: one base per lane, plain offsets
    const int vb = 64 * lk < H ? (boff + 64 * lk) * 4 : (1 << 30);
#pragma unroll
    for (int t = 0; t < 16; ++t)
      bq[t] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(dw2, vb + 16 * t, 0, 0));
  } else {
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int k = 64 * lk + 4 * t;
      bq[t] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(dw2, (k < H ? boff + k : -4) * 4, 0, 0));
    }
  }
  const auto dm1 = rsrc(c.h1p, (int64_t)n * H);
  float m1[4];
  auto m1_loads = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i) m1[i] = bload(dm1, col < H ? (r0 + 4 * lk + i) * H + col : -1);
  };
  if constexpr (FZ < 2 || B1_LATE) m1_loads();
  if constexpr (FZ >= 1) {
    unsigned* tmo = sync + SYNC_N * nrb * SYNC_STRIDE;
    stamp(st, 5);
    if constexpr (FZ >= 2 && !B1_LATE) {
      handoff_wait(sync_at(sync, rb, SYNC_PI_S), (unsigned)c.ncq, tmo);
      f1_loads();
      m1_loads();
    }
    handoff_wait(sync_at(sync, rb, SYNC_F2_MAIN), 2u * (unsigned)c.ncq, tmo);
    stamp(st, 6);
    handed();
  }
  stamp(st, 1);
  // ---- squashed-Gaussian head backward (mopo.py:282-308 differentiated; pi_loss mopo.py:371-377)
  float* dmu_s = hs + 128;
  float* dls_s = hs + 256;
  if (tid < 128) {
    float dmu = 0.f, dls = 0.f;
    if (hon) {
      float da = 0.f;                                               // -dmin q / da through Q1 / Q2:
      float q12[2];                                                 // the selected critic's partials, x -1/n
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        float qs = b3v[i];
#pragma unroll
        for (int q = 0; q < MAX_NCQ; ++q) qs += qv[i][q];
        q12[i] = qs;
      }
      const int sel = q12[0] <= q12[1] ? 0 : 1;
#pragma unroll
      for (int q = 0; q < MAX_NCQ; ++q) da += sel == 0 ? dap[0][q] : dap[1][q];
      da *= -1.f / (float)n;
      const float g = expf(la) / (float)n;                         // d L_pi / d logp (stop_gradient(alpha))
      const float ls = fminf(fmaxf(raw, -20.f), 2.f);
      const float sd = expf(ls);
      const float u = mu + ep * sd;
      const float a = tanhf(u);
      const float inv = 1.f / (sd + 1e-8f);
      const float zz = (u - mu) * inv;
      if (c.prior) da += a * (1.f / (float)n);                       // -mean(log N(a; 0, I))' = a / n
      float du = da * (1.f - a * a);                                // tanh grad (y-based)
      du += g * (-zz * inv);                                        // gaussian_likelihood wrt x
      du += g * (2.f - 4.f / (1.f + expf(2.f * u)));                // squash correction: 2 - 4 sigmoid(-2u)
      dmu = g * zz * inv + du;
      const float dstd = g * zz * zz * inv + du * ep;
      dls = -g + dstd * sd;
      if (!(raw >= -20.f && raw <= 2.f)) dls = 0.f;                 // clip_by_value grad
      if (cq == 0) {
        hstore<false>(&c.dhead[(int64_t)hrow * 2 * A + hj], dmu);
        hstore<false>(&c.dhead[(int64_t)hrow * 2 * A + A + hj], dls);
      }
    }
    dmu_s[tid] = dmu;
    dls_s[tid] = dls;
  }
  lds_barrier();
  stamp(st, 2);
  // ---- dh2p = dhead [dWm; dWl]^T (K = 16: mu parts 0..7, log-std parts 8..15) masked by h2p > 0 ->
  //      LDS rows of stride HS (and dh2p in HBM from the cq == 0 blocks)
  {
    float av[4];
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) av[s2] = (s2 < 2 ? dmu_s : dls_s)[li * 8 + 4 * (s2 & 1) + lk];
#pragma unroll
    for (int q = 0; q < DH2_TILES; ++q) {
      if (w + q * nw >= nt2) break;
      f32x4 d = zero4();
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) d = mfma4(av[s2], wb[q][s2], d);
      const int c2 = (w + q * nw) * 16 + li;
      if (c2 < H) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {                                // D: row 4 lk + i, col li
          const int row = 4 * lk + i;
          const float v = h2v[q][i] > 0.f ? d[i] : 0.f;
          S[row * HS + c2] = v;
          if (cq == 0 && r0 + row < n) hstore<false>(&c.dh2p[(int64_t)(r0 + row) * H + c2], v);
        }
      }
    }
  }
  lds_barrier();
  stamp(st, 3);
  // ---- dh1p tile = dh2p W2p^T * (h1p > 0): rows r0.., columns j0.. (wave w)
  if (!tile_on) return;
  f32x4 acc[4] = {zero4(), zero4(), zero4(), zero4()};
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    const int k = 64 * lk + 4 * t;
    const f32x4 a = k < H ? *reinterpret_cast<const f32x4*>(S + li * HS + k) : zero4();
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = mfma4(a[u], bq[t][u], acc[u]);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = r0 + 4 * lk + i;                                // D: col li, row 4 lk + i
    if (row < n && col < H) {
      const float v = acc[0][i] + acc[1][i] + acc[2][i] + acc[3][i];
      hstore<false>(&c.dh1p[(int64_t)row * H + col], m1[i] > 0.f ? v : 0.f);
    }
  }
}

constexpr int RB_COLS = 64;  // second-layer columns per workgroup (4 waves x 16); OPW: gemm_group.h

struct FwdInst {
  const float* x; int ldx; int kx;   // layer-1 inputs from memory: columns [0, kx) of x[n][ldx]
  int k1;                            // layer-1 input width (F2: kx + A, the action from the head)
  const float* w1; const float* b1;  // [k1][H], [H]
  const float* w2; const float* b2;  // [H][H], [H]
  float* h1; float* h2;              // stored for the backward pass when non-NULL
  const float* wo; const float* wo2; // output layer [H][nout]: columns [0, split) from wo (ld split),
  int nout, split;                   //   [split, nout) from wo2 (ld nout - split)
  float* opart;                      // [ncq][n][OPW] (policy) / [ncq][n] (critic) partial dots of the block's 64 outputs
  int head;                          // F2: 0 = pi(s) head (s, pi(s)), 1 = pi(s') head
  // F2 (s, pi) critics: the block's partial of d Q / d action = (W3 * (h2 > 0)) W2^T * (h1 > 0) W1[O:]^T
  // over its 64 columns (dq = 1; the policy-row consumer applies the min-Q selection and -1/n)
  const float* w1a;                  // W1[O:] = the action rows [A][H], or NULL
  float* dapart;                     // [ncq][n][DPW]
};

struct FwdHead {                     // F2: the squashed-Gaussian head of pi(s) / pi(s') (HeadCtx math)
  const float* opart[2];             // pi(s), pi(s') partials: [ncq][n][OPW], mean j < A, log_std A + j
  const float* bm; const float* bl;  // output biases
  const float* eps_in[2];            // injected noise [n][A] or NULL (Philox)
  float* eps_out[2]; float* head_out[2]; float* logp[2];   // written by the designated blocks
  uint64_t seed; const int64_t* iter;
  int gen_eps;                       // F1: bit i draws head i's noise into eps_out[i] (not injected; F2 loads it)
};

struct FwdArgsR {
  int ninst, n, H, A, ncq, nrb;
  FwdInst in[4];
  FwdHead hd;
  Stamps st;
  unsigned* sync;                    // fused F2 + B1: [nrb][2] counters (policy / target instances) + timeout
  unsigned* sync_reset; int n_sync;  // F1: block (0, 0, 0) zeroes the step's counters
};

// the head of row r, action j (8 lanes per row; every lane of the 8 calls both halves): the loads (issued
// before every other operand of the launch: the head is the first link of the launch's chain), then the
// pre-activation mean / raw log_std from the partials and head_fwd_elem's math; returns the action (tanh u)
struct HeadIn { float pm[MAX_NCQ], pl[MAX_NCQ], bm, bl, z; };

// the policy noise of row r, action j (mopo.py:306 tf.random_normal): Philox keyed by (seed, step, row,
// which head, action block) -- generated by F1 (it depends on nothing F1 computes), so F2's head only loads it
static __device__ __forceinline__ float head_noise(uint64_t seed, int64_t it, int r, int nxt, int j) {
  const int blk = j >> 2;
  u32x4 c{(uint32_t)r | ((uint32_t)nxt << 31), (uint32_t)it ^ ((uint32_t)blk << 24), (uint32_t)((uint64_t)it >> 32),
          RNG_SAC + 16};
  u32x4 q = philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  float z0, z1;
  if (j & 2) box_muller(q.z, q.w, z0, z1);
  else box_muller(q.x, q.y, z0, z1);
  return (j & 1) ? z1 : z0;
}

static __device__ __forceinline__ HeadIn rows_head_load(const FwdHead& h, int nxt, int n, int A, int ncq, int r,
                                                        int j, bool ok) {
  HeadIn o;
  const bool on = ok && j < A;
  const int ns = rows_ns(n);
  const auto dp = rsrc(h.opart[nxt], (int64_t)ncq * ns * OPW);
#pragma unroll
  for (int c = 0; c < MAX_NCQ; ++c) {     // unconditional loads (out-of-range ones return 0)
    o.pm[c] = bload(dp, (on && c < ncq) ? (c * ns + r) * OPW + j : -1);
    o.pl[c] = bload(dp, (on && c < ncq) ? (c * ns + r) * OPW + A + j : -1);
  }
  o.bm = bload(rsrc(h.bm, A), on ? j : -1);
  o.bl = bload(rsrc(h.bl, A), on ? j : -1);
  const float* ein = h.eps_in[nxt] ? h.eps_in[nxt] : h.eps_out[nxt];   // injected ([n][A]), or F1's draws ([n][EPW])
  const int lde = h.eps_in[nxt] ? A : EPW;
  o.z = bload(rsrc(ein, (int64_t)n * lde), on ? r * lde + j : -1);
  return o;
}

template <bool SC1>
static __device__ __forceinline__ float rows_head(const FwdHead& h, const HeadIn& in, int nxt, int A, int r, int j,
                                                  bool ok, bool store) {
  const bool on = ok && j < A;
  float v = 0.f, act = 0.f;
  if (on) {
    float mu = in.bm, raw = in.bl;
    const float z = in.z;
#pragma unroll
    for (int c = 0; c < MAX_NCQ; ++c) {   // the sums in column-block order
      mu += in.pm[c];
      raw += in.pl[c];
    }
    const float ls = fminf(fmaxf(raw, -20.f), 2.f);               // mopo.py:304
    const float sd = expf(ls);
    const float u = mu + z * sd;                                    // mopo.py:306
    const float zz = (u - mu) / (sd + 1e-8f);
    v = -0.5f * (zz * zz + 2.f * ls + 1.8378770664093453f)          // gaussian_likelihood (:282-284)
        - 2.f * (0.6931471805599453f - u - softplusf(-2.f * u));    // squash correction (:292)
    act = tanhf(u);
    if (store) {
      if (h.eps_in[nxt]) hstore<SC1>(&h.eps_out[nxt][r * EPW + j], z);   // (B1 reads the injected noise itself)
      hstore<SC1>(&h.head_out[nxt][r * 2 * A + j], mu);
      hstore<SC1>(&h.head_out[nxt][r * 2 * A + A + j], raw);
    }
  }
  v += __shfl_xor(v, 1);
  v += __shfl_xor(v, 2);
  v += __shfl_xor(v, 4);
  if (store && ok && j == 0) hstore<SC1>(&h.logp[nxt][lp_idx(r)], v);
  return act;
}

// The instance of a workgroup, selected field by field from the kernel arguments with the uniform
// blockIdx.z: a dynamically indexed argument array (a.in[blockIdx.z]) compiles to per-lane global loads
// of the argument block and waterfall loops around every buffer descriptor built from it.
template <typename T>
static __device__ __forceinline__ T pick4(const T (&in)[4], int i) {
  T p = in[0];
  if (i == 1) p = in[1];
  if (i == 2) p = in[2];
  if (i == 3) p = in[3];
  return p;
}

// LDS of the row-block kernels (floats).  The A slab is row-major with the contraction index fastest
// and a 4-float pad per row: lane (li, lk) of the 16x16x4 MFMA contributes k = 64 lk + 4 s + u at step
// (s, u) (any assignment of the K range to the four lane groups sums the same products), so one
// ds_read_b128 feeds four MFMAs, and the 16 lanes of each b128 read group hit distinct bank quads (row
// stride 260 = 65 quads: quad index li + s mod 16).  The B operand (the wave's own 16 weight columns)
// never touches LDS: each lane loads its 64 values for those k straight into registers, so the kernels
// need 26 KB of LDS and run two workgroups per CU.
constexpr int RB_LD = GKC + 4;            // the A slab [16 rows][K]
constexpr int RB_LDS_A = 16 * RB_LD;
constexpr int RB_TLD = RB_COLS + 4;       // the block's 16 x 64 output tile [row][c], the output-layer
constexpr int RB_LDS_T = 16 * RB_TLD;     //   columns [j][c] (j < 16) of the block's 64 rows

// the wave's 16 x 16 tile over the whole K: D(r, c) = sum_k A[r][k] B(k, c), with lane (li, lk) holding
// B(64 lk + 4 s + u, c = li) in b[s][u]
static __device__ __forceinline__ void rows_contract(const float* As, const f32x4 (&b)[16], int li, int lk,
                                                     f32x4 (&acc)[4]) {
#pragma unroll
  for (int u = 0; u < 4; ++u) acc[u] = zero4();
#pragma unroll
  for (int s = 0; s < GKC / 16; ++s) {
    const f32x4 a4 = ld4(As + li * RB_LD + 64 * lk + 4 * s);
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = mfma4(a4[u], b[s][u], acc[u]);
  }
}

// wave 0: partial output dots of the block's tile, Out[r][j] = sum_{c < COLS} T[r][c] WT[j][c] (COLS / 4
// MFMAs; row stride COLS + 4); rows r < n and j < nout are stored: a critic's (nout == 1) at qp_idx, the
// policy's to opart[cq][row][OPW] (row stride rows_ns(n))
template <int COLS, bool SC1>
static __device__ __forceinline__ void rows_partial_out(const float* T, const float* WT, int li, int lk, int i0, int n,
                                                        int nout, int cq, int ncq, float* opart) {
  constexpr int LD = COLS + 4;
  f32x4 acc[4] = {zero4(), zero4(), zero4(), zero4()};
#pragma unroll
  for (int s = 0; s < COLS / 16; ++s) {
    const f32x4 a4 = ld4(T + li * LD + (COLS / 4) * lk + 4 * s), b4 = ld4(WT + li * LD + (COLS / 4) * lk + 4 * s);
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = mfma4(a4[u], b4[u], acc[u]);
  }
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {                          // D: column li = output j, row 4 lk + rr
    const int orow = i0 + 4 * lk + rr;
    if (li < nout && orow < n) {
      const float v = acc[0][rr] + acc[1][rr] + acc[2][rr] + acc[3][rr];
      hstore<SC1>(opart + (nout == 1 ? qp_idx(cq, orow, ncq) : ((int64_t)cq * rows_ns(n) + orow) * OPW + li), v);
    }
  }
}

#ifndef MOPO_SAC_S7_PRE
#define MOPO_SAC_S7_PRE 0   // fused F2 (FZ >= 2): the step-7 operands before the wait on F1 (A/B knob)
#endif
#ifndef MOPO_SAC_S7_EARLY
// 1: issue step 7's operand loads right after the layer-2 MFMAs instead of in step 7 -- measured 45.4 vs
// 43.6 us/step (same-box A/B): they delay the epilogue's own loads and stores more than they hide
#define MOPO_SAC_S7_EARLY 0
#endif

// F2 (s, pi) critics: step 7's operands.  A(m = k, K = c): lane (li, lk) holds W2[64 w + 16 t + li][c0 +
// 16 s + 4 lk + u] (one b128 per (t, s)); B(K = k, n = a) of the action contraction: W1[O + a = li][64 w +
// 16 t + 4 lk .. + 3]
static __device__ __forceinline__ void step7_loads(const FwdInst& p, int w, int li, int lk, int c0, int H, int A,
                                                   f32x4 (&wa2)[4][4], f32x4 (&wb1)[4]) {
  const int kw = 64 * w;
  const auto dw2 = rsrc(p.w2, (int64_t)H * H);
  if (MOPO_SAC_LDOFF2 && (H & 63) == 0) {
    // whole 64-column blocks: every c < H, and rows k >= H fall past the range (H H): plain offsets
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int vb = ((kw + 16 * t + li) * H + c0 + 4 * lk) * 4;
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2)
        wa2[t][s2] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(dw2, vb + 64 * s2, 0, 0));
    }
  } else {
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) {
        const int k = kw + 16 * t + li, c = c0 + 16 * s2 + 4 * lk;
        wa2[t][s2] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                   dw2, ((k < H && c < H) ? k * H + c : -4) * 4, 0, 0));
      }
  }
  const auto dwa = rsrc(p.w1a, p.w1a ? (int64_t)A * H : 0);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int k = kw + 16 * t + 4 * lk;
    wb1[t] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                           dwa, ((p.w1a && li < A && k < H) ? li * H + k : -4) * 4, 0, 0));
  }
}

// LDS of one forward row-block workgroup (F1 / F2)
struct FwdLds {
  float As[RB_LDS_A];
  float Ts[RB_LDS_T];
  float Wo[RB_LDS_T];
  float act_s[16][8];
  float da_s[4][16][9];
};

// One forward row-block workgroup: column block cq, row block rb, instance ii (grid indices, SGPRs: the
// instance's fields then come from the kernel arguments by scalar loads -- a divided linear index made them
// VGPRs, and every buffer descriptor built from them needed a waterfall loop).  H <= GKC, H % 16 == 0.
// FZ, the fusion level: 0 a launch of its own; 1 F2 inside sac_f2b1_kernel (F2 + B1); 2 F1 or F2 inside
// sac_f12b1_kernel (F1 + F2 + B1).  A fused block's stores that a later phase of the launch reads are
// write-through, and the block ends by signalling its row block's counter; a fused F2 block (FZ = 2) issues
// its weight operands, then waits for its row block's pi blocks of F1 before loading the head's partials.
template <bool HEAD, int FZ>
static __device__ __forceinline__ void fwd_block(const FwdArgsR a, int cq, int rb, int ii, FwdLds& L) {
  constexpr bool SC = HEAD ? FZ >= 1 : FZ >= 2;   // this block's stores are handed over in-launch
  float* As = L.As;
  float* Ts = L.Ts;
  float* Wo = L.Wo;
  auto& act_s = L.act_s;
  auto& da_s = L.da_s;
  stamp(a.st, 0);
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const FwdInst p = pick4(a.in, ii);
  if (!HEAD && a.sync_reset && cq == 0 && rb == 0 && ii == 0 && tid < a.n_sync) a.sync_reset[tid * SYNC_STRIDE] = 0u;
  const int n = a.n, H = a.H, A = a.A;
  const int i0 = rb * 16, c0 = cq * RB_COLS, jw = c0 + w * 16;
  // ---- 0. F2: the head's operands first (the head is the first link of this launch's chain)
  const int hr = tid >> 3, hj = tid & 7, hrow = i0 + hr;
  HeadIn hin{};
  if (HEAD && FZ < 2 && tid < 128) hin = rows_head_load(a.hd, p.head, n, A, a.ncq, hrow, hj, hrow < n);
  // ---- 1. every global operand, issued up front in the order the chain consumes them: layer 1 (its
  //         MFMAs then run while the layer-2 operand is still arriving -- loads return in order, so
  //         layer-1 operands queued behind it waited for all of it), this wave's W2 operand straight into
  //         MFMA registers (lane (li, lk): W2[64 lk + 4 s + u][jw + li]; 16 lanes read 64 contiguous bytes
  //         of a row), the output-layer columns of the block's 64 rows
  const int li = lane & 15, lk = lane >> 4;
  const int r = lane & 15, q4 = lane >> 4;
  const int row = i0 + r;
  const int k1 = p.k1, ns = (k1 + 4) >> 2, sb = k1 >> 2;
  float xb[8], wa[4][8], bv[4];
  {
    const auto dx = rsrc(p.x, (int64_t)(n - 1) * p.ldx + p.kx);
    const auto dw = rsrc(p.w1, (int64_t)k1 * H);
    const auto db = rsrc(p.b1, H);
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int j = 4 * s + q4;
      const float v = bload(dx, (j < p.kx && row < n) ? row * p.ldx + j : -1);
      xb[s] = j == k1 ? 1.f : v;
    }
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      const int k = w * 64 + kt * 16 + r;
#if MOPO_SAC_LDOFF
      // W1 rows j >= k1 fall past the descriptor's range (k1 H) and read 0; a lane past H reads nothing
      const int vb = k < H ? (q4 * H + k) * 4 : (1 << 30);
#pragma unroll
      for (int s = 0; s < 8; ++s)
        wa[kt][s] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(dw, vb + 16 * s * H, 0, 0));
#else
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const int j = 4 * s + q4;
        wa[kt][s] = bload(dw, (j < k1 && k < H) ? j * H + k : -1);
      }
#endif
      bv[kt] = bload(db, k < H ? k : -1);
    }
  }
  f32x4 bp[16];
  {
    const auto dbw = rsrc(p.w2, (int64_t)H * H);
    const bool con = jw + li < H;
#if MOPO_SAC_LDOFF
    // plain offsets (one add per load): rows k >= H fall past the range (H H) and read 0
    const int vb = con ? (64 * lk * H + jw + li) * 4 : (1 << 30);
#pragma unroll
    for (int s2 = 0; s2 < 16; ++s2)
#pragma unroll
      for (int u = 0; u < 4; ++u)
        bp[s2][u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(dbw, vb + (4 * s2 + u) * H * 4, 0, 0));
#else
#pragma unroll
    for (int s2 = 0; s2 < 16; ++s2)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = 64 * lk + 4 * s2 + u;
        bp[s2][u] = bload(dbw, (con && k < H) ? k * H + jw + li : -1);
      }
#endif
  }
  float wov[4];
  {
    const int ld2 = p.nout - p.split;
    const auto d1 = rsrc(p.wo, (int64_t)H * p.split), d2 = rsrc(p.wo2, (int64_t)H * (ld2 > 0 ? ld2 : 1));
#pragma unroll
    for (int q = 0; q < 4; ++q) {           // element e = c * OPW + j of Wo: c = e / 16, j = e % 16
      const int e = tid + 256 * q, c = c0 + (e >> 4), j = e & 15;
      const bool in1 = j < p.split, on = c < H && j < p.nout;
      const float v1 = bload(d1, on && in1 ? c * p.split + j : -1);
      const float v2 = bload(d2, on && !in1 ? c * ld2 + (j - p.split) : -1);
      wov[q] = in1 ? v1 : v2;
    }
  }
  float b2v = bload(rsrc(p.b2, H), jw + (lane & 15) < H ? jw + (lane & 15) : -1);
  // ---- F1, pi(s) / pi(s') blocks of column block 0: this step's policy noise of their 16 rows (while the
  //      operands arrive), which F2's head loads
  if (!HEAD && ii < 2 && cq == 0 && ((a.hd.gen_eps >> ii) & 1) && tid < 128 && hj < A && hrow < n)
    hstore<SC>(&a.hd.eps_out[ii][hrow * EPW + hj], head_noise(a.hd.seed, *a.hd.iter, hrow, ii, hj));
  // ---- F2 inside the F1 + F2 + B1 launch: the head's partials once the row block's pi blocks are done (with
  //      MOPO_SAC_S7_PRE the main critics' step-7 operands are issued before the wait too: the block idles there)
  f32x4 wa2[4][4], wb1[4];
  constexpr bool S7PRE = HEAD && FZ >= 2 && MOPO_SAC_S7_PRE;
  if constexpr (S7PRE) {
    if (p.dapart) step7_loads(p, w, li, lk, c0, H, A, wa2, wb1);
  }
  if constexpr (HEAD && FZ >= 2) {
    stamp(a.st, 5);
    handoff_wait(sync_at(a.sync, rb, p.head == 0 ? SYNC_PI_S : SYNC_PI_N), (unsigned)a.ncq, a.sync + SYNC_N * a.nrb * SYNC_STRIDE);
    stamp(a.st, 6);
    if (tid < 128) hin = rows_head_load(a.hd, p.head, n, A, a.ncq, hrow, hj, hrow < n);
  }
  // ---- 2. F2: the policy head of the block's 16 rows (its action feeds layer 1)
  if (HEAD) {
    if (tid < 128) {
      const bool store = cq == 0 && (ii == 0 || ii == 2);  // Q1(s,pi) / Qt1(s',pi') blocks publish the head
      act_s[hr][hj] = rows_head<SC>(a.hd, hin, p.head, A, hrow, hj, hrow < n, store);
    }
    lds_barrier();
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int j = 4 * s + q4;
      if (j >= p.kx && j < k1) xb[s] = act_s[r][(j - p.kx) & 7];
    }
  }
  stamp(a.st, 1);
  // ---- 3. layer 1 on MFMA: D(k, r) = relu(W1^T X^T + b1) (the bias rides as input column k1)
#pragma unroll
  for (int kt = 0; kt < 4; ++kt)
#pragma unroll
    for (int s = 0; s < 8; ++s)
      if (s == sb && q4 == (k1 & 3)) wa[kt][s] = bv[kt];
  {
    f32x4 acc[4] = {zero4(), zero4(), zero4(), zero4()};
#pragma unroll
    for (int s = 0; s < 8; ++s)
      if (s < ns)
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) acc[kt] = mfma4(wa[kt][s], xb[s], acc[kt]);
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {  // rows r, k = w 64 + kt 16 + 4 q4 .. + 3: one b128 store
      const int kl = w * 64 + kt * 16 + 4 * q4;
      f32x4 v;
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) v[tt] = (row < n && kl + tt < H) ? fmaxf(acc[kt][tt], 0.f) : 0.f;
      *reinterpret_cast<f32x4*>(As + r * RB_LD + kl) = v;
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {     // Wo[j][c]: element e = c * 16 + j of the loads
    const int e = tid + 256 * q;
    Wo[(e & 15) * RB_TLD + (e >> 4)] = wov[q];
  }
  lds_barrier();
  stamp(a.st, 2);
  if (cq == 0 && p.h1 && tid < H) {  // the first-layer slab for the backward pass (coalesced in k)
#pragma unroll 4
    for (int rr = 0; rr < 16; ++rr)
      if (i0 + rr < n) hstore<SC>(&p.h1[(int64_t)(i0 + rr) * H + tid], As[rr * RB_LD + tid]);
  }
  // ---- 4. layer 2: the wave's 16 x 16 tile over the whole K
  f32x4 acc[4];
  rows_contract(As, bp, li, lk, acc);
#if MOPO_SAC_S7_EARLY
  if (HEAD && p.dapart) step7_loads(p, w, li, lk, c0, H, A, wa2, wb1);
#endif
  stamp(a.st, 3);
  // ---- 5. bias + relu (D: column li, rows 4 lk + rr); h2 store; the tile into LDS
  const int col = jw + li;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int orow = i0 + 4 * lk + rr;
    const float v = (col < H && orow < n) ? fmaxf(acc[0][rr] + acc[1][rr] + acc[2][rr] + acc[3][rr] + b2v, 0.f) : 0.f;
    if (p.h2 && orow < n && col < H) hstore<SC>(&p.h2[(int64_t)orow * H + col], v);
    Ts[(4 * lk + rr) * RB_TLD + w * 16 + li] = v;
  }
  lds_barrier();
  // ---- 6. partial output dots of the block's 64 columns (wave 0, MFMA)
  if (w == 0)                       // a critic's records are 1 float, row-block-major (qp_idx)
    rows_partial_out<RB_COLS, SC>(Ts, Wo, li, lk, i0, n, p.nout, cq, a.ncq, p.opart);
  // ---- 7. F2, Q1 / Q2 at (s, pi(s)): the critic's backward share of the block (dq = 1): wave w forms
  //         dh1 rows k in [64 w, 64 w + 64) of D(k, r) = sum_c W2[k][c0 + c] G(r, c), G = W3[c0 + c]
  //         (h2 > 0) (K = the block's 64 columns), masked by h1 > 0, then its partial of the action
  //         gradient sum_k dh1(r, k) W1[O + a][k], so the policy's backward needs no critic backward at
  //         (s, pi) in the next launch
  {
    if (HEAD && p.dapart) {
#if !MOPO_SAC_S7_EARLY
      if constexpr (!S7PRE) step7_loads(p, w, li, lk, c0, H, A, wa2, wb1);
#endif
      const int kw = 64 * w;
      // G(r = li, c = 16 s + 4 lk + u) from the block's h2 tile and W3 (Wo row 0)
      float gb[4][4];
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int c = 16 * s2 + 4 * lk + u;
          gb[s2][u] = Ts[li * RB_TLD + c] > 0.f ? Wo[c] : 0.f;
        }
      f32x4 da = zero4();
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        f32x4 d = zero4();                                   // D: k = kw + 16 t + 4 lk + i, r = li
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
          for (int u = 0; u < 4; ++u) d = mfma4(wa2[t][s2][u], gb[s2][u], d);
        f32x4 um;
#pragma unroll
        for (int i = 0; i < 4; ++i) {                        // * (h1 > 0); A(m = r = li, K = k)
          const int k = kw + 16 * t + 4 * lk + i;
          um[i] = (k < H && As[li * RB_LD + k] > 0.f) ? d[i] : 0.f;
          da = mfma4(um[i], wb1[t][i], da);
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)                            // D: r = 4 lk + i, a = li
        if (li < 8) da_s[w][4 * lk + i][li] = da[i];
      lds_barrier();
      if (tid < 128) {                                       // waves' partials in wave order
        const int rr = tid >> 3, aa = tid & 7, orow = i0 + rr;
        const float v = da_s[0][rr][aa] + da_s[1][rr][aa] + da_s[2][rr][aa] + da_s[3][rr][aa];
        if (aa < A && orow < n) hstore<SC>(&p.dapart[((int64_t)cq * rows_ns(n) + orow) * DPW + aa], v);
      }
    }
  }
  if constexpr (SC)
    handoff_signal(sync_at(a.sync, rb, HEAD ? (ii >= 2 ? SYNC_F2_TGT : SYNC_F2_MAIN) : (ii < 2 ? ii : SYNC_Q_SA)));
  stamp(a.st, 4);
}

// Grid (column block, row block, instance): linear block id cq + ncq (rb + nrb ii).
template <bool HEAD>
static __global__ __launch_bounds__(256, 2) void sac_fwd_kernel(const FwdArgsR a) {
  __shared__ __attribute__((aligned(16))) FwdLds L;
  fwd_block<HEAD, 0>(a, blockIdx.x, blockIdx.y, blockIdx.z, L);
}

// ---- B1 -----------------------------------------------------------------------------------------
// The critics' per-row losses from the forward partials (mopo.py:361-404): q = sum of the column-block
// partials + b3, in column-block order.  Instances of the partial arrays: 0 Q1(s,a) 1 Q2(s,a)
// 2 Q1(s,pi) 3 Q2(s,pi) 4 Qt1(s',pi') 5 Qt2(s',pi').
struct LossRows {
  const float* qpart[6];             // [ncq][n]
  const float* b3[6];
  const float* logp_s; const float* logp_n; const float* head_s; const float* rew; const float* term;
  const float* log_alpha;
  float gamma, rscale;
};

struct RowQ { float q[6]; float y, alpha; };

// The loads of row r's loss terms, all issued at once (out-of-range rows read 0), and the terms from them:
// q = sum of the column-block partials + b3, in column-block order.
struct RowIn { float pv[6][MAX_NCQ]; float b3[6]; float la, rew, term, logp_n; };

static __device__ __forceinline__ RowIn row_losses_load(const LossRows& L, int n, int ncq, int r, bool on) {
  RowIn o;
  const int ns = rows_ns(n);
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const auto dp = rsrc(L.qpart[i], (int64_t)ncq * ns);
#pragma unroll
    for (int c = 0; c < MAX_NCQ; ++c) o.pv[i][c] = bload(dp, (on && c < ncq) ? qp_idx(c, r, ncq) : -1);
    o.b3[i] = *L.b3[i];
  }
  o.la = *L.log_alpha;
  o.rew = bload(rsrc(L.rew, n), on ? r : -1);
  o.term = bload(rsrc(L.term, n), on ? r : -1);
  o.logp_n = bload(rsrc(L.logp_n, 2 * ns), on ? lp_idx(r) : -1);
  return o;
}

static __device__ __forceinline__ RowQ row_losses(const LossRows& L, const RowIn& in) {
  RowQ o;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    float s = in.b3[i];
#pragma unroll
    for (int c = 0; c < MAX_NCQ; ++c) s += in.pv[i][c];
    o.q[i] = s;
  }
  o.alpha = expf(in.la);                                              // mopo.py:361
  const float qt = fminf(o.q[4], o.q[5]);                             // mopo.py:368
  o.y = L.rscale * in.rew + L.gamma * ((1.f - in.term) * (qt - o.alpha * in.logp_n));  // :380-386
  return o;
}

struct Dh1Inst {
  const float* h1; const float* h2; const float* w2; const float* w3;
  int kind;                          // dq of the row: 0 (q1 - y) / n, 1 (q2 - y) / n
  float* dh1;
  float* dq;                         // stored by the column-block-0 workgroups
};

#ifndef MOPO_SAC_B1_WAVES
// 4: 16 rows x 64 columns per workgroup (twice the workgroups of the 8-wave form, half the W2 panel each):
// 41.4 vs 43.5 us/step (same-box A/B, profiles/r04_sac_ab.txt)
#define MOPO_SAC_B1_WAVES 4
#endif
constexpr int B1_WAVES = MOPO_SAC_B1_WAVES, B1_COLS = 16 * B1_WAVES;   // B1 workgroups: 16 rows x 16 B1_WAVES columns
constexpr int B1_TLD = B1_COLS + 4;

struct Dh1Args {
  int n, H, A;
  int ncq;                           // column blocks of the forward partials (64 wide)
  int ncq1;                          // B1's column blocks (128 wide)
  int nrb;
  Dh1Inst in[2];
  LossRows L;
  // step control (block 0): lr_t, beta powers, the target-update flag of this step
  float lr;
  float* beta_pow; const int64_t* iter;
  const int64_t* tctl;               // target schedule {base, n_train_repeat, interval} (sac.hip mopo_sac_set_target_schedule)
  PolicyRows pr;                     // the policy's row-local backward chain (blocks z = 3)
  int gather;                        // 1: the other z = 0 blocks gather the next step's batch (ga)
  GatherArgs ga;
  Stamps st;
  unsigned* sync;                    // fused launches: the row-block counters (sync_at) and the global words
};

// Block 0: the step's scalar control -- TF1 Adam's step size from the beta powers (every Adam of the step
// shares it: identical step counts), the beta powers of the next step, and whether this step's timestep
// moves the targets (mopo.py:780-799, 843-845: n_train_repeat steps share one timestep).  The step counter
// itself advances in the loss tail of the next launch (sac_wgrad.h), after every reader of this step's.
static __device__ __forceinline__ void step_control(const Dh1Args& a) {
  if (threadIdx.x != 0) return;
  const float b1p = a.beta_pow[0], b2p = a.beta_pow[1];
  const int64_t it = *a.iter, base = a.tctl[0];
  const int64_t rep = a.tctl[1] > 0 ? a.tctl[1] : 1, every = a.tctl[2] > 0 ? a.tctl[2] : 1;
  hstore<false>(&a.beta_pow[2], a.lr * sqrtf(1.f - b2p) / (1.f - b1p));   // TF1 Adam step size
  a.beta_pow[0] = b1p * 0.9f;
  a.beta_pow[1] = b2p * 0.999f;
  const int64_t ts = (it - base) / rep;
  hstore<false>(&a.beta_pow[3], ((ts % every) + every) % every == 0 ? 1.f : 0.f);
}

// LDS of one B1 workgroup
struct Dh1Lds {
  float As[RB_LDS_A];
  float Ts[16 * B1_TLD];
  float dqs[16];
};

// One B1 workgroup (grid indices x = column block, y = row block, z): z = 0: block (0, 0) the step control,
// the other blocks the gather of the next step's batch; z = 1, 2: Q1 / Q2(s, a) dh1 tiles; z = 3: the
// policy-row blocks.  FZ >= 1 (inside a fused launch): the z = 1..3 blocks issue the operands of earlier
// launches, then wait for their row block's F2 producers before loading what F2 wrote; FZ = 2 (F1 + F2 + B1)
// also waits for the row block's F1 blocks before loading F1's activations (h1, h2).
template <int FZ>
static __device__ __forceinline__ void dh1_block(const Dh1Args a, int x, int y, int z, Dh1Lds& S) {
  float* As = S.As;
  float* Ts = S.Ts;
  float* dqs = S.dqs;
  stamp(a.st, 0);
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (z == 0) {
    const int zb = x + a.ncq1 * y;
    if (zb == 0) {
      step_control(a);
    } else if (a.gather) {
      const GatherArgs& g = a.ga;
      const int C = 2 * g.O + g.A + 2, tot = g.n * C, stride = (a.ncq1 * a.nrb - 1) * (int)blockDim.x;
      for (int e = (zb - 1) * blockDim.x + tid; e < tot; e += stride) gather_elem(g, e / C, e % C);
    }
    stamp(a.st, 4);
    return;
  }
  if (z == 3) {                       // the policy-row blocks: the action-gradient partials came from F2
    policy_rows_block<FZ>(a.pr, y * a.ncq1 + x, As, Ts, a.st, a.sync, a.nrb);
    stamp(a.st, 4);
    return;
  }
  const int rb = y, cq = x;
  const Dh1Inst p = z == 1 ? a.in[0] : a.in[1];
  const int n = a.n, H = a.H;
  const int i0 = rb * 16, c0 = cq * B1_COLS, jw = c0 + w * 16;
  const int li = lane & 15, lk = lane >> 4;
  if constexpr (FZ >= 2 && B1_LATE)   // F1's Q(s, a) blocks of this row block first, then every operand
    handoff_wait(sync_at(a.sync, rb, SYNC_Q_SA), 2u * (unsigned)a.ncq, a.sync + SYNC_N * a.nrb * SYNC_STRIDE);
  // ---- 0. the dq of the block's 16 rows first (the partials of F1 / F2; one lane per row): the A slab
  //         below waits on it (fused: after the wait below)
  RowIn rin{};
  if (FZ == 0 && tid < 16) rin = row_losses_load(a.L, n, a.ncq, i0 + tid, i0 + tid < n);
  // ---- 1. operands in the order the chain consumes them: the A slab's h2 rows and W3, the h1 mask of this
  //         lane's outputs, then this wave's W2^T operand straight into MFMA registers (B(m, c) = W2[c][m]:
  //         lane (li, lk) holds W2[jw + li][64 lk + 4 s .. + 3])
  // A slab: thread (m-quad tid % 64, rows 4 (tid / 64) .. + 3), waves 0-3
  const bool slab = w < 4;
  const int am = 4 * (tid & 63), ar = 4 * (w & 3);
  const auto dh2 = rsrc(p.h2, (int64_t)n * H);
  f32x4 h2v[4];
  float m1[4];
  auto f1_loads = [&]() {             // F1's Q(s, a) activations: the slab's h2 rows, this lane's h1 mask
#pragma unroll
    for (int q = 0; q < 4; ++q)
      h2v[q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                             dh2, ((slab && am < H && i0 + ar + q < n) ? (i0 + ar + q) * H + am : -4) * 4, 0, 0));
    const auto dm1 = rsrc(p.h1, (int64_t)n * H);
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) m1[rr] = bload(dm1, (jw + li < H && i0 + 4 * lk + rr < n) ? (i0 + 4 * lk + rr) * H + jw + li : -1);
  };
  if constexpr (FZ < 2 || B1_LATE) f1_loads();
  const f32x4 w3v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                  rsrc(p.w3, H), ((slab && am < H) ? am : -4) * 4, 0, 0));
  const auto dw2 = rsrc(p.w2, (int64_t)H * H);
  f32x4 bp[16];
  if (MOPO_SAC_LDOFF2 && (H & 63) == 0) {
    // m < H exactly when 64 lk < H; c >= H: past the range
    const int vb = (64 * lk < H && jw + li < H) ? ((jw + li) * H + 64 * lk) * 4 : (1 << 30);
#pragma unroll
    for (int i = 0; i < 16; ++i)
      bp[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(dw2, vb + 16 * i, 0, 0));
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int m = 64 * lk + 4 * i, c = jw + li;
      bp[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                            dw2, ((m < H && c < H) ? c * H + m : -4) * 4, 0, 0));
    }
  }
  if constexpr (FZ >= 1) {            // the targets' partials and logp(s') come from this launch's F2 blocks
    unsigned* tmo = a.sync + SYNC_N * a.nrb * SYNC_STRIDE;
    stamp(a.st, 5);
    if constexpr (FZ >= 2 && !B1_LATE) {   // ... and the Q(s, a) activations from its F1 blocks
      handoff_wait(sync_at(a.sync, rb, SYNC_Q_SA), 2u * (unsigned)a.ncq, tmo);
      f1_loads();
    }
    handoff_wait(sync_at(a.sync, rb, SYNC_F2_TGT), 2u * (unsigned)a.ncq, tmo);
    stamp(a.st, 6);
    if (tid < 16) rin = row_losses_load(a.L, n, a.ncq, i0 + tid, i0 + tid < n);
  }
  // ---- 2. dq of the block's 16 rows (one lane per row)
  if (tid < 16) {
    float dq = 0.f;
    if (i0 + tid < n) {
      const RowQ rq = row_losses(a.L, rin);
      dq = ((p.kind == 0 ? rq.q[0] : rq.q[1]) - rq.y) * (1.f / (float)n);
      if (cq == 0) hstore<false>(&p.dq[i0 + tid], dq);
    }
    dqs[tid] = dq;
  }
  lds_barrier();
  stamp(a.st, 1);
  // ---- 3. A slab dh2 = dq (x) W3 * (h2 > 0) into LDS (b128 stores; waves 0-3)
  if (slab) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float u = dqs[ar + q];
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = (am + e < H && h2v[q][e] > 0.f) ? u * w3v[e] : 0.f;
      *reinterpret_cast<f32x4*>(As + (ar + q) * RB_LD + am) = v;
    }
  }
  lds_barrier();
  stamp(a.st, 2);
  // ---- 4. dh1 tile of the wave: 16 rows x 16 columns over the whole K
  f32x4 acc[4];
  rows_contract(As, bp, li, lk, acc);
  stamp(a.st, 3);
  // ---- 5. relu mask from h1; store
  const int col = jw + li;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int orow = i0 + 4 * lk + rr;
    const float v = (col < H && orow < n && m1[rr] > 0.f) ? acc[0][rr] + acc[1][rr] + acc[2][rr] + acc[3][rr] : 0.f;
    if (orow < n && col < H) hstore<false>(&p.dh1[(int64_t)orow * H + col], v);
  }
  stamp(a.st, 4);
}

// B1 as its own launch: grid (ncq1, nrb, 4), B1_WAVES-wave workgroups
static __global__ __launch_bounds__(B1_WAVES * 64, 1) void sac_dh1_kernel(const Dh1Args a) {
  __shared__ __attribute__((aligned(16))) Dh1Lds S;
  dh1_block<0>(a, blockIdx.x, blockIdx.y, blockIdx.z, S);
}

// F2 and B1 as ONE launch, grid (ncq, nrb, 8): z < 4 the F2 blocks (instance z), z >= 4 the B1 blocks (B1's
// z - 4).  Blocks are dispatched in linear-id order (z-major), so every F2 block is resident or done before a
// B1 block starts, and a B1 block only waits on F2 blocks: no wait can block a producer.  What it buys: B1's
// operands from earlier launches (weights, F1's activations) arrive while F2 runs, and the F2 -> B1 seam is a
// per-row-block hand-off instead of a grid-wide boundary.  Requires ncq1 == ncq (B1_COLS == RB_COLS).
union F2B1Lds {
  FwdLds f;
  Dh1Lds b;
};
static __global__ __launch_bounds__(256, 2) void sac_f2b1_kernel(const FwdArgsR f, const Dh1Args b) {
  __shared__ __attribute__((aligned(16))) F2B1Lds S;
  if (blockIdx.z < 4)
    fwd_block<true, 1>(f, blockIdx.x, blockIdx.y, blockIdx.z, S.f);
  else
    dh1_block<1>(b, blockIdx.x, blockIdx.y, blockIdx.z - 4, S.b);
}

// F1, F2 and B1 as ONE launch, grid (ncq, nrb, 12): z < 4 F1 (instance z), 4 <= z < 8 F2 (instance z - 4),
// z >= 8 B1 (B1's z - 8).  Dispatch in linear-id order again means a block only ever waits on producers with
// lower ids: F2 on its row block's pi blocks of F1, B1 on its row block's F1 and F2 blocks.  Besides B1's, the
// F2 blocks' weight operands now arrive while F1 runs.  The counters are zeroed by the previous step's
// weight-gradient launch (sac_wgrad.h) and at creation.
static __global__ __launch_bounds__(256, 2) void sac_f12b1_kernel(const FwdArgsR f1, const FwdArgsR f2, const Dh1Args b) {
  __shared__ __attribute__((aligned(16))) F2B1Lds S;
  if (blockIdx.z < 4)
    fwd_block<false, 2>(f1, blockIdx.x, blockIdx.y, blockIdx.z, S.f);
  else if (blockIdx.z < 8)
    fwd_block<true, 2>(f2, blockIdx.x, blockIdx.y, blockIdx.z - 4, S.f);
  else
    dh1_block<2>(b, blockIdx.x, blockIdx.y, blockIdx.z - 8, S.b);
}

}  // namespace mopo
