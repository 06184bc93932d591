// Grouped small-GEMM kernel with fused epilogues (activation, activation-derivative masks,
// bias-gradient column sums, TF1 Adam), used by the ensemble training step (bnn_train.hip); the
// Adam context, the range-checked buffer loads and the stamps are shared with the SAC step (sac.hip).
//
// One 16x16 output tile per 256-thread block; K is split over the four waves and reduced through
// LDS.  f32 MFMA (v_mfma_f32_16x16x4_f32).  The shapes these updates see are small (batch 256,
// width 200-256), so the kernel is built for latency: many independent tiles of up to MAXP
// problems per launch, every operand load unconditional (range-checked buffer loads), panels
// staged through an XOR-swizzled LDS layout.  Everything here has internal linkage: each
// translation unit that includes it gets its own copy of the kernel.
#pragma once
#include <type_traits>
#include <cstdlib>
#include <vector>

#include "internal.h"

namespace mopo {

// swish'(z) = s + z s (1 - s), s = sigmoid(z) (TF: the product rule through tf.sigmoid, fc.py:21)
static __device__ __forceinline__ float dswish_fast(float z) {
  const float s = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-z * 1.4426950408889634f));
  return s + z * s * (1.0f - s);
}

constexpr int MAXP = 16;

#ifndef MOPO_SAC_STAMPS
#define MOPO_SAC_STAMPS 0    // 1: diagnostic build, per-workgroup phase timestamps (s_memrealtime)
#endif

// per-workgroup phase stamps of the diagnostic build: [launch slot][block][8] u64
struct Stamps { uint64_t* p; int slot; };
static __device__ __forceinline__ void stamp(const Stamps& s, int i) {
#if MOPO_SAC_STAMPS
  // wave 0 (a wave-uniform branch: a lane-divergent one here moved the workgroup ids into VGPRs and
  // de-uniformised the whole kernel); its lanes all store the same value
  if (s.p && __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 0) {
    uint64_t t = __builtin_amdgcn_s_memrealtime();
    const int b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    uint64_t* q = s.p + ((int64_t)s.slot * 1024 + b) * 8;
    __hip_atomic_store(q + i, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#else
  (void)s; (void)i;
#endif
}


enum { ACT_NONE = 0, ACT_RELU = 1, ACT_SWISH = 2 };   // GemmProb::act
enum { MASK_RELU = 0, MASK_DSWISH = 1 };             // GemmProb::mask_kind

struct GemmProb {
  int M, N, K;
  const float* A; int lda; int ta;   // ta=0: A(i,k)=A[i*lda+k]; ta=1: A(i,k)=A[k*lda+i]
  const float* B; int ldb; int tb;   // tb=0: B(k,j)=B[k*ldb+j]; tb=1: B(k,j)=B[j*ldb+k]
  float* C; int ldc;
  const float* bias;                 // C += bias[j]
  int act;                           // ACT_RELU: C = max(C, 0); ACT_SWISH: C = swish(C), Z = pre-activation
  float* Z;                          //   (ACT_SWISH, optional; same layout as C)
  const float* mask; int ldm;        // MASK_RELU: C *= (mask(i,j) > 0) (relu' from the saved activation)
  int mask_kind;                     // MASK_DSWISH: C *= swish'(mask(i,j)) (mask = saved pre-activation)
  float wd;                          // adam: gradient += wd * param (TF l2_loss weight decay, fc.py:156-157)
  float* colsum;                     // colsum[j] = sum_k B(k,j)   (bias gradient), by tile-row 0
  // rank-1 masked operands (the critic's 1-wide output layer backward, fused into its consumer):
  // when a_u != NULL:  A(i,k) = a_u[i] * a_v[k] * (a_m[i*a_ldm + k] > 0);  same for B with (k, j)
  const float* a_u; const float* a_v; const float* a_m; int a_ldm;
  const float* b_u; const float* b_v; const float* b_m; int b_ldm;
  int adam;                          // C (and colsum) are gradient slices of AdamCtx::G: apply Adam
  int nb;                            // > 1: nb independent problems of these dims with dense-packed operands
                                     //   (batch b: A + b (ta ? K : M) lda, B + b (tb ? N : K) ldb, C + b M ldc,
                                     //   colsum + b N); no bias / Z / mask / rank-1 / two-segment operands
  // two-segment plain B (operand mode 3): columns [0, split) from B, [split, N) from B2 (same ldb),
  // bias likewise from bias / bias2
  const float* B2; int split; const float* bias2;
};

// Fused optimizer (the four TF1 Adams + Polyak, mopo.py:407-447): a weight-gradient tile is final
// when its epilogue runs (K spans the whole batch), so the epilogue updates the parameters it
// covers right there.  Parameters are double-buffered (read Pc, write Pn) because the same launch
// and later backward launches still read the pre-step weights; M, V and T are updated in place
// (each element is touched by exactly one tile, and T is only read by earlier forward stages).
struct AdamCtx {
  const float* G; const float* Pc; float* Pn; float* M; float* V; float* T;
  const float* lr_t;                 // this step's step size (sac_loss_kernel)
  float tau; int64_t total, n_pi, n_q; // grad-norm logs: [0, n_pi) policy, [n_pi, n_pi + n_q) Q1
  float* norm_part;                  // [slot][2] squared-gradient partials (pi, q) per block
  int slot0;                         // this launch's first slot
  const float* tgt_on;               // SAC: this step's target-update flag (mopo.py:843-845; NULL: every step)
};

// SAC log slots (sac.hip, mopo_sac_buffers)
enum {
  LOG_Q1_LOSS = 0, LOG_Q2_LOSS, LOG_Q1, LOG_Q2, LOG_ALPHA, LOG_ENTROPY, LOG_LOGP, LOG_PI_GNORM, LOG_Q_GNORM,
  LOG_PI_LOSS, LOG_PI_GSQ, LOG_Q_GSQ,
  LOG_N = 16
};

// buffer descriptor over n floats at p (wave-uniform inputs only)
static __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* p, int64_t n) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), 0, (int)(n * 4), 0x00020000);
}

static __device__ __forceinline__ float bload(__amdgpu_buffer_rsrc_t d, int idx) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(d, idx * 4, 0, 0));
}

struct GemmGroup {
  int n;
  int prefix[MAXP + 1];
  AdamCtx ad;
  Stamps st;                         // diagnostic builds (MOPO_SAC_STAMPS): per-block phase stamps
  GemmProb p[MAXP];
};

struct AdamIn { float p, m, v, t; };

static __device__ __forceinline__ AdamIn adam_load(const AdamCtx& ad, int64_t i) {
  return AdamIn{ad.Pc[i], ad.M[i], ad.V[i], ad.T ? ad.T[i] : 0.f};
}

// TF1 Adam (m += (g - m)(1 - b1), v += (g^2 - v)(1 - b2), p -= lr_t m / (sqrt(v) + eps)) + Polyak.
// Returns the new parameter; *t_new (when given) the new target, or the old one where it did not move.
// hold: the step's operands are not trusted (a fused SAC launch gave up waiting on a hand-off, sac_rows.h
// handoff_wait): the parameter carries over unchanged into the other ping-pong copy, the moments and the target
// stay, so a give-up never applies an update computed from stale data.
static __device__ __forceinline__ float adam_apply(const AdamCtx& ad, int64_t i, float g, AdamIn a, float lr_t,
                                                   float* t_new = nullptr, bool hold = false) {
  if (hold) {
    ad.Pn[i] = a.p;
    if (t_new) *t_new = a.t;
    return a.p;
  }
  const float m = a.m + (g - a.m) * (1.f - 0.9f);
  const float v = a.v + (g * g - a.v) * (1.f - 0.999f);
  const float p = a.p - (m * lr_t) / (sqrtf(v) + 1e-8f);
  ad.M[i] = m;
  ad.V[i] = v;
  ad.Pn[i] = p;
  float t = a.t;
  // mopo.py:446-447 (after the updates), on the steps whose timestep % target_update_interval == 0 (:843-845)
  if (ad.T && i < ad.total && (!ad.tgt_on || *ad.tgt_on != 0.f)) {
    t = (1.f - ad.tau) * a.t + ad.tau * p;
    ad.T[i] = t;
  }
  if (t_new) *t_new = t;
  return p;
}


constexpr int GKC = 256;  // K chunk staged in LDS

// One 16-wide panel (A: rows i0..i0+15, or B: cols j0..j0+15) x K-chunk, staged as S[k][r].
// MODE 0: plain, 1: transposed, 2: rank-1 masked (see GemmProb).  Loads are raw buffer loads through
// a descriptor sized to the operand's extent: a 32-bit byte offset per element (no 64-bit address
// pairs) and hardware range checking (reads past the extent return 0), so every load is issued
// unconditionally; elements outside the tile or the K chunk are zeroed by a select at the store.
struct PanelRegs { float x[16], u[16], w[16]; };

// Panels are S[k][r ^ psw(k)]: 64 4-byte banks, a 16-float row puts k and k+4 on the same banks, so
// without the XOR the k-fast stores (64 consecutive k per wave) hit 4 banks 16 ways.  With it the
// k-fast and r-fast stores and the MFMA operand reads (16 r x 4 k per instruction) are conflict-free.
// 32-wide panels (gemm32 kernel, 128-deep chunks) use S[k][r ^ ((k >> 1) & 31)]: a 32-float row puts
// k and k+2 on the same banks; the XOR spreads 64 consecutive k (k-fast stores) over all 64 banks and
// keeps the r-fast stores (32 r x 2 k) and the MFMA operand reads (16 r x 4 k) conflict-free.
template <int TW>
static __device__ __forceinline__ int pswz(int k) { return TW == 16 ? ((k >> 2) & 15) : ((k >> 1) & 31); }
static __device__ __forceinline__ int psw(int k) { return pswz<16>(k); }

// element q (0..15) of this thread's share of a TW-wide panel chunk (TW = 16: 256 deep; 32: 128)
template <int MODE, bool IS_A, int TW = 16>
static __device__ __forceinline__ void panel_rk(int q, int tid, int& r, int& k) {
  constexpr bool rfast = IS_A ? (MODE == 1) : (MODE != 1);
  if (TW == 16) {
    if (rfast) { r = tid & 15; k = (tid >> 4) + 16 * q; }
    else { k = (tid & 63) + 64 * (q & 3); r = (tid >> 6) + 4 * (q >> 2); }
  } else {
    if (rfast) { r = tid & 31; k = (tid >> 5) + 8 * q; }
    else { k = (tid & 63) + 64 * (q & 1); r = (tid >> 6) + 4 * (q >> 1); }
  }
}

template <int MODE, bool IS_A, int TW = 16>
static __device__ __forceinline__ void load_panel(const GemmProb& p, int r0, int kc, int tid, PanelRegs& R,
                                                  int64_t off = 0) {
  constexpr int KPER = TW == 16 ? 4 : 2;  // k-fast panel: consecutive q share a row in runs of KPER
  const int Rn = IS_A ? p.M : p.N;  // panel axis extent
  if (MODE == 2) {
    const int ldm = IS_A ? p.a_ldm : p.b_ldm;
    // A(i,k) = u[i] v[k] (m[i,k] > 0);  B(k,j) = u[k] v[j] (m[k,j] > 0).  The A panel is k-fast
    // (q / KPER picks the row, q % KPER the k run), so it needs 16/KPER u and KPER v values per
    // thread; the B panel is r-fast (one column per thread, 16 k): 16 u, 1 v.
    const auto dm = IS_A ? rsrc(p.a_m, (int64_t)(Rn - 1) * ldm + p.K) : rsrc(p.b_m, (int64_t)(p.K - 1) * ldm + Rn);
    const auto du = IS_A ? rsrc(p.a_u, Rn) : rsrc(p.b_u, p.K);
    const auto dv = IS_A ? rsrc(p.a_v, p.K) : rsrc(p.b_v, Rn);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      int r, k;
      panel_rk<MODE, IS_A, TW>(q, tid, r, k);
      const int gr = r0 + r, gk = kc + k;
      if (IS_A) {
        if ((q % KPER) == 0) R.u[q / KPER] = bload(du, gr);
        if (q < KPER) R.w[q] = bload(dv, gk);
      } else {
        R.u[q] = bload(du, gk);
        if (q == 0) R.w[0] = bload(dv, gr);
      }
      R.x[q] = bload(dm, IS_A ? gr * ldm + gk : gk * ldm + gr);
    }
  } else if (MODE == 3) {
    // two-segment B: per-lane segment select, so flat loads with clamped addresses
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      int r, k;
      panel_rk<MODE, IS_A, TW>(q, tid, r, k);
      const int gr = min(r0 + r, Rn - 1), gk = min(kc + k, p.K - 1);
      const float* src = gr < p.split ? p.B + gr : p.B2 + (gr - p.split);
      R.x[q] = src[(int64_t)gk * p.ldb];
    }
  } else {
    const float* base = (IS_A ? p.A : p.B) + off;   // off: a batched problem's batch (plain modes only)
    const int ld = IS_A ? p.lda : p.ldb;
    // element (r, k) of the panel's operand lives at r*ld + k (row-major in r) or k*ld + r
    constexpr bool r_major = IS_A ? (MODE == 0) : (MODE == 1);
    const auto d = r_major ? rsrc(base, (int64_t)(Rn - 1) * ld + p.K) : rsrc(base, (int64_t)(p.K - 1) * ld + Rn);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      int r, k;
      panel_rk<MODE, IS_A, TW>(q, tid, r, k);
      const int gr = r0 + r, gk = kc + k;
      R.x[q] = bload(d, r_major ? gr * ld + gk : gk * ld + gr);
    }
  }
}

// keep the loads batched ahead of the first use
template <int MODE, bool IS_A, int TW = 16>
static __device__ __forceinline__ void pin_panel(PanelRegs& R) {
  constexpr int KPER = TW == 16 ? 4 : 2;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    asm volatile("" : "+v"(R.x[q]));
    if (MODE == 2 && (IS_A ? q < 16 / KPER : true)) asm volatile("" : "+v"(R.u[q]));
    if (MODE == 2 && (IS_A ? q < KPER : q == 0)) asm volatile("" : "+v"(R.w[q]));
  }
}

// element q of a rank-1 panel: u * v (the A panel indexes u by q / KPER and v by q % KPER)
template <bool IS_A, int TW = 16>
static __device__ __forceinline__ float rank1_uv(const PanelRegs& R, int q) {
  constexpr int KPER = TW == 16 ? 4 : 2;
  return IS_A ? R.u[q / KPER] * R.w[q % KPER] : R.u[q] * R.w[0];
}

// S: [chunk depth][TW] floats
template <int MODE, bool IS_A, int TW = 16>
static __device__ __forceinline__ void store_panel(const GemmProb& p, int r0, int kn, int tid, const PanelRegs& R,
                                                   float* S) {
  const int Rmax = IS_A ? p.M : p.N;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    int r, k;
    panel_rk<MODE, IS_A, TW>(q, tid, r, k);
    const float v = MODE == 2 ? (R.x[q] > 0.f ? rank1_uv<IS_A, TW>(R, q) : 0.f) : R.x[q];
    S[k * TW + (r ^ pswz<TW>(k))] = (r0 + r < Rmax && k < kn) ? v : 0.f;
  }
}

// operand modes (A: 0 plain, 1 transposed, 2 rank-1; B: the same, 3 two-segment) as am * 4 + bm
__host__ static __device__ __forceinline__ int operand_modes(const GemmProb& p) {
  const int am = p.a_u ? 2 : p.ta, bm = p.b_u ? 2 : p.B2 ? 3 : p.tb;
  return am * 4 + bm;
}

template <int AM, int BM, int TW = 16>
static __device__ __forceinline__ void stage_ab(const GemmProb& p, int i0, int j0, int kc, int kn, int tid, float* As,
                                                float* Bs, int64_t oA = 0, int64_t oB = 0) {
  PanelRegs ra, rb;
  load_panel<AM, true, TW>(p, i0, kc, tid, ra, oA);
  load_panel<BM, false, TW>(p, j0, kc, tid, rb, oB);
  pin_panel<AM, true, TW>(ra);
  pin_panel<BM, false, TW>(rb);
  store_panel<AM, true, TW>(p, i0, kn, tid, ra, As);
  store_panel<BM, false, TW>(p, j0, kn, tid, rb, Bs);
}

template <int TW>
static __device__ __forceinline__ void stage_dispatch(const GemmProb& p, int i0, int j0, int kc, int kn, int t,
                                                      float* As, float* Bs, int64_t oA = 0, int64_t oB = 0) {
  switch (operand_modes(p)) {  // the combinations the callers use (launch_group rejects others)
    case 0: stage_ab<0, 0, TW>(p, i0, j0, kc, kn, t, As, Bs, oA, oB); break;
    case 1: stage_ab<0, 1, TW>(p, i0, j0, kc, kn, t, As, Bs, oA, oB); break;
    case 3: stage_ab<0, 3, TW>(p, i0, j0, kc, kn, t, As, Bs); break;
    case 4: stage_ab<1, 0, TW>(p, i0, j0, kc, kn, t, As, Bs, oA, oB); break;
    case 6: stage_ab<1, 2, TW>(p, i0, j0, kc, kn, t, As, Bs); break;
    default: stage_ab<2, 1, TW>(p, i0, j0, kc, kn, t, As, Bs); break;
  }
}

// One 16x16 output tile per 256-thread block.  The A[16 x K] and B[K x 16] panels are staged in
// LDS with loads ordered along each operand's contiguous axis (all issued before the first use:
// one memory latency per chunk), then the four waves split K and run v_mfma_f32_16x16x4_f32 out
// of LDS; partial tiles are summed through LDS and the epilogue fuses bias / activation / the
// activation-derivative mask, and (for weight gradients) the optimizer.
#ifndef MOPO_GEMM_KERNELS
#define MOPO_GEMM_KERNELS 1   // 0: a translation unit that uses only the shared helpers (sac.hip)
#endif
#if MOPO_GEMM_KERNELS
static __global__ __launch_bounds__(256, 4) void gemm_group_kernel(const GemmGroup g) {
  __shared__ __attribute__((aligned(16))) float ABs[2 * GKC * 16];  // the A and B panels
  float (*As)[16] = reinterpret_cast<float (*)[16]>(ABs);
  float (*Bs)[16] = reinterpret_cast<float (*)[16]>(ABs + GKC * 16);
  __shared__ __attribute__((aligned(16))) float part[4][256];
  __shared__ float csum[16][17];
  stamp(g.st, 0);
  const int bid = (int)blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int pi = 0;
  while (pi + 1 < g.n && bid >= g.prefix[pi + 1]) ++pi;
  const GemmProb& p = g.p[pi];
  int t = bid - g.prefix[pi];
  const int tn_cnt = ceil_div(p.N, 16);
  int first = g.prefix[pi];   // block id of this (batch's) tile 0
  // batched problem: batch b's operands are dense-packed at these offsets (floats)
  int64_t oA = 0, oB = 0, oC = 0, oCs = 0;
  if (p.nb > 1) {
    const int per = ceil_div(p.M, 16) * tn_cnt, b = t / per;
    t -= b * per;
    first += b * per;
    oA = (int64_t)b * (p.ta ? p.K : p.M) * p.lda;
    oB = (int64_t)b * (p.tb ? p.N : p.K) * p.ldb;
    oC = (int64_t)b * p.M * p.ldc;
    oCs = (int64_t)b * p.N;
  }
  float* const pC = p.C + oC;
  float* const pcs = p.colsum ? p.colsum + oCs : nullptr;
#ifndef MOPO_GEMM_XCD
#define MOPO_GEMM_XCD 1
#endif
  // XCD-aware tile order: workgroups are dealt round-robin over the 8 XCDs (block b on XCD b mod 8),
  // so when a problem's first block sits on XCD 0 and its column-tile count divides by 8, XCD x takes
  // column tiles [x C/8, (x+1) C/8) of every row tile: each B panel (the weight columns of an MLP
  // layer) is fetched into one XCD's L2 instead of all eight.
  int tm, tn;
  if (MOPO_GEMM_XCD && (tn_cnt & 7) == 0 && (first & 7) == 0) {
    const int per = tn_cnt >> 3, x = t & 7, j = t >> 3;
    tn = x * per + j % per;
    tm = j / per;
  } else {
    tm = t / tn_cnt;
    tn = t % tn_cnt;
  }
  const int i0 = tm * 16, j0 = tn * 16;
  const int li = lane & 15, lk = lane >> 4;
  const bool do_cs = p.colsum && tm == 0;
  // epilogue operands are fetched up front so their latency overlaps the panel loads
  const int ei = tid >> 4, ej = tid & 15;
  const int gi = i0 + ei, gj = j0 + ej;
  const int gic = min(gi, p.M - 1), gjc = min(gj, p.N - 1);
  float e_bias = p.bias ? (p.bias2 && gjc >= p.split ? p.bias2[gjc - p.split] : p.bias[gjc]) : 0.f;
  float e_mask = p.mask ? p.mask[(int64_t)gic * p.ldm + gjc] : 1.f;
  asm volatile("" : "+v"(e_bias), "+v"(e_mask));
  const AdamCtx& ad = g.ad;
  const int64_t a_idx = p.adam ? (int64_t)(pC - ad.G) + (int64_t)gic * p.ldc + gjc : 0;
  const int64_t c_idx = p.adam && p.colsum ? (int64_t)(pcs - ad.G) + min(j0 + (tid & 15), p.N - 1) : 0;
  AdamIn a_in{0.f, 0.f, 0.f, 0.f}, c_in{0.f, 0.f, 0.f, 0.f};
  float lr_t = 0.f;
  if (p.adam) {
    a_in = adam_load(ad, a_idx);
    if (p.colsum && tm == 0 && tid < 16) c_in = adam_load(ad, c_idx);
    lr_t = *ad.lr_t;
    asm volatile("" : "+v"(a_in.p), "+v"(a_in.m), "+v"(a_in.v), "+v"(a_in.t));
  }
  f32x4 acc0 = zero4(), acc1 = zero4();
  float cs = 0.f;
  for (int kc = 0; kc < p.K; kc += GKC) {
    const int kn = min(GKC, p.K - kc);
    // re-derive the thread index inside the chunk loop: otherwise the ~100 per-thread LDS and
    // buffer offsets are hoisted out of it and stay live across the loop (VGPRs -> occupancy)
    int t = tid;
    asm volatile("" : "+v"(t));
    // 16 elements of each panel per thread; the per-operand mode is dispatched once (uniform
    // branch) so that all 32+ loads are unconditional and issue back to back -- one memory latency
    // per chunk instead of one per element.
    stage_dispatch<16>(p, i0, j0, kc, kn, t, &As[0][0], &Bs[0][0], oA, oB);
    lds_barrier();
    stamp(g.st, 1);
    // the staged panels are zero-padded to GKC rows, so every wave runs exactly 16 k-steps of its
    // quarter with no guards: all 32 LDS reads first, then 16 MFMAs on two accumulators
    float ra[16], rb[16];
    const int tli = t & 15, tlk = (t >> 4) & 3, tw = t >> 6;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int k = 4 * (tw * 16 + s) + tlk;
      ra[s] = As[k][tli ^ psw(k)];
      rb[s] = Bs[k][tli ^ psw(k)];
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s & 1) acc1 = mfma4(ra[s], rb[s], acc1);
      else acc0 = mfma4(ra[s], rb[s], acc0);
    }
    if (do_cs)
      for (int k = tid >> 4; k < kn; k += 16) cs += Bs[k][(tid & 15) ^ psw(k)];
    lds_barrier();
  }
  stamp(g.st, 2);
#pragma unroll
  for (int r = 0; r < 4; ++r) part[w][(lk * 4 + r) * 16 + li] = acc0[r] + acc1[r];  // D: col li, row 4*lk+r
  if (do_cs) csum[tid >> 4][tid & 15] = cs;
  lds_barrier();
  float gsq = 0.f;
  {
    float v = part[0][tid] + part[1][tid] + part[2][tid] + part[3][tid];
    if (gi < p.M && gj < p.N) {
      v += e_bias;
      if (p.act == ACT_RELU) {
        v = fmaxf(v, 0.f);
      } else if (p.act == ACT_SWISH) {
        if (p.Z) p.Z[(int64_t)gi * p.ldc + gj] = v;
        v = swish_fast(v);
      }
      if (p.mask_kind == MASK_DSWISH) v *= dswish_fast(e_mask);
      else if (!(e_mask > 0.f)) v = 0.f;
      if (p.adam) v += p.wd * a_in.p;
      pC[(int64_t)gi * p.ldc + gj] = v;
      if (p.adam) {
        adam_apply(ad, a_idx, v, a_in, lr_t);
        gsq = v * v;
      }
    }
  }
  if (do_cs && tid < 16) {
    float c = 0.f;
    for (int q = 0; q < 16; ++q) c += csum[q][tid];
    if (j0 + tid < p.N) {
      pcs[j0 + tid] = c;
      if (p.adam) {
        adam_apply(ad, c_idx, c, c_in, lr_t);
        gsq += c * c;
      }
    }
  }
  if (ad.norm_part) {  // per-block squared-gradient partial (grad-norm logs; summed by sac_logs_kernel)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) gsq += __shfl_xor(gsq, off);
    lds_barrier();
    if (lane == 0) part[0][w] = gsq;
    lds_barrier();
    if (tid == 0) {
      const float b = part[0][0] + part[0][1] + part[0][2] + part[0][3];
      const int64_t off = p.adam ? (int64_t)(pC - ad.G) : -1;
      float* np = ad.norm_part + 2 * (int64_t)(ad.slot0 + bid);
      np[0] = off >= 0 && off < ad.n_pi ? b : 0.f;
      np[1] = off >= ad.n_pi && off < ad.n_pi + ad.n_q ? b : 0.f;
    }
  }
  stamp(g.st, 4);
}


// ---- epilogue helpers (gemm32_group_kernel) ---------------------------------------------------
struct EpiPre { float bias, mask; AdamIn a; int64_t a_idx; };

static __device__ __forceinline__ EpiPre epi_prefetch(const GemmProb& p, float* C, const AdamCtx& ad, int gi, int gj) {
  const int gic = min(gi, p.M - 1), gjc = min(gj, p.N - 1);
  EpiPre e;
  e.bias = p.bias ? (p.bias2 && gjc >= p.split ? p.bias2[gjc - p.split] : p.bias[gjc]) : 0.f;
  e.mask = p.mask ? p.mask[(int64_t)gic * p.ldm + gjc] : 1.f;
  e.a_idx = p.adam ? (int64_t)(C - ad.G) + (int64_t)gic * p.ldc + gjc : 0;
  e.a = AdamIn{0.f, 0.f, 0.f, 0.f};
  if (p.adam) e.a = adam_load(ad, e.a_idx);
  return e;
}

// bias, activation (+ pre-activation), activation-derivative mask, decay; store; fused Adam
static __device__ __forceinline__ void epi_apply(const GemmProb& p, float* C, const AdamCtx& ad, int gi, int gj, float v,
                                                 const EpiPre& e, float lr_t, float& gsq) {
  v += e.bias;
  if (p.act == ACT_RELU) {
    v = fmaxf(v, 0.f);
  } else if (p.act == ACT_SWISH) {
    if (p.Z) p.Z[(int64_t)gi * p.ldc + gj] = v;
    v = swish_fast(v);
  }
  if (p.mask_kind == MASK_DSWISH) v *= dswish_fast(e.mask);
  else if (!(e.mask > 0.f)) v = 0.f;
  if (p.adam) v += p.wd * e.a.p;
  C[(int64_t)gi * p.ldc + gj] = v;
  if (p.adam) {
    adam_apply(ad, e.a_idx, v, e.a, lr_t);
    gsq += v * v;
  }
}

// One 32x32 output tile per 256-thread block (for launches whose problems are all >= 32 x 32):
// each wave owns a 16x16 quadrant over the whole K (no cross-wave reduction), A[32 x 128] and
// B[128 x 32] chunks are staged through LDS with the same unconditional loads as the 16-wide kernel
// (16 per operand and thread), half the operand traffic per output of 16x16 tiles and a quarter of
// the blocks.  Epilogue: the tile goes through LDS, 4 elements per thread (same fused operations).
constexpr int GKC32 = 128;
// The 32x32 tile `bid` of a group; GG: GemmGroup or any struct with its n / prefix / p / ad members
// (bnn_train.hip's weight-gradient launch with the loss tail as its last block)
template <class GG>
static __device__ __forceinline__ void gemm32_body(const GG& g, int bid) {
  __shared__ __attribute__((aligned(16))) float As[GKC32 * 32];
  __shared__ __attribute__((aligned(16))) float Bs[GKC32 * 32];
  __shared__ float tile[32][33];
  __shared__ float csum[8][33];
  __shared__ float red[4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int pi = 0;
  while (pi + 1 < g.n && bid >= g.prefix[pi + 1]) ++pi;
  const GemmProb& p = g.p[pi];
  int t0 = bid - g.prefix[pi];
  const int tn_cnt = ceil_div(p.N, 32);
  int64_t oA = 0, oB = 0, oC = 0, oCs = 0;   // a batched problem's batch (gemm_group_kernel)
  if (p.nb > 1) {
    const int per = ceil_div(p.M, 32) * tn_cnt, b = t0 / per;
    t0 -= b * per;
    oA = (int64_t)b * (p.ta ? p.K : p.M) * p.lda;
    oB = (int64_t)b * (p.tb ? p.N : p.K) * p.ldb;
    oC = (int64_t)b * p.M * p.ldc;
    oCs = (int64_t)b * p.N;
  }
  float* const pC = p.C + oC;
  float* const pcs = p.colsum ? p.colsum + oCs : nullptr;
  const int tm = t0 / tn_cnt, tn = t0 % tn_cnt;
  const int i0 = tm * 32, j0 = tn * 32;
  const int wi = w >> 1, wj = w & 1, li = lane & 15, lk = lane >> 4;
  const bool do_cs = p.colsum && tm == 0;
  const AdamCtx& ad = g.ad;
  EpiPre pre[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) pre[q] = epi_prefetch(p, pC, ad, i0 + (tid >> 5) + 8 * q, j0 + (tid & 31));
  const int64_t c_idx = p.adam && p.colsum ? (int64_t)(pcs - ad.G) + min(j0 + (tid & 31), p.N - 1) : 0;
  AdamIn c_in{0.f, 0.f, 0.f, 0.f};
  float lr_t = 0.f;
  if (p.adam) {
    if (do_cs && tid < 32) c_in = adam_load(ad, c_idx);
    lr_t = *ad.lr_t;
  }
  f32x4 acc0 = zero4(), acc1 = zero4();
  float cs = 0.f;
  // one 128-deep chunk of the tile out of the staged panels (measured: loading chunk c + 1 during chunk
  // c's MFMAs from a second LDS buffer pair took 238 VGPRs and 68 KB, 2 workgroups per CU instead of 4,
  // and BNN.train fell 10.24k -> 9.47k grad-steps/s, same-box A/B)
  auto compute = [&](const float* A_s, const float* B_s, int kn, int t) {
    const int ra_r = wi * 16 + (t & 15), rb_r = wj * 16 + (t & 15), tlk = (t >> 4) & 3;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      float ra[16], rb[16];
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int k = 4 * (half * 16 + s) + tlk;
        ra[s] = A_s[k * 32 + (ra_r ^ pswz<32>(k))];
        rb[s] = B_s[k * 32 + (rb_r ^ pswz<32>(k))];
      }
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        if (s & 1) acc1 = mfma4(ra[s], rb[s], acc1);
        else acc0 = mfma4(ra[s], rb[s], acc0);
      }
    }
    if (do_cs)
      for (int k = tid >> 5; k < kn; k += 8) cs += B_s[k * 32 + ((tid & 31) ^ pswz<32>(k))];
  };
  for (int kc = 0; kc < p.K; kc += GKC32) {
    const int kn = min(GKC32, p.K - kc);
    int t = tid;
    asm volatile("" : "+v"(t));
    stage_dispatch<32>(p, i0, j0, kc, kn, t, As, Bs, oA, oB);
    __syncthreads();
    compute(As, Bs, kn, t);
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) tile[wi * 16 + 4 * lk + r][wj * 16 + li] = acc0[r] + acc1[r];
  if (do_cs) csum[tid >> 5][tid & 31] = cs;
  __syncthreads();
  float gsq = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int ei = (tid >> 5) + 8 * q, ej = tid & 31;
    const int gi = i0 + ei, gj = j0 + ej;
    if (gi < p.M && gj < p.N) epi_apply(p, pC, ad, gi, gj, tile[ei][ej], pre[q], lr_t, gsq);
  }
  if (do_cs && tid < 32) {
    float c = 0.f;
    for (int q = 0; q < 8; ++q) c += csum[q][tid];
    if (j0 + tid < p.N) {
      pcs[j0 + tid] = c;
      if (p.adam) {
        adam_apply(ad, c_idx, c, c_in, lr_t);
        gsq += c * c;
      }
    }
  }
  if (ad.norm_part) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) gsq += __shfl_xor(gsq, off);
    if (lane == 0) red[w] = gsq;
    __syncthreads();
    if (tid == 0) {
      const float b = red[0] + red[1] + red[2] + red[3];
      const int64_t off = p.adam ? (int64_t)(pC - ad.G) : -1;
      float* np = ad.norm_part + 2 * (int64_t)(ad.slot0 + bid);
      np[0] = off >= 0 && off < ad.n_pi ? b : 0.f;
      np[1] = off >= ad.n_pi && off < ad.n_pi + ad.n_q ? b : 0.f;
    }
  }
}

static __global__ __launch_bounds__(256, 2) void gemm32_group_kernel(const GemmGroup g) { gemm32_body(g, (int)blockIdx.x); }
#endif

// ---------------------------------------------------------------------------------------------
static inline GemmProb mk(int M, int N, int K, const float* A, int lda, int ta, const float* B, int ldb, int tb, float* C,
                   int ldc) {
  GemmProb p{};
  p.M = M; p.N = N; p.K = K; p.A = A; p.lda = lda; p.ta = ta; p.B = B; p.ldb = ldb; p.tb = tb; p.C = C; p.ldc = ldc;
  return p;
}

#if MOPO_GEMM_KERNELS
// Tile policy: 16x16 (gemm_group_kernel).  MOPO_GEMM_TILE=32 selects gemm32_group_kernel for launches
// whose problems are all >= 32 x 32.  Measured on MI355X: 32x32 tiles are slower
// for both users (SAC step 115.7 vs 99.8 us, BNN.train 6.09k vs 6.51k steps/s): these launches are
// latency-bound and the 16x16 tiles split K over four waves (16-deep MFMA chains instead of 64).
static inline int gemm_tile_override() {
  static const int v = [] {
    const char* e = std::getenv("MOPO_GEMM_TILE");
    return e ? std::atoi(e) : 0;
  }();
  return v;
}

// tile: 0 the policy above; 32 the 32x32 kernel whatever the problem sizes (partial tiles are range-checked)
static inline int launch_group(std::vector<GemmProb> ps, hipStream_t s, const AdamCtx* ad = nullptr, int* slot = nullptr,
                               const Stamps* st = nullptr, int tile = 0) {
  GemmGroup g{};
  if (st) g.st = *st;
  g.n = (int)ps.size();
  if (g.n > MAXP) return fail("gemm group too large");
  bool big = true;
  for (int i = 0; i < g.n; ++i) {
    GemmProb& q = ps[i];
    if (q.nb < 1) q.nb = 1;
    if (q.nb > 1 && (q.bias || q.Z || q.mask || q.a_u || q.b_u || q.B2))
      return fail("gemm group: a batched problem takes plain operands only");
    const int c = operand_modes(q);
    if (!(c == 0 || c == 1 || c == 3 || c == 4 || c == 6 || c == 9)) return fail("unsupported gemm operand modes");
    if ((int64_t)q.M * q.K >= (1ll << 29) || (int64_t)q.N * q.K >= (1ll << 29)) return fail("gemm operand too large");
    big = big && q.M >= 32 && q.N >= 32;
  }
  const int ov = gemm_tile_override();
  const int TW = (tile == 32 || (ov == 32 && big)) ? 32 : 16;
  int tot = 0;
  for (int i = 0; i < g.n; ++i) {
    g.p[i] = ps[i];
    g.prefix[i] = tot;
    tot += ps[i].nb * ceil_div(ps[i].M, TW) * ceil_div(ps[i].N, TW);
  }
  g.prefix[g.n] = tot;
  if (ad) {
    g.ad = *ad;
    g.ad.slot0 = slot ? *slot : 0;
    if (slot) *slot += tot;
  }
  if (TW == 32) hipLaunchKernelGGL(gemm32_group_kernel, dim3(tot), dim3(256), 0, s, g);
  else hipLaunchKernelGGL(gemm_group_kernel, dim3(tot), dim3(256), 0, s, g);
  MOPO_HIP(hipGetLastError());
  return 0;
}

#endif

}  // namespace mopo
