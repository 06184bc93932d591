// The SAC step's weight-gradient launch (B2, sac.hip): every weight gradient of the step, each with
// its TF1 Adam (+ Polyak for the critics) fused into the epilogue, plus the batch loss tail.
//
// Every problem is C[M][N] = A^T B with the batch rows as the contraction index k < n:
//   A(i, k) = A[k lda + i]                              (an activation / input slab, rows = batch)
//   B(k, j) = B[k ldb + j]                              (a delta slab), or rank-1 masked
//   B(k, j) = bu[k] bv[j] (bm[k bldm + j] > 0)          (a critic's dh2 = dq (x) W3 * (h2 > 0), never stored)
// (mopo.py:337-447: the gradients TF forms for the four optimizers).
//
// One 32 x 32 output tile per 1024-thread workgroup (16 waves): wave w owns the 16 x 16 quadrant w & 3 of
// the tile over the K quarter w >> 2 (16 v_mfma_f32_16x16x4_f32), the four K quarters are summed through
// LDS in a fixed order.  Against 16 x 16 tiles of 4 waves (gemm_group.h, the previous form of this launch)
// a CU stages one 32 x 256 A panel and one 256 x 32 B panel (64 KB) instead of ~3.6 tiles' worth (116 KB):
// the launch is bound by how fast each CU pulls the operands the previous launches wrote, not by the MFMAs.
// Panels are staged as [row][k] (k contiguous, stride 260 floats) so one ds_read_b128 feeds four MFMAs and
// the 16 lanes of each b128 read group hit distinct bank quads.
//
// Block 0 is the loss tail (mopo.py:361-404, 415-443): the batch sums of every per-row loss term in a fixed
// order, the logs, the alpha gradient and its Adam, and the step counter -- nothing else in this launch
// reads them, so it runs beside the tiles (it used to bound the activation-gradient launch B1).
#pragma once
#include "sac_rows.h"

namespace mopo {

struct WgProb {
  int M, N;
  int cls;                           // the single-launch step: 0 = a critic's (waits on B1's critic blocks), 1 = the policy's
  const float* A; int lda;
  const float* B; int ldb;
  const float* bu; const float* bv; const float* bm; int bldm;   // rank-1 masked B when bu != NULL
  float* C; int ldc;                 // a gradient slice of AdamCtx::G
  float* colsum;                     // bias gradient colsum[j] = sum_k B(k, j) (tiles of tile-row 0), or NULL
};

constexpr int WG_MAXP = 12;
constexpr int WG_TILE = 32;
constexpr int WG_KC = 256;           // K chunk staged per pass (the batch; n <= 1024 takes up to 4 passes)
constexpr int WG_KP = WG_KC + 4;     // panel row stride (floats)

struct WgradArgs {
  int n, np;
  int prefix[WG_MAXP + 1];           // tile offsets of the problems (block 1 + prefix[p] is problem p's tile 0)
  WgProb p[WG_MAXP];
  AdamCtx ad;
  // the loss tail (block 0)
  LossRows L;
  int A, ncq;
  float tent;
  float* logs;
  int64_t* iter;
  int prior;                         // action_prior 'normal': the policy loss logs - log N(a; 0, I)
  const float* eps_s;                // [n][EPW] the step's policy noise of pi(s) (for the action)
  Stamps st;
  const unsigned* sync_tmo;          // a fused launch's sticky timeout word, or NULL
  unsigned* sync_reset; int n_sync;  // F1 + F2 + B1 fused: the loss tail zeroes the next step's counters
};

// Block 0: per-row loss terms of all n rows (thread t: rows t, t + 1024, ...), block sums in a fixed order
// (deterministic), then thread 0 applies the batch-level updates.  lr_t was formed by the activation-
// gradient launch (sac_dh1_kernel's step control) from the beta powers of this step.
static __device__ __forceinline__ void wgrad_loss_tail(const WgradArgs& a, float* sh) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, nw = blockDim.x >> 6;
  const int n = a.n, A = a.A;
  const AdamCtx& ad = a.ad;
  if (a.sync_reset && tid < a.n_sync) a.sync_reset[tid * SYNC_STRIDE] = 0u;   // read by the next launch only
  AdamIn al{0.f, 0.f, 0.f, 0.f};
  float lr_t = 0.f;
  if (tid == 0) {
    al = adam_load(ad, ad.total);                                     // log_alpha = the last parameter
    lr_t = *ad.lr_t;
  }
  float red[7] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const auto dls = rsrc(a.L.head_s, (int64_t)n * 2 * A), dlp = rsrc(a.L.logp_s, 2 * rows_ns(n));
  for (int r0 = 0; r0 < n; r0 += blockDim.x) {
    const int r = r0 + tid;
    const bool on = r < n;
    // every load of the row first (one memory latency), then the terms
    const RowIn in = row_losses_load(a.L, n, a.ncq, r, on);
    const float lps = bload(dlp, on ? lp_idx(r) : -1);
    float lsv[8], muv[8], epv[8];
    const auto dep = rsrc(a.eps_s, (int64_t)n * EPW);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      lsv[j] = bload(dls, (on && j < A) ? r * 2 * A + A + j : -1);
      muv[j] = bload(dls, (a.prior && on && j < A) ? r * 2 * A + j : -1);
      epv[j] = bload(dep, (a.prior && on && j < A) ? r * EPW + j : -1);
    }
    if (!on) continue;
    const RowQ o = row_losses(a.L, in);
    const float q1 = o.q[0], q2 = o.q[1], q1p = o.q[2], q2p = o.q[3];
    float ent = 0.f;                                                  // pi_entropy terms (mopo.py:341)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (j >= A) break;
      const float ls = fminf(fmaxf(lsv[j], -20.f), 2.f);
      ent += logf(expf(ls) + 1e-8f) + 0.5f * logf(2.f * 3.14159265358979f * 2.718281828459045f);
    }
    red[0] += (q1 - o.y) * (q1 - o.y); red[1] += (q2 - o.y) * (q2 - o.y); red[2] += q1; red[3] += q2;
    float lprior = 0.f;                                               // log N(a; 0, I) of pi(s)'s action
    if (a.prior) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (j >= A) break;
        const float act = tanhf(muv[j] + epv[j] * expf(fminf(fmaxf(lsv[j], -20.f), 2.f)));
        lprior -= 0.5f * act * act;
      }
      lprior -= 0.5f * (float)A * 1.8378770664093453f;
    }
    red[4] += lps; red[5] += ent; red[6] += o.alpha * lps - fminf(q1p, q2p) - lprior;
  }
#pragma unroll
  for (int i = 0; i < 7; ++i)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) red[i] += __shfl_xor(red[i], off);
  if (lane == 0)
#pragma unroll
    for (int i = 0; i < 7; ++i) sh[w * 8 + i] = red[i];
  lds_barrier();
  if (tid != 0) return;
#pragma unroll
  for (int i = 0; i < 7; ++i) {                                       // wave partials in wave order
    float t = 0.f;
    for (int q = 0; q < nw; ++q) t += sh[8 * q + i];
    red[i] = t;
  }
  const float fn = (float)n;
  const float l1 = red[0] / fn * 0.5f, l2 = red[1] / fn * 0.5f;       // mopo.py:403-404
  const float m1 = red[2] / fn, m2 = red[3] / fn, mlp = red[4] / fn, ment = red[5] / fn;
  const float pil = red[6] / fn;                                      // mopo.py:371-377
  const float ga = -(mlp + a.tent);                                   // d/dlog_alpha of -mean(la*(logp+H))
  if (a.sync_tmo && *a.sync_tmo) {    // a fused launch gave up waiting (sac_rows.h handoff_wait): poison the logs,
    const float nan = __builtin_nanf("");   // hold log_alpha (as the tiles hold every parameter); the host's
    for (int i = 0; i < LOG_N; ++i) a.logs[i] = nan;   // mopo_sac_check reports it and clears the word
    adam_apply(ad, ad.total, ga, al, lr_t, nullptr, true);
    *a.iter += 1;
    return;
  }
  const_cast<float*>(ad.G)[ad.total] = ga;
  float* logs = a.logs;
  logs[LOG_Q1_LOSS] = l1; logs[LOG_Q2_LOSS] = l2; logs[LOG_Q1] = m1; logs[LOG_Q2] = m2;
  logs[LOG_ALPHA] = expf(al.p); logs[LOG_ENTROPY] = ment; logs[LOG_LOGP] = mlp; logs[LOG_PI_LOSS] = pil;
  *a.iter += 1;
  adam_apply(ad, ad.total, ga, al, lr_t);
}

// Grid: 1 + tiles blocks of 1024 threads (block 0 the loss tail).  n >= 1; problems as WgProb.
static __global__ __launch_bounds__(1024, 1) void sac_wgrad_kernel(const WgradArgs g) {
  __shared__ __attribute__((aligned(16))) float As[WG_TILE * WG_KP];   // [i][k]; later the K-quarter partials
  __shared__ __attribute__((aligned(16))) float Bs[WG_TILE * WG_KP];   // [j][k]
  __shared__ float red[16];
  stamp(g.st, 0);
  if (blockIdx.x == 0) {
    wgrad_loss_tail(g, As);
    stamp(g.st, 4);
    return;
  }
  const int bid = (int)blockIdx.x - 1;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  int pi = 0;
  while (pi + 1 < g.np && bid >= g.prefix[pi + 1]) ++pi;
  const WgProb& p = g.p[pi];
  const int t = bid - g.prefix[pi];
  const int tn_cnt = ceil_div(p.N, WG_TILE);
  const int tm = t / tn_cnt, tn = t % tn_cnt;
  const int i0 = tm * WG_TILE, j0 = tn * WG_TILE;
  const int n = g.n;
  const bool do_cs = p.colsum && tm == 0;
  // ---- epilogue operands first (their latency overlaps the panel loads): this thread's output element
  //      (tid / 32, tid % 32) and, for tile-row 0, the bias element of column tid / 32
  const AdamCtx& ad = g.ad;
  const int ei = tid >> 5, ej = tid & 31;
  const int gi = i0 + ei, gj = j0 + ej;
  const bool e_on = gi < p.M && gj < p.N;
  const int64_t a_idx = (int64_t)(p.C - ad.G) + (int64_t)min(gi, p.M - 1) * p.ldc + min(gj, p.N - 1);
  AdamIn a_in = adam_load(ad, a_idx);
  const int cj = tid >> 5;                                            // colsum: column cj, k-slice tid % 32
  const bool c_on = do_cs && (tid & 31) == 0 && j0 + cj < p.N;
  const int64_t c_idx = p.colsum ? (int64_t)(p.colsum - ad.G) + min(j0 + cj, p.N - 1) : 0;
  AdamIn c_in{0.f, 0.f, 0.f, 0.f};
  if (c_on) c_in = adam_load(ad, c_idx);
  const float lr_t = *ad.lr_t;
  const bool hold = g.sync_tmo && *g.sync_tmo;   // a give-up in the fused launch: no update from stale operands
  asm volatile("" : "+v"(a_in.p), "+v"(a_in.m), "+v"(a_in.v), "+v"(a_in.t));
  const int qd = w & 3, qi = qd >> 1, qj = qd & 1, kq = w >> 2;
  const int li = lane & 15, lk = lane >> 4;
  f32x4 acc0 = zero4(), acc1 = zero4();
  float cs = 0.f;
  const auto dA = rsrc(p.A, (int64_t)(n - 1) * p.lda + p.M);
  const bool r1 = p.bu != nullptr;
  const auto dB = rsrc(r1 ? p.bm : p.B, (int64_t)(n - 1) * (r1 ? p.bldm : p.ldb) + p.N);
  const auto dU = rsrc(p.bu, r1 ? n : 0);
  const float bv = r1 ? bload(rsrc(p.bv, p.N), j0 + ej) : 0.f;
  for (int kc = 0; kc < n; kc += WG_KC) {
    // ---- panels: element e = tid + 1024 q (q < 8) is (row e % 32, k e / 32) -- 32 consecutive floats of
    //      one batch row per half-wave; loads past the operand's extent (k >= n) return 0
    int tt = tid;
    asm volatile("" : "+v"(tt));
    float va[8], vb[8], vu[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = tt + 1024 * q, r = e & 31, k = kc + (e >> 5);
      va[q] = bload(dA, k * p.lda + i0 + r);
      vb[q] = bload(dB, k * (r1 ? p.bldm : p.ldb) + j0 + r);
      vu[q] = r1 ? bload(dU, k) : 1.f;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = tt + 1024 * q, r = e & 31, k = e >> 5;
      As[r * WG_KP + k] = va[q];
      Bs[r * WG_KP + k] = r1 ? (vb[q] > 0.f ? vu[q] * bv : 0.f) : vb[q];
    }
    lds_barrier();
    stamp(g.st, 1);
    // ---- the wave's quadrant over its K quarter: k = 64 kq + 16 lk + 4 s + u
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int k = 64 * kq + 16 * lk + 4 * s;
      const f32x4 a4 = ld4(As + (16 * qi + li) * WG_KP + k), b4 = ld4(Bs + (16 * qj + li) * WG_KP + k);
      acc0 = mfma4(a4[0], b4[0], acc0);
      acc1 = mfma4(a4[1], b4[1], acc1);
      acc0 = mfma4(a4[2], b4[2], acc0);
      acc1 = mfma4(a4[3], b4[3], acc1);
    }
    if (do_cs) {                                                      // column cj, k = 8 (tid % 32) .. + 7
      const float* bp = Bs + cj * WG_KP + 8 * (tid & 31);
      const f32x4 x0 = ld4(bp), x1 = ld4(bp + 4);
      cs += ((x0[0] + x0[1]) + (x0[2] + x0[3])) + ((x1[0] + x1[1]) + (x1[2] + x1[3]));
    }
    lds_barrier();
  }
  stamp(g.st, 2);
  // ---- K quarters through LDS (As reused): part[kq][row * 32 + col], D: col li, rows 4 lk + r
  float* part = As;
#pragma unroll
  for (int r = 0; r < 4; ++r) part[kq * 1024 + (16 * qi + 4 * lk + r) * 32 + 16 * qj + li] = acc0[r] + acc1[r];
  if (do_cs) {                                                        // the 32 k-slices of column cj
#pragma unroll
    for (int off = 16; off > 0; off >>= 1) cs += __shfl_xor(cs, off);
  }
  lds_barrier();
  float gsq = 0.f;
  {
    const float v = (part[tid] + part[1024 + tid]) + (part[2048 + tid] + part[3072 + tid]);
    if (e_on) {
      p.C[(int64_t)gi * p.ldc + gj] = v;
      adam_apply(ad, a_idx, v, a_in, lr_t, nullptr, hold);
      gsq = v * v;
    }
  }
  if (c_on) {
    p.colsum[j0 + cj] = cs;
    adam_apply(ad, c_idx, cs, c_in, lr_t, nullptr, hold);
    gsq += cs * cs;
  }
  if (ad.norm_part) {  // per-block squared-gradient partial (grad-norm logs; summed by sac_logs_kernel)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) gsq += __shfl_xor(gsq, off);
    if (lane == 0) red[w] = gsq;
    lds_barrier();
    if (tid == 0) {
      float b = 0.f;
      for (int q = 0; q < 16; ++q) b += red[q];
      const int64_t off = (int64_t)(p.C - ad.G);
      float* np = ad.norm_part + 2 * (int64_t)(ad.slot0 + bid);
      np[0] = off >= 0 && off < ad.n_pi ? b : 0.f;
      np[1] = off >= ad.n_pi && off < ad.n_pi + ad.n_q ? b : 0.f;
    }
  }
  stamp(g.st, 4);
}

static inline WgProb wprob(int M, int N, const float* A, int lda, const float* B, int ldb, float* C, int ldc,
                           float* colsum) {
  WgProb p{};
  p.M = M; p.N = N; p.A = A; p.lda = lda; p.B = B; p.ldb = ldb; p.C = C; p.ldc = ldc; p.colsum = colsum;
  return p;
}

static inline int wgrad_tiles(int M, int N) { return ceil_div(M, WG_TILE) * ceil_div(N, WG_TILE); }

}  // namespace mopo
