// MOPO's in-graph SAC update (K6/K7): forward, hand-derived backward, four TF1 Adams, Polyak.
//
// Replaces MOPO._build's training graph and MOPO._do_training / _update_target
// (mopo/algorithms/mopo.py:275-466, 834-853); batch assembly MOPO._training_batch (mopo.py:801-821).
// Semantics: every forward and gradient uses the pre-step parameters; then pi, q1, q2
// and alpha are updated by their own Adam (identical step counts -> one shared lr_t); then Polyak.
//
// Structure: ~17 launches per step on one stream (batch gather, 3 grouped-GEMM forward stages for
// pi(s), pi(s'), Q1/Q2(s,a), the squashed-Gaussian head, 3 for Q1/Q2(s,pi) and the targets, a
// single-block loss kernel, 4 grouped-GEMM backward stages with fused relu masks and bias-gradient
// column sums, the policy-head backward, one fused Adam+Polyak pass).  The sequence has fixed
// pointers, so it is captured once into a hipGraph and replayed (no host work per step).
// GEMMs are f32-in/f32-acc MFMA (v_mfma_f32_16x16x4_f32): a 16x16 output tile per 256-thread
// block, K split across the four waves and reduced through LDS -- the shapes are tiny (batch 256,
// width 256), so the kernel is built for latency (many small independent tiles), not throughput.
#include <vector>
#include <cstring>

#include "internal.h"

namespace mopo {

constexpr int MAXP = 8;

struct GemmProb {
  int M, N, K;
  const float* A; int lda; int ta;   // ta=0: A(i,k)=A[i*lda+k]; ta=1: A(i,k)=A[k*lda+i]
  const float* B; int ldb; int tb;   // tb=0: B(k,j)=B[k*ldb+j]; tb=1: B(k,j)=B[j*ldb+k]
  float* C; int ldc;
  const float* bias;                 // C += bias[j]
  int relu;                          // C = max(C, 0)
  const float* mask; int ldm;        // C *= (mask(i,j) > 0)   (relu' from the saved activation)
  float* colsum;                     // colsum[j] = sum_k B(k,j)   (bias gradient), by tile-row 0
  // rank-1 masked operands (the critic's 1-wide output layer backward, fused into its consumer):
  // when a_u != NULL:  A(i,k) = a_u[i] * a_v[k] * (a_m[i*a_ldm + k] > 0);  same for B with (k, j)
  const float* a_u; const float* a_v; const float* a_m; int a_ldm;
  const float* b_u; const float* b_v; const float* b_m; int b_ldm;
};

struct GemmGroup {
  int n;
  int prefix[MAXP + 1];
  GemmProb p[MAXP];
};


constexpr int GKC = 256;  // K chunk staged in LDS

// One 16-wide panel (A: rows i0..i0+15, or B: cols j0..j0+15) x K-chunk, staged as S[k][r].
// MODE 0: plain, 1: transposed, 2: rank-1 masked (see GemmProb).  Addresses are clamped so every
// load is valid and unconditional; out-of-range elements are zeroed by a select afterwards.
struct PanelRegs { float x[16], u[16], w[16]; };

template <int MODE, bool IS_A>
__device__ __forceinline__ void panel_rk(int q, int tid, int& r, int& k) {
  constexpr bool rfast = IS_A ? (MODE == 1) : (MODE != 1);
  if (rfast) { r = tid & 15; k = (tid >> 4) + 16 * q; }
  else { k = (tid & 63) + 64 * (q & 3); r = (tid >> 6) + 4 * (q >> 2); }
}

template <int MODE, bool IS_A>
__device__ __forceinline__ void load_panel(const GemmProb& p, int r0, int kc, int tid, PanelRegs& R) {
  const int Rmax = IS_A ? p.M : p.N;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    int r, k;
    panel_rk<MODE, IS_A>(q, tid, r, k);
    const int rc = min(r0 + r, Rmax - 1), kk = min(kc + k, p.K - 1);
    if (MODE == 2) {
      const float* m = IS_A ? p.a_m : p.b_m;
      const int ldm = IS_A ? p.a_ldm : p.b_ldm;
      R.u[q] = IS_A ? p.a_u[rc] : p.b_u[kk];
      R.w[q] = IS_A ? p.a_v[kk] : p.b_v[rc];
      R.x[q] = IS_A ? m[(int64_t)rc * ldm + kk] : m[(int64_t)kk * ldm + rc];
    } else if (IS_A) {
      R.x[q] = MODE == 0 ? p.A[(int64_t)rc * p.lda + kk] : p.A[(int64_t)kk * p.lda + rc];
    } else {
      R.x[q] = MODE == 0 ? p.B[(int64_t)kk * p.ldb + rc] : p.B[(int64_t)rc * p.ldb + kk];
    }
  }
}

// pin the loads as unconditional (else hipcc sinks each into a branch followed by vmcnt(0))
template <int MODE>
__device__ __forceinline__ void pin_panel(PanelRegs& R) {
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    asm volatile("" : "+v"(R.x[q]));
    if (MODE == 2) asm volatile("" : "+v"(R.u[q]), "+v"(R.w[q]));
  }
}

template <int MODE, bool IS_A>
__device__ __forceinline__ void store_panel(const GemmProb& p, int r0, int kn, int tid, const PanelRegs& R,
                                            float (*S)[16]) {
  const int Rmax = IS_A ? p.M : p.N;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    int r, k;
    panel_rk<MODE, IS_A>(q, tid, r, k);
    const float v = MODE == 2 ? (R.x[q] > 0.f ? R.u[q] * R.w[q] : 0.f) : R.x[q];
    S[k][r] = (r0 + r < Rmax && k < kn) ? v : 0.f;
  }
}

template <int AM, int BM>
__device__ __forceinline__ void stage_ab(const GemmProb& p, int i0, int j0, int kc, int kn, int tid, float (*As)[16],
                                         float (*Bs)[16]) {
  PanelRegs ra, rb;
  load_panel<AM, true>(p, i0, kc, tid, ra);
  load_panel<BM, false>(p, j0, kc, tid, rb);
  pin_panel<AM>(ra);
  pin_panel<BM>(rb);
  store_panel<AM, true>(p, i0, kn, tid, ra, As);
  store_panel<BM, false>(p, j0, kn, tid, rb, Bs);
}

// One 16x16 output tile per 256-thread block.  The A[16 x K] and B[K x 16] panels are staged in
// LDS with loads ordered along each operand's contiguous axis (all issued before the first use:
// one memory latency per chunk), then the four waves split K and run v_mfma_f32_16x16x4_f32 out
// of LDS; partial tiles are summed through LDS and the epilogue fuses bias / relu / relu'-mask.
__global__ __launch_bounds__(256) void gemm_group_kernel(const GemmGroup g) {
  __shared__ float As[GKC][16];
  __shared__ float Bs[GKC][16];
  __shared__ float part[4][256];
  __shared__ float csum[16][17];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int pi = 0;
  while (pi + 1 < g.n && (int)blockIdx.x >= g.prefix[pi + 1]) ++pi;
  const GemmProb& p = g.p[pi];
  const int t = blockIdx.x - g.prefix[pi];
  const int tn_cnt = ceil_div(p.N, 16);
  const int tm = t / tn_cnt, tn = t % tn_cnt;
  const int i0 = tm * 16, j0 = tn * 16;
  const int li = lane & 15, lk = lane >> 4;
  const bool do_cs = p.colsum && tm == 0;
  // epilogue operands are fetched up front so their latency overlaps the panel loads
  const int ei = tid >> 4, ej = tid & 15;
  const int gi = i0 + ei, gj = j0 + ej;
  const int gic = min(gi, p.M - 1), gjc = min(gj, p.N - 1);
  float e_bias = p.bias ? p.bias[gjc] : 0.f;
  float e_mask = p.mask ? p.mask[(int64_t)gic * p.ldm + gjc] : 1.f;
  asm volatile("" : "+v"(e_bias), "+v"(e_mask));
  f32x4 acc0 = zero4(), acc1 = zero4();
  float cs = 0.f;
  for (int kc = 0; kc < p.K; kc += GKC) {
    const int kn = min(GKC, p.K - kc);
    const int kpad = (kn + 3) & ~3;
    // 16 elements of each panel per thread; the per-operand mode is dispatched once (uniform
    // branch) so that all 32+ loads are unconditional (clamped addresses, select after the load)
    // and issue back to back -- one memory latency per chunk instead of one per element.
    const int am = p.a_u ? 2 : p.ta, bm = p.b_u ? 2 : p.tb;
    switch (am * 3 + bm) {
      case 0: stage_ab<0, 0>(p, i0, j0, kc, kn, tid, As, Bs); break;
      case 1: stage_ab<0, 1>(p, i0, j0, kc, kn, tid, As, Bs); break;
      case 2: stage_ab<0, 2>(p, i0, j0, kc, kn, tid, As, Bs); break;
      case 3: stage_ab<1, 0>(p, i0, j0, kc, kn, tid, As, Bs); break;
      case 4: stage_ab<1, 1>(p, i0, j0, kc, kn, tid, As, Bs); break;
      case 5: stage_ab<1, 2>(p, i0, j0, kc, kn, tid, As, Bs); break;
      case 6: stage_ab<2, 0>(p, i0, j0, kc, kn, tid, As, Bs); break;
      case 7: stage_ab<2, 1>(p, i0, j0, kc, kn, tid, As, Bs); break;
      default: stage_ab<2, 2>(p, i0, j0, kc, kn, tid, As, Bs); break;
    }
    __syncthreads();
    (void)kpad;
    // the staged panels are zero-padded to GKC rows, so every wave runs exactly 16 k-steps of its
    // quarter with no guards: all 32 LDS reads first, then 16 MFMAs on two accumulators
    float ra[16], rb[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int k = 4 * (w * 16 + s) + lk;
      ra[s] = As[k][li];
      rb[s] = Bs[k][li];
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s & 1) acc1 = mfma4(ra[s], rb[s], acc1);
      else acc0 = mfma4(ra[s], rb[s], acc0);
    }
    if (do_cs)
      for (int k = tid >> 4; k < kn; k += 16) cs += Bs[k][tid & 15];
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) part[w][(lk * 4 + r) * 16 + li] = acc0[r] + acc1[r];  // D: col li, row 4*lk+r
  if (do_cs) csum[tid >> 4][tid & 15] = cs;
  __syncthreads();
  {
    float v = part[0][tid] + part[1][tid] + part[2][tid] + part[3][tid];
    if (gi < p.M && gj < p.N) {
      v += e_bias;
      if (p.relu) v = fmaxf(v, 0.f);
      if (!(e_mask > 0.f)) v = 0.f;
      p.C[(int64_t)gi * p.ldc + gj] = v;
    }
  }
  if (do_cs && tid < 16) {
    float c = 0.f;
    for (int q = 0; q < 16; ++q) c += csum[q][tid];
    if (j0 + tid < p.N) p.colsum[j0 + tid] = c;
  }
}

// ---------------------------------------------------------------------------------------------
struct SacDims { int O, A, H, n, n_env; int64_t P; };

// parameter offsets (flat, TF creation order; mopo.py:32-33)
struct Offs {
  int64_t pW1, pb1, pW2, pb2, pWm, pbm, pWl, pbl;
  int64_t q[2][6];  // W1 b1 W2 b2 W3 b3 for q1, q2
  int64_t n_pi, n_q, total;
};

static Offs make_offs(int O, int A, int H) {
  Offs o{};
  int64_t c = 0;
  auto take = [&](int64_t n) { int64_t r = c; c += n; return r; };
  o.pW1 = take((int64_t)O * H); o.pb1 = take(H); o.pW2 = take((int64_t)H * H); o.pb2 = take(H);
  o.pWm = take((int64_t)H * A); o.pbm = take(A); o.pWl = take((int64_t)H * A); o.pbl = take(A);
  o.n_pi = c;
  for (int qi = 0; qi < 2; ++qi) {
    o.q[qi][0] = take((int64_t)(O + A) * H); o.q[qi][1] = take(H); o.q[qi][2] = take((int64_t)H * H);
    o.q[qi][3] = take(H); o.q[qi][4] = take(H); o.q[qi][5] = take(1);
  }
  o.n_q = o.q[1][0] - o.q[0][0];
  o.total = c;
  return o;
}

enum {
  LOG_Q1_LOSS = 0, LOG_Q2_LOSS, LOG_Q1, LOG_Q2, LOG_ALPHA, LOG_ENTROPY, LOG_LOGP, LOG_PI_GNORM, LOG_Q_GNORM,
  LOG_PI_LOSS, LOG_N = 16
};

struct Sac {
  SacDims d{};
  Offs o{};
  float lr, gamma, tau, rscale, tent;
  void* mem = nullptr;
  float *P, *G, *M, *V, *T;       // [total + 1]: last element = log_alpha
  float* beta_pow;                // [2] f32 beta1_power, beta2_power (TF1 non-slot vars)
  int64_t* iter;                  // device step counter (Philox)
  unsigned* ticket;               // last-block ticket of the Adam kernel
  float* logs;                    // [LOG_N]
  float* norm_part;               // [nblk][2]
  int adam_blocks = 0;
  // activations
  float *sa, *xpi, *xn, *rew, *term;
  float *h1[8], *h2[8], *out[8];  // 0 pi(s) 1 pi(s') 2 Q1(s,a) 3 Q2(s,a) 4 Q1(s,pi) 5 Q2(s,pi) 6 Qt1 7 Qt2
  float *logp_s, *logp_n, *eps_s, *eps_n;
  float *dq[4];                   // dq for instances 2,3,4,5
  float *dh2[4], *dh1[4];
  float *dx1, *dx2, *dhead, *dh2p, *dh1p;
  int64_t* idx;                   // [n] sampled rows
  // device arrays of pointers for the multi-instance element-wise kernels
  float** outp_dev;               // [8] out[]
  float** dq_dev;                 // [4]
  float** w3_dev;                 // [4] main W3 of Q1, Q2, Q1, Q2
  float** h2q_dev;                // [4] h2[2..5]
  float** dh2_dev;                // [4]
  // graph
  bool use_graph = true;
  hipGraphExec_t gexec = nullptr;
  hipGraph_t graph = nullptr;
  mopo_pool_desc genv{}, gmod{};
  hipStream_t gstream = nullptr;
  hipEvent_t ev_in = nullptr, ev_out = nullptr;
  uint64_t gseed = 0;
};

// ---- batch gather (_training_batch, mopo.py:801-821): rows [0, n_env) from the env pool, rest
// from the model pool; each index uniform over the pool's live size (Philox) unless injected
// One block per GR rows: phase 1 draws the GR source rows, phase 2 copies their fields with
// consecutive threads on consecutive columns (all loads independent -> one memory latency).
constexpr int GR = 16;
__global__ __launch_bounds__(256) void sac_gather_kernel(const mopo_pool_desc env, const mopo_pool_desc mod, int n,
                                                         int n_env, int O, int A, const int64_t* idx_in,
                                                         int64_t* idx_out, uint64_t seed, const int64_t* iter,
                                                         float* sa, float* xpi, float* xn, float* rew, float* term) {
  __shared__ int64_t src_s[GR];
  const int tid = threadIdx.x;
  const int r0 = blockIdx.x * GR;
  if (tid < GR && r0 + tid < n) {
    const int r = r0 + tid;
    int64_t src;
    if (idx_in) {
      src = idx_in[r];
    } else {
      const uint64_t size = (uint64_t)(r < n_env ? env.d_state[1] : mod.d_state[1]);
      const int64_t it = *iter;
      u32x4 c{(uint32_t)r, (uint32_t)it, (uint32_t)((uint64_t)it >> 32), RNG_SAC};
      u32x4 q = philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
      src = (int64_t)(((uint64_t)q.x * size) >> 32);
    }
    src_s[tid] = src;
    idx_out[r] = src;
  }
  __syncthreads();
  const int W = O + A, C = 2 * O + A + 2;  // obs | act | next_obs | rew | term
  for (int e = tid; e < GR * C; e += 256) {
    const int rr = e / C, c = e % C, r = r0 + rr;
    if (r >= n) continue;
    const bool fe = r < n_env;
    const int64_t src = src_s[rr];
    if (c < O) {
      const float v = (fe ? env.d_obs : mod.d_obs)[src * O + c];
      sa[r * W + c] = v;
      xpi[r * W + c] = v;
    } else if (c < O + A) {
      sa[r * W + c] = (fe ? env.d_act : mod.d_act)[src * A + (c - O)];
    } else if (c < 2 * O + A) {
      xn[r * W + (c - O - A)] = (fe ? env.d_next_obs : mod.d_next_obs)[src * O + (c - O - A)];
    } else if (c == 2 * O + A) {
      rew[r] = (fe ? env.d_rew : mod.d_rew)[src];
    } else {
      term[r] = (float)(fe ? env.d_term : mod.d_term)[src];
    }
  }
}

__device__ __forceinline__ float softplus_f(float x) { return softplusf(x); }

// ---- squashed Gaussian head, forward (mopo.py:282-308, 286-296) for pi(s) and pi(s')
__global__ void pi_head_fwd_kernel(int n, int O, int A, const float* head_s, const float* head_n, const float* eps_in_s,
                                   const float* eps_in_n, float* eps_s, float* eps_n, uint64_t seed,
                                   const int64_t* iter, float* xpi, float* xn, float* logp_s, float* logp_n) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 2 * n) return;
  const bool nxt = t >= n;
  const int r = nxt ? t - n : t;
  const float* hd = (nxt ? head_n : head_s) + r * 2 * A;
  const float* ein = nxt ? eps_in_n : eps_in_s;
  float* eo = (nxt ? eps_n : eps_s) + r * A;
  float z[8];
  if (ein) {
    for (int j = 0; j < A; ++j) z[j] = ein[r * A + j];
  } else {
    for (int blk = 0; blk * 4 < A; ++blk) {
      u32x4 c{(uint32_t)r | ((uint32_t)nxt << 31), (uint32_t)(*iter) ^ ((uint32_t)blk << 24),
              (uint32_t)((uint64_t)(*iter) >> 32), RNG_SAC + 16};
      u32x4 q = philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
      float zz[4];
      box_muller(q.x, q.y, zz[0], zz[1]);
      box_muller(q.z, q.w, zz[2], zz[3]);
      for (int i = 0; i < 4 && blk * 4 + i < A; ++i) z[blk * 4 + i] = zz[i];
    }
  }
  float logp = 0.f, corr = 0.f;
  float* x = (nxt ? xn : xpi) + r * (O + A) + O;
  for (int j = 0; j < A; ++j) {
    const float mu = hd[j];
    const float ls = fminf(fmaxf(hd[A + j], -20.f), 2.f);
    const float sd = expf(ls);
    const float u = mu + z[j] * sd;
    const float zz = (u - mu) / (sd + 1e-8f);
    logp += -0.5f * (zz * zz + 2.f * ls + 1.8378770664093453f);
    corr += 2.f * (0.6931471805599453f - u - softplus_f(-2.f * u));
    x[j] = tanhf(u);
    eo[j] = z[j];
  }
  (nxt ? logp_n : logp_s)[r] = logp - corr;
}

// Deterministic block-wide sums of NV values at once: butterfly within each wave (__shfl_xor),
// then the per-wave partials added in wave order.  Two barriers for all NV sums.
// sh must hold 16 * NV floats; blockDim.x a multiple of 64 (<= 1024).
template <int NV>
__device__ __forceinline__ void block_sums(float (&v)[NV], float* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v[i] += __shfl_xor(v[i], off);
  if (lane == 0)
#pragma unroll
    for (int i = 0; i < NV; ++i) sh[w * NV + i] = v[i];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    float s = 0.f;
    for (int q = 0; q < nw; ++q) s += sh[q * NV + i];
    v[i] = s;
  }
  __syncthreads();
}

__device__ __forceinline__ float block_sum(float v, float* sh) {
  float a[1] = {v};
  block_sums<1>(a, sh);
  return a[0];
}

// ---- losses, output gradients, alpha gradient, logs (single block, one thread per row)
__global__ __launch_bounds__(1024) void sac_loss_kernel(int n, int A, float gamma, float rscale, float tent,
                                                        float* const* outs, const float* logp_s, const float* logp_n,
                                                        const float* rew, const float* term, const float* head_s,
                                                        const float* log_alpha, float* dq1, float* dq2, float* dq1p,
                                                        float* dq2p, float* g_alpha, float* logs) {
  __shared__ float sh[1024];
  const int r = threadIdx.x;
  const bool ok = r < n;
  const float alpha = expf(*log_alpha);                             // mopo.py:361
  float q1 = 0, q2 = 0, q1p = 0, q2p = 0, lps = 0, ent = 0, y = 0;
  if (ok) {
    q1 = outs[2][r]; q2 = outs[3][r]; q1p = outs[4][r]; q2p = outs[5][r];
    const float qt = fminf(outs[6][r], outs[7][r]);                 // mopo.py:368
    y = rscale * rew[r] + gamma * ((1.f - term[r]) * (qt - alpha * logp_n[r]));  // mopo.py:380-386
    lps = logp_s[r];
    const float inv_n = 1.f / (float)n;
    dq1[r] = (q1 - y) * inv_n;                                      // d(0.5 mean (q-y)^2)
    dq2[r] = (q2 - y) * inv_n;
    const bool sel1 = q1p <= q2p;                                   // tf.minimum grad -> x where x <= y
    dq1p[r] = sel1 ? -inv_n : 0.f;
    dq2p[r] = sel1 ? 0.f : -inv_n;
    for (int j = 0; j < A; ++j) {                                   // pi_entropy (mopo.py:341)
      const float ls = fminf(fmaxf(head_s[r * 2 * A + A + j], -20.f), 2.f);
      ent += logf(expf(ls) + 1e-8f) + 0.5f * logf(2.f * 3.14159265358979f * 2.718281828459045f);
    }
  }
  const float fn = (float)n;
  float red[7] = {ok ? (q1 - y) * (q1 - y) : 0.f, ok ? (q2 - y) * (q2 - y) : 0.f, q1, q2, lps, ent,
                  ok ? alpha * lps - fminf(q1p, q2p) : 0.f};
  block_sums<7>(red, sh);
  const float l1 = red[0] / fn * 0.5f, l2 = red[1] / fn * 0.5f;           // mopo.py:403-404
  const float m1 = red[2] / fn, m2 = red[3] / fn, mlp = red[4] / fn, ment = red[5] / fn;
  const float pil = red[6] / fn;                                          // mopo.py:371-377
  if (r == 0) {
    *g_alpha = -(mlp + tent);                                       // d/dlog_alpha of -mean(la*(logp+H))
    logs[LOG_Q1_LOSS] = l1; logs[LOG_Q2_LOSS] = l2; logs[LOG_Q1] = m1; logs[LOG_Q2] = m2;
    logs[LOG_ALPHA] = alpha; logs[LOG_ENTROPY] = ment; logs[LOG_LOGP] = mlp; logs[LOG_PI_LOSS] = pil;
  }
}

// ---- dh2 = dq (x) W3 * (h2 > 0) for the 4 critic instances (rank-1 output layer backward)
__global__ void q_out_bwd_kernel(int n, int H, const float* const* dq, const float* const* W3, const float* const* h2,
                                 float* const* dh2) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int inst = blockIdx.y;
  if (t >= (int64_t)n * H) return;
  const int r = t / H, j = t % H;
  const float h = h2[inst][t];
  dh2[inst][t] = h > 0.f ? dq[inst][r] * W3[inst][j] : 0.f;
}

// ---- squashed Gaussian head backward + dh2 of the policy trunk (one block per batch row)
__global__ __launch_bounds__(256) void pi_head_bwd_kernel(int n, int O, int A, int H, const float* head_s,
                                                          const float* eps_s, const float* dx1, const float* dx2,
                                                          const float* log_alpha, const float* Wm, const float* Wl,
                                                          const float* h2p, float* dhead, float* dh2p) {
  __shared__ float dmu_s[8], dls_s[8];
  const int r = blockIdx.x, tid = threadIdx.x;
  if (tid < A) {
    const int j = tid;
    const float g = expf(*log_alpha) / (float)n;                    // d L_pi / d logp (stop_gradient(alpha))
    const float mu = head_s[r * 2 * A + j], raw = head_s[r * 2 * A + A + j];
    const float ls = fminf(fmaxf(raw, -20.f), 2.f);
    const float sd = expf(ls);
    const float e = eps_s[r * A + j];
    const float u = mu + e * sd;
    const float a = tanhf(u);
    const float inv = 1.f / (sd + 1e-8f);
    const float zz = (u - mu) * inv;
    const float da = dx1[r * (O + A) + O + j] + dx2[r * (O + A) + O + j];  // -dmin q / da through Q1/Q2
    float du = da * (1.f - a * a);                                  // tanh grad (y-based)
    du += g * (-zz * inv);                                          // gaussian_likelihood wrt x
    du += g * (2.f - 4.f / (1.f + expf(2.f * u)));                  // squash correction: 2 - 4 sigmoid(-2u)
    const float dmu = g * zz * inv + du;
    const float dstd = g * zz * zz * inv + du * e;
    float dls = -g + dstd * sd;
    if (!(raw >= -20.f && raw <= 2.f)) dls = 0.f;                   // clip_by_value grad
    dhead[r * 2 * A + j] = dmu;
    dhead[r * 2 * A + A + j] = dls;
    dmu_s[j] = dmu;
    dls_s[j] = dls;
  }
  __syncthreads();
  for (int j = tid; j < H; j += blockDim.x) {
    float v = 0.f;
    for (int k = 0; k < A; ++k) v += dmu_s[k] * Wm[j * A + k] + dls_s[k] * Wl[j * A + k];
    dh2p[(int64_t)r * H + j] = h2p[(int64_t)r * H + j] > 0.f ? v : 0.f;
  }
}

// ---- four TF1 Adams (identical step counts -> one lr_t) + Polyak, and grad-norm partials
__global__ __launch_bounds__(256) void sac_adam_kernel(int64_t total, int64_t n_pi, int64_t n_q, float* P, const float* G,
                                                       float* Mm, float* Vv, float* T, float* beta_pow, float lr,
                                                       float tau, float* norm_part, unsigned* ticket, float* logs,
                                                       int64_t* iter) {
  __shared__ float sh[256];
  const float b1 = 0.9f, b2 = 0.999f, eps = 1e-8f;
  const float lr_t = lr * sqrtf(1.f - beta_pow[1]) / (1.f - beta_pow[0]);
  float npi = 0.f, nq = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i <= total; i += (int64_t)gridDim.x * blockDim.x) {
    const float g = G[i];
    if (i < n_pi) npi += g * g;
    else if (i < n_pi + n_q) nq += g * g;
    float m = Mm[i], v = Vv[i];
    m += (g - m) * (1.f - b1);
    v += (g * g - v) * (1.f - b2);
    Mm[i] = m;
    Vv[i] = v;
    const float p = P[i] - (m * lr_t) / (sqrtf(v) + eps);
    P[i] = p;
    if (i < total) T[i] = (1.f - tau) * T[i] + tau * p;             // mopo.py:446-447 (after the updates)
  }
  float nn[2] = {npi, nq};
  block_sums<2>(nn, sh);
  // publish this block's partial norms; the last-arriving block reduces them in block order
  // (agent-scope release -> relaxed ticket -> acquire; cdna_hip_programming.md §6 Guideline 16)
  __shared__ int last;
  if (threadIdx.x == 0) {
    norm_part[blockIdx.x * 2] = nn[0];
    norm_part[blockIdx.x * 2 + 1] = nn[1];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = (t == gridDim.x - 1);
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!last) return;
  float a = 0.f, b = 0.f;
  for (int i = threadIdx.x; i < (int)gridDim.x; i += blockDim.x) {
    a += __hip_atomic_load(norm_part + 2 * i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    b += __hip_atomic_load(norm_part + 2 * i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  float ab[2] = {a, b};
  block_sums<2>(ab, sh);
  if (threadIdx.x == 0) {
    logs[LOG_PI_GNORM] = sqrtf(ab[0]);
    logs[LOG_Q_GNORM] = 0.5f * sqrtf(ab[1]);                          // grads of Q_loss = (l1+l2)/2 wrt q1
    beta_pow[0] *= 0.9f;                                              // TF1 beta power updates (f32)
    beta_pow[1] *= 0.999f;
    *iter += 1;
    *ticket = 0u;                                                     // stream order: next launch sees 0
  }
}


// ---------------------------------------------------------------------------------------------
static GemmProb mk(int M, int N, int K, const float* A, int lda, int ta, const float* B, int ldb, int tb, float* C,
                   int ldc) {
  GemmProb p{};
  p.M = M; p.N = N; p.K = K; p.A = A; p.lda = lda; p.ta = ta; p.B = B; p.ldb = ldb; p.tb = tb; p.C = C; p.ldc = ldc;
  return p;
}

static int launch_group(std::vector<GemmProb> ps, hipStream_t s) {
  GemmGroup g{};
  g.n = (int)ps.size();
  if (g.n > MAXP) return fail("sac: gemm group too large");
  int tot = 0;
  for (int i = 0; i < g.n; ++i) {
    g.p[i] = ps[i];
    g.prefix[i] = tot;
    tot += ceil_div(ps[i].M, 16) * ceil_div(ps[i].N, 16);
  }
  g.prefix[g.n] = tot;
  hipLaunchKernelGGL(gemm_group_kernel, dim3(tot), dim3(256), 0, s, g);
  MOPO_HIP(hipGetLastError());
  return 0;
}

static int sac_step_impl(Sac* h, const mopo_pool_desc* env, const mopo_pool_desc* mod, uint64_t seed,
                         const int64_t* idx_in, const float* eps_in_s, const float* eps_in_n, hipStream_t s) {
  const SacDims& d = h->d;
  const Offs& o = h->o;
  const int n = d.n, O = d.O, A = d.A, H = d.H, W = O + A;
  const float* P = h->P;
  const float* T = h->T;
  float* G = h->G;
  hipLaunchKernelGGL(sac_gather_kernel, dim3(ceil_div(n, GR)), dim3(256), 0, s, *env, *mod, n, d.n_env, O, A, idx_in,
                     h->idx, seed, h->iter, h->sa, h->xpi, h->xn, h->rew, h->term);
  MOPO_HIP(hipGetLastError());
  auto Wq = [&](int qi, int k) { return P + o.q[qi][k]; };
  auto Tq = [&](int qi, int k) { return T + o.q[qi][k]; };
  // ---- forward stage 1-3: pi(s), pi(s'), Q1(s,a), Q2(s,a)
  {
    std::vector<GemmProb> g;
    auto a = mk(n, H, O, h->sa, W, 0, P + o.pW1, H, 0, h->h1[0], H); a.bias = P + o.pb1; a.relu = 1; g.push_back(a);
    auto b = mk(n, H, O, h->xn, W, 0, P + o.pW1, H, 0, h->h1[1], H); b.bias = P + o.pb1; b.relu = 1; g.push_back(b);
    for (int qi = 0; qi < 2; ++qi) {
      auto c = mk(n, H, W, h->sa, W, 0, Wq(qi, 0), H, 0, h->h1[2 + qi], H); c.bias = Wq(qi, 1); c.relu = 1; g.push_back(c);
    }
    if (launch_group(g, s)) return -1;
  }
  {
    std::vector<GemmProb> g;
    for (int i = 0; i < 4; ++i) {
      const float* w2 = i < 2 ? P + o.pW2 : Wq(i - 2, 2);
      const float* b2 = i < 2 ? P + o.pb2 : Wq(i - 2, 3);
      auto a = mk(n, H, H, h->h1[i], H, 0, w2, H, 0, h->h2[i], H); a.bias = b2; a.relu = 1; g.push_back(a);
    }
    if (launch_group(g, s)) return -1;
  }
  {
    std::vector<GemmProb> g;
    for (int i = 0; i < 2; ++i) {
      auto m = mk(n, A, H, h->h2[i], H, 0, P + o.pWm, A, 0, h->out[i], 2 * A); m.bias = P + o.pbm; g.push_back(m);
      auto l = mk(n, A, H, h->h2[i], H, 0, P + o.pWl, A, 0, h->out[i] + A, 2 * A); l.bias = P + o.pbl; g.push_back(l);
    }
    for (int qi = 0; qi < 2; ++qi) {
      auto q = mk(n, 1, H, h->h2[2 + qi], H, 0, Wq(qi, 4), 1, 0, h->out[2 + qi], 1); q.bias = Wq(qi, 5); g.push_back(q);
    }
    if (launch_group(g, s)) return -1;
  }
  hipLaunchKernelGGL(pi_head_fwd_kernel, dim3(ceil_div(2 * n, 256)), dim3(256), 0, s, n, O, A, h->out[0], h->out[1],
                     eps_in_s, eps_in_n, h->eps_s, h->eps_n, seed, h->iter, h->xpi, h->xn, h->logp_s, h->logp_n);
  MOPO_HIP(hipGetLastError());
  // ---- forward stage 4-6: Q1/Q2(s, pi(s)) with main params, Qt1/Qt2(s', pi(s')) with target params
  {
    std::vector<GemmProb> g;
    for (int i = 0; i < 4; ++i) {
      const int qi = i & 1;
      const bool tgt = i >= 2;
      const float* x = tgt ? h->xn : h->xpi;
      auto a = mk(n, H, W, x, W, 0, tgt ? Tq(qi, 0) : Wq(qi, 0), H, 0, h->h1[4 + i], H);
      a.bias = tgt ? Tq(qi, 1) : Wq(qi, 1); a.relu = 1; g.push_back(a);
    }
    if (launch_group(g, s)) return -1;
  }
  {
    std::vector<GemmProb> g;
    for (int i = 0; i < 4; ++i) {
      const int qi = i & 1;
      const bool tgt = i >= 2;
      auto a = mk(n, H, H, h->h1[4 + i], H, 0, tgt ? Tq(qi, 2) : Wq(qi, 2), H, 0, h->h2[4 + i], H);
      a.bias = tgt ? Tq(qi, 3) : Wq(qi, 3); a.relu = 1; g.push_back(a);
    }
    if (launch_group(g, s)) return -1;
  }
  {
    std::vector<GemmProb> g;
    for (int i = 0; i < 4; ++i) {
      const int qi = i & 1;
      const bool tgt = i >= 2;
      auto a = mk(n, 1, H, h->h2[4 + i], H, 0, tgt ? Tq(qi, 4) : Wq(qi, 4), 1, 0, h->out[4 + i], 1);
      a.bias = tgt ? Tq(qi, 5) : Wq(qi, 5); g.push_back(a);
    }
    if (launch_group(g, s)) return -1;
  }
  // ---- losses
  hipLaunchKernelGGL(sac_loss_kernel, dim3(1), dim3(ceil_div(n, 64) * 64), 0, s, n, A, h->gamma, h->rscale, h->tent, h->outp_dev,
                     h->logp_s, h->logp_n, h->rew, h->term, h->out[0], P + o.total, h->dq[0], h->dq[1], h->dq[2],
                     h->dq[3], G + o.total, h->logs);
  MOPO_HIP(hipGetLastError());
  // ---- critic backward.  The 1-wide output layer's backward dh2 = dq (x) W3 * (h2 > 0) is rank-1,
  // so it is never materialised: the consumers below read it as a rank-1 masked operand.
  {
    std::vector<GemmProb> g;
    for (int i = 0; i < 4; ++i) {  // dh1 = dh2 W2^T * (h1 > 0); instances Q1(sa) Q2(sa) Q1(pi) Q2(pi)
      const int qi = i & 1;
      auto a = mk(n, H, H, nullptr, H, 0, Wq(qi, 2), H, 1, h->dh1[i], H); a.mask = h->h1[2 + i]; a.ldm = H;
      a.a_u = h->dq[i]; a.a_v = Wq(qi, 4); a.a_m = h->h2[2 + i]; a.a_ldm = H;
      g.push_back(a);
    }
    for (int qi = 0; qi < 2; ++qi) {  // dW2 = h1^T dh2 (+db2), dW3 = h2^T dq (+db3)
      auto w2 = mk(H, H, n, h->h1[2 + qi], H, 1, nullptr, H, 0, G + o.q[qi][2], H); w2.colsum = G + o.q[qi][3];
      w2.b_u = h->dq[qi]; w2.b_v = Wq(qi, 4); w2.b_m = h->h2[2 + qi]; w2.b_ldm = H;
      g.push_back(w2);
      auto w3 = mk(H, 1, n, h->h2[2 + qi], H, 1, h->dq[qi], 1, 0, G + o.q[qi][4], 1); w3.colsum = G + o.q[qi][5];
      g.push_back(w3);
    }
    if (launch_group(g, s)) return -1;
  }
  {
    std::vector<GemmProb> g;
    g.push_back(mk(n, W, H, h->dh1[2], H, 0, Wq(0, 0), H, 1, h->dx1, W));   // d/dx of Q1(s, pi)
    g.push_back(mk(n, W, H, h->dh1[3], H, 0, Wq(1, 0), H, 1, h->dx2, W));   // d/dx of Q2(s, pi)
    for (int qi = 0; qi < 2; ++qi) {  // dW1 = [s,a]^T dh1 (+db1)
      auto w1 = mk(W, H, n, h->sa, W, 1, h->dh1[qi], H, 0, G + o.q[qi][0], H); w1.colsum = G + o.q[qi][1];
      g.push_back(w1);
    }
    if (launch_group(g, s)) return -1;
  }
  // ---- policy backward
  hipLaunchKernelGGL(pi_head_bwd_kernel, dim3(n), dim3(256), 0, s, n, O, A, H, h->out[0], h->eps_s, h->dx1, h->dx2,
                     P + o.total, P + o.pWm, P + o.pWl, h->h2[0], h->dhead, h->dh2p);
  MOPO_HIP(hipGetLastError());
  {
    std::vector<GemmProb> g;
    auto a = mk(n, H, H, h->dh2p, H, 0, P + o.pW2, H, 1, h->dh1p, H); a.mask = h->h1[0]; a.ldm = H; g.push_back(a);
    auto w2 = mk(H, H, n, h->h1[0], H, 1, h->dh2p, H, 0, G + o.pW2, H); w2.colsum = G + o.pb2; g.push_back(w2);
    auto wm = mk(H, A, n, h->h2[0], H, 1, h->dhead, 2 * A, 0, G + o.pWm, A); wm.colsum = G + o.pbm; g.push_back(wm);
    auto wl = mk(H, A, n, h->h2[0], H, 1, h->dhead + A, 2 * A, 0, G + o.pWl, A); wl.colsum = G + o.pbl; g.push_back(wl);
    if (launch_group(g, s)) return -1;
  }
  {
    std::vector<GemmProb> g;
    auto w1 = mk(O, H, n, h->sa, W, 1, h->dh1p, H, 0, G + o.pW1, H); w1.colsum = G + o.pb1; g.push_back(w1);
    if (launch_group(g, s)) return -1;
  }
  // ---- Adam x4 + Polyak, norms, counters
  hipLaunchKernelGGL(sac_adam_kernel, dim3(h->adam_blocks), dim3(256), 0, s, o.total, o.n_pi, o.n_q, h->P, h->G, h->M,
                     h->V, h->T, h->beta_pow, h->lr, h->tau, h->norm_part, h->ticket, h->logs, h->iter);
  MOPO_HIP(hipGetLastError());
  return 0;
}

}  // namespace mopo

using namespace mopo;

extern "C" int mopo_sac_create(mopo_sac_t* out, int O, int A, int H, int batch, int n_env, const float* h_params,
                               float log_alpha, float lr, float gamma, float tau, float reward_scale,
                               float target_entropy) {
  MOPO_REQUIRE(out && h_params, "mopo_sac_create: NULL argument");
  MOPO_REQUIRE(O >= 1 && A >= 1 && A <= 8 && H >= 1, "mopo_sac_create: bad dims (act_dim <= 8)");
  MOPO_REQUIRE(batch >= 1 && batch <= 1024, "mopo_sac_create: batch must be in [1, 1024]");
  MOPO_REQUIRE(n_env >= 0 && n_env <= batch, "mopo_sac_create: n_env must be in [0, batch]");
  Sac* h = new Sac();
  h->d = SacDims{O, A, H, batch, n_env, 0};
  h->o = make_offs(O, A, H);
  h->d.P = h->o.total;
  h->lr = lr; h->gamma = gamma; h->tau = tau; h->rscale = reward_scale; h->tent = target_entropy;
  const int64_t tot = h->o.total + 1, n = batch, W = O + A;
  h->adam_blocks = (int)std::min<int64_t>(256, (tot + 255) / 256);
  std::vector<std::pair<void**, size_t>> reg;
  auto f = [&](float** p, size_t cnt) { reg.push_back({(void**)p, cnt * 4}); };
  f(&h->P, tot); f(&h->G, tot); f(&h->M, tot); f(&h->V, tot); f(&h->T, tot);
  f(&h->beta_pow, 2); f(&h->logs, LOG_N); f(&h->norm_part, 2 * h->adam_blocks);
  reg.push_back({(void**)&h->iter, 8});
  reg.push_back({(void**)&h->ticket, 4});
  f(&h->sa, n * W); f(&h->xpi, n * W); f(&h->xn, n * W); f(&h->rew, n); f(&h->term, n);
  for (int i = 0; i < 8; ++i) { f(&h->h1[i], n * H); f(&h->h2[i], n * H); f(&h->out[i], n * 2 * A); }
  f(&h->logp_s, n); f(&h->logp_n, n); f(&h->eps_s, n * A); f(&h->eps_n, n * A);
  for (int i = 0; i < 4; ++i) { f(&h->dq[i], n); f(&h->dh2[i], n * H); f(&h->dh1[i], n * H); }
  f(&h->dx1, n * W); f(&h->dx2, n * W); f(&h->dhead, n * 2 * A); f(&h->dh2p, n * H); f(&h->dh1p, n * H);
  reg.push_back({(void**)&h->idx, (size_t)n * 8});
  reg.push_back({(void**)&h->outp_dev, 8 * sizeof(float*)});
  reg.push_back({(void**)&h->dq_dev, 4 * sizeof(float*)});
  reg.push_back({(void**)&h->w3_dev, 4 * sizeof(float*)});
  reg.push_back({(void**)&h->h2q_dev, 4 * sizeof(float*)});
  reg.push_back({(void**)&h->dh2_dev, 4 * sizeof(float*)});
  size_t total = 0;
  for (auto& r : reg) total += (r.second + 255) & ~(size_t)255;
  if (hipMalloc(&h->mem, total) != hipSuccess) { delete h; return fail("mopo_sac_create: out of device memory"); }
  if (hipMemset(h->mem, 0, total) != hipSuccess) { (void)hipFree(h->mem); delete h; return fail("mopo_sac_create: memset"); }
  char* m = (char*)h->mem;
  for (auto& r : reg) { *r.first = m; m += (r.second + 255) & ~(size_t)255; }
  // parameters, target = main (target_init, mopo.py:449-450), log_alpha, beta powers
  std::vector<float> pv(h_params, h_params + h->o.total);
  pv.push_back(log_alpha);
  MOPO_HIP(hipMemcpy(h->P, pv.data(), tot * 4, hipMemcpyHostToDevice));
  MOPO_HIP(hipMemcpy(h->T, pv.data(), tot * 4, hipMemcpyHostToDevice));
  float bp[2] = {0.9f, 0.999f};
  MOPO_HIP(hipMemcpy(h->beta_pow, bp, 8, hipMemcpyHostToDevice));
  float* outs[8];
  for (int i = 0; i < 8; ++i) outs[i] = h->out[i];
  MOPO_HIP(hipMemcpy(h->outp_dev, outs, sizeof(outs), hipMemcpyHostToDevice));
  MOPO_HIP(hipMemcpy(h->dq_dev, h->dq, 4 * sizeof(float*), hipMemcpyHostToDevice));
  float* w3[4] = {h->P + h->o.q[0][4], h->P + h->o.q[1][4], h->P + h->o.q[0][4], h->P + h->o.q[1][4]};
  MOPO_HIP(hipMemcpy(h->w3_dev, w3, sizeof(w3), hipMemcpyHostToDevice));
  float* h2q[4] = {h->h2[2], h->h2[3], h->h2[4], h->h2[5]};
  MOPO_HIP(hipMemcpy(h->h2q_dev, h2q, sizeof(h2q), hipMemcpyHostToDevice));
  MOPO_HIP(hipMemcpy(h->dh2_dev, h->dh2, 4 * sizeof(float*), hipMemcpyHostToDevice));
  *out = reinterpret_cast<mopo_sac_t>(h);
  return 0;
}

extern "C" int mopo_sac_destroy(mopo_sac_t hh) {
  Sac* h = reinterpret_cast<Sac*>(hh);
  if (!h) return 0;
  if (h->gexec) (void)hipGraphExecDestroy(h->gexec);
  if (h->graph) (void)hipGraphDestroy(h->graph);
  if (h->ev_in) (void)hipEventDestroy(h->ev_in);
  if (h->ev_out) (void)hipEventDestroy(h->ev_out);
  if (h->gstream) (void)hipStreamDestroy(h->gstream);
  if (h->mem) (void)hipFree(h->mem);
  delete h;
  return 0;
}

extern "C" int mopo_sac_buffers(mopo_sac_t hh, float** params, float** target, float** adam_m, float** adam_v,
                                float** grads, float** logs, int64_t* n_params) {
  Sac* h = reinterpret_cast<Sac*>(hh);
  MOPO_REQUIRE(h, "mopo_sac_buffers: NULL handle");
  if (params) *params = h->P;
  if (target) *target = h->T;
  if (adam_m) *adam_m = h->M;
  if (adam_v) *adam_v = h->V;
  if (grads) *grads = h->G;
  if (logs) *logs = h->logs;
  if (n_params) *n_params = h->o.total;
  return 0;
}

extern "C" int mopo_sac_copy(mopo_sac_t hh, int which, int to_handle, void* d_buf, int64_t count, void* stream) {
  Sac* h = reinterpret_cast<Sac*>(hh);
  MOPO_REQUIRE(h && d_buf, "mopo_sac_copy: NULL argument");
  float* bufs[6] = {h->P, h->T, h->M, h->V, h->G, h->logs};
  MOPO_REQUIRE(which >= 0 && which < 6, "mopo_sac_copy: which must be in [0, 6)");
  const int64_t cap = which == 5 ? LOG_N : h->o.total + 1;
  MOPO_REQUIRE(count >= 0 && count <= cap, "mopo_sac_copy: count exceeds the buffer");
  if (to_handle)
    MOPO_HIP(hipMemcpyAsync(bufs[which], d_buf, count * 4, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  else
    MOPO_HIP(hipMemcpyAsync(d_buf, bufs[which], count * 4, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return 0;
}

extern "C" int mopo_sac_set_graph(mopo_sac_t hh, int enable) {
  Sac* h = reinterpret_cast<Sac*>(hh);
  MOPO_REQUIRE(h, "mopo_sac_set_graph: NULL handle");
  h->use_graph = enable != 0;
  return 0;
}

static bool same_desc(const mopo_pool_desc& a, const mopo_pool_desc& b) { return std::memcmp(&a, &b, sizeof(a)) == 0; }

extern "C" int mopo_sac_step(mopo_sac_t hh, const mopo_pool_desc* env, const mopo_pool_desc* mod, int n_steps,
                             uint64_t seed, const int64_t* d_idx, const float* d_eps_s, const float* d_eps_n,
                             void* stream) {
  Sac* h = reinterpret_cast<Sac*>(hh);
  MOPO_REQUIRE(h && env && mod, "mopo_sac_step: NULL argument");
  MOPO_REQUIRE(env->d_state && mod->d_state, "mopo_sac_step: pool state required");
  hipStream_t s = (hipStream_t)stream;
  const bool injected = d_idx || d_eps_s || d_eps_n;
  if (injected) {
    MOPO_REQUIRE(n_steps == 1, "mopo_sac_step: injected streams drive exactly one step");
    return sac_step_impl(h, env, mod, seed, d_idx, d_eps_s, d_eps_n, s);
  }
  if (!h->use_graph) {
    for (int i = 0; i < n_steps; ++i)
      if (sac_step_impl(h, env, mod, seed, nullptr, nullptr, nullptr, s)) return -1;
    return 0;
  }
  // graphs are captured and replayed on the handle's own stream (the caller's may be the legacy
  // NULL stream, which cannot capture); event edges order it after / before the caller's work
  if (!h->gstream) {
    MOPO_HIP(hipStreamCreateWithFlags(&h->gstream, hipStreamNonBlocking));
    MOPO_HIP(hipEventCreateWithFlags(&h->ev_in, hipEventDisableTiming));
    MOPO_HIP(hipEventCreateWithFlags(&h->ev_out, hipEventDisableTiming));
  }
  hipStream_t gs = h->gstream;
  if (!h->gexec || !same_desc(h->genv, *env) || !same_desc(h->gmod, *mod) || h->gseed != seed) {
    if (h->gexec) { (void)hipGraphExecDestroy(h->gexec); h->gexec = nullptr; }
    if (h->graph) { (void)hipGraphDestroy(h->graph); h->graph = nullptr; }
    MOPO_HIP(hipStreamBeginCapture(gs, hipStreamCaptureModeThreadLocal));
    const int rc = sac_step_impl(h, env, mod, seed, nullptr, nullptr, nullptr, gs);
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(gs, &g);
    if (rc) { if (g) (void)hipGraphDestroy(g); return -1; }
    if (e != hipSuccess) return fail(std::string("mopo_sac_step: capture failed: ") + hipGetErrorString(e));
    h->graph = g;
    MOPO_HIP(hipGraphInstantiate(&h->gexec, g, nullptr, nullptr, 0));
    h->genv = *env; h->gmod = *mod; h->gseed = seed;
  }
  MOPO_HIP(hipEventRecord(h->ev_in, s));
  MOPO_HIP(hipStreamWaitEvent(gs, h->ev_in, 0));
  for (int i = 0; i < n_steps; ++i) MOPO_HIP(hipGraphLaunch(h->gexec, gs));
  MOPO_HIP(hipEventRecord(h->ev_out, gs));
  MOPO_HIP(hipStreamWaitEvent(s, h->ev_out, 0));
  return 0;
}
