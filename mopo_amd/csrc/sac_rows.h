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
//       (action, log-prob, noise: mopo.py:282-308) -- the action is the critic's layer-1 input
//   B1  sac_dh1_kernel: dh1 = (dq (x) W3 * (h2 > 0)) W2^T * (h1 > 0) for Q1/Q2(s,a) and Q1/Q2(s,pi), the
//       prologue forming each row's dq from the critics' partials (the TD target y, mopo.py:380-404;
//       the min-Q selection, :367-377); the (s, pi) instances emit partials of d(-min Q)/d action
//       (dh1 W1[O:]^T) for the policy backward; one extra block reduces the batch losses (logs,
//       alpha Adam, lr_t, beta powers, step counter: mopo.py:403-443); the policy's row-local
//       backward chain runs in the same launch, each row block's 4 workgroups starting as soon as the
//       8 workgroups that produce its action-gradient partials have published them
//
// Replaces the previous 4-launch chain (forward hidden layers / output layers + head / (s, pi) hidden
// layers / losses + critic output layers) + the critic dh1 launch: 5 -> 3 launches.
#pragma once
#include "gemm_group.h"

namespace mopo {

constexpr int RB_COLS = 64;  // second-layer columns per workgroup (4 waves x 16); OPW: gemm_group.h

struct FwdInst {
  const float* x; int ldx; int kx;   // layer-1 inputs from memory: columns [0, kx) of x[n][ldx]
  int k1;                            // layer-1 input width (F2: kx + A, the action from the head)
  const float* w1; const float* b1;  // [k1][H], [H]
  const float* w2; const float* b2;  // [H][H], [H]
  float* h1; float* h2;              // stored for the backward pass when non-NULL
  const float* wo; const float* wo2; // output layer [H][nout]: columns [0, split) from wo (ld split),
  int nout, split;                   //   [split, nout) from wo2 (ld nout - split)
  float* opart;                      // [ncq][n][OPW] partial dots of the block's 64 outputs
  int head;                          // F2: 0 = pi(s) head (s, pi(s)), 1 = pi(s') head
  // F2 (s, pi) critics: the block's partial of d Q / d action = (W3 * (h2 > 0)) W2^T * (h1 > 0) W1[O:]^T
  // over its 64 columns (dq = 1; the policy-row consumer applies the min-Q selection and -1/n)
  const float* w1a;                  // W1[O:] = the action rows [A][H], or NULL
  float* dapart;                     // [ncq][n][OPW]
  // F1 Q1 / Q2(s, a): the block's partial of dh1 / dq = (W3 * (h2 > 0)) W2^T * (h1 > 0) over its 64
  // columns, all H hidden units ([ncq][n][H]); B1 sums them and scales by the row's dq
  float* upart;
};

struct FwdHead {                     // F2: the squashed-Gaussian head of pi(s) / pi(s') (HeadCtx math)
  const float* opart[2];             // pi(s), pi(s') partials: [ncq][n][OPW], mean j < A, log_std A + j
  const float* bm; const float* bl;  // output biases
  const float* eps_in[2];            // injected noise [n][A] or NULL (Philox)
  float* eps_out[2]; float* head_out[2]; float* logp[2];   // written by the designated blocks
  uint64_t seed; const int64_t* iter;
};

struct FwdArgsR {
  int ninst, n, H, A, ncq, nrb;
  FwdInst in[4];
  FwdHead hd;
  Stamps st;
};

// the head of row r, action j (8 lanes per row; every lane of the 8 calls it): pre-activation
// mean / raw log_std from the partials, then head_fwd_elem's math; returns the action (tanh u)
static __device__ __forceinline__ float rows_head(const FwdHead& h, int nxt, int n, int A, int ncq, int r, int j,
                                                  bool ok, bool store) {
  const bool on = ok && j < A;
  float mu = 0.f, raw = 0.f, z = 0.f;
  if (on) {
    const auto dp = rsrc(h.opart[nxt], (int64_t)ncq * n * OPW);
    float pm[MAX_NCQ], pl[MAX_NCQ];
#pragma unroll
    for (int c = 0; c < MAX_NCQ; ++c) {   // unconditional loads, then the sums in column-block order
      pm[c] = bload(dp, c < ncq ? (c * n + r) * OPW + j : -1);
      pl[c] = bload(dp, c < ncq ? (c * n + r) * OPW + A + j : -1);
    }
    mu = h.bm[j];
    raw = h.bl[j];
#pragma unroll
    for (int c = 0; c < MAX_NCQ; ++c) {
      mu += pm[c];
      raw += pl[c];
    }
    const float* ein = h.eps_in[nxt];
    if (ein) {
      z = ein[r * A + j];
    } else {
      const int64_t it = *h.iter;
      const int blk = j >> 2;
      u32x4 c{(uint32_t)r | ((uint32_t)nxt << 31), (uint32_t)it ^ ((uint32_t)blk << 24), (uint32_t)((uint64_t)it >> 32),
              RNG_SAC + 16};
      u32x4 q = philox(c, (uint32_t)h.seed, (uint32_t)(h.seed >> 32));
      float z0, z1;
      if (j & 2) box_muller(q.z, q.w, z0, z1);
      else box_muller(q.x, q.y, z0, z1);
      z = (j & 1) ? z1 : z0;
    }
  }
  float v = 0.f, act = 0.f;
  if (on) {
    const float ls = fminf(fmaxf(raw, -20.f), 2.f);               // mopo.py:304
    const float sd = expf(ls);
    const float u = mu + z * sd;                                    // mopo.py:306
    const float zz = (u - mu) / (sd + 1e-8f);
    v = -0.5f * (zz * zz + 2.f * ls + 1.8378770664093453f)          // gaussian_likelihood (:282-284)
        - 2.f * (0.6931471805599453f - u - softplusf(-2.f * u));    // squash correction (:292)
    act = tanhf(u);
    if (store) {
      h.eps_out[nxt][r * A + j] = z;
      h.head_out[nxt][r * 2 * A + j] = mu;
      h.head_out[nxt][r * 2 * A + A + j] = raw;
    }
  }
  v += __shfl_xor(v, 1);
  v += __shfl_xor(v, 2);
  v += __shfl_xor(v, 4);
  if (store && ok && j == 0) h.logp[nxt][r] = v;
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
// MFMAs; row stride COLS + 4); rows r < n and j < nout are stored to part[row][OPW]
template <int COLS, bool SC1 = false>
static __device__ __forceinline__ void rows_partial_out(const float* T, const float* WT, int li, int lk, int i0, int n,
                                                        int nout, float* part) {
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
      if constexpr (SC1) __hip_atomic_store(part + (int64_t)orow * OPW + li, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else part[(int64_t)orow * OPW + li] = v;
    }
  }
}

// Grid (column block, row block, instance): linear block id cq + ncq (rb + nrb ii).  H <= GKC, H % 16 == 0.
template <bool HEAD>
static __global__ __launch_bounds__(256, 2) void sac_fwd_kernel(const FwdArgsR a) {
  __shared__ __attribute__((aligned(16))) float As[RB_LDS_A];
  __shared__ __attribute__((aligned(16))) float Ts[RB_LDS_T];
  __shared__ __attribute__((aligned(16))) float Wo[RB_LDS_T];
  __shared__ float act_s[16][8];
  __shared__ float da_s[4][16][9];
  stamp(a.st, 0);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // grid (ncq, nrb, ninst): the indices are SGPRs, so the instance's fields come from the kernel
  // arguments by scalar loads (a divided linear index made them VGPRs: every buffer descriptor built
  // from them then needed a waterfall loop)
  const int ii = blockIdx.z, rb = blockIdx.y, cq = blockIdx.x;
  const FwdInst p = pick4(a.in, ii);
  const int n = a.n, H = a.H, A = a.A;
  const int i0 = rb * 16, c0 = cq * RB_COLS, jw = c0 + w * 16;
  // ---- 1. every global operand, issued up front: this wave's W2 operand straight into MFMA registers
  //         (lane (li, lk): W2[64 lk + 4 s + u][jw + li]; 16 lanes read 64 contiguous bytes of a row),
  //         the output-layer columns of the block's 64 rows, layer 1
  const int li = lane & 15, lk = lane >> 4;
  f32x4 bp[16];
  {
    const auto dbw = rsrc(p.w2, (int64_t)H * H);
    const bool con = jw + li < H;
#pragma unroll
    for (int s2 = 0; s2 < 16; ++s2)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = 64 * lk + 4 * s2 + u;
        bp[s2][u] = bload(dbw, (con && k < H) ? k * H + jw + li : -1);
      }
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
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const int j = 4 * s + q4;
        wa[kt][s] = bload(dw, (j < k1 && k < H) ? j * H + k : -1);
      }
      bv[kt] = bload(db, k < H ? k : -1);
    }
  }
  float b2v = bload(rsrc(p.b2, H), jw + (lane & 15) < H ? jw + (lane & 15) : -1);
  // ---- 2. F2: the policy head of the block's 16 rows (its action feeds layer 1)
  if (HEAD) {
    if (tid < 128) {
      const int hr = tid >> 3, hj = tid & 7, hrow = i0 + hr;
      const bool store = cq == 0 && (ii == 0 || ii == 2);  // Q1(s,pi) / Qt1(s',pi') blocks publish the head
      act_s[hr][hj] = rows_head(a.hd, p.head, n, A, a.ncq, hrow, hj, hrow < n, store);
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
      if (i0 + rr < n) p.h1[(int64_t)(i0 + rr) * H + tid] = As[rr * RB_LD + tid];
  }
  // ---- 4. layer 2: the wave's 16 x 16 tile over the whole K
  f32x4 acc[4];
  rows_contract(As, bp, li, lk, acc);
  stamp(a.st, 3);
  // ---- 5. bias + relu (D: column li, rows 4 lk + rr); h2 store; the tile into LDS
  const int col = jw + li;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int orow = i0 + 4 * lk + rr;
    const float v = (col < H && orow < n) ? fmaxf(acc[0][rr] + acc[1][rr] + acc[2][rr] + acc[3][rr] + b2v, 0.f) : 0.f;
    if (p.h2 && orow < n && col < H) p.h2[(int64_t)orow * H + col] = v;
    Ts[(4 * lk + rr) * RB_TLD + w * 16 + li] = v;
  }
  lds_barrier();
  // ---- 6. partial output dots of the block's 64 columns (wave 0, MFMA)
  if (w == 0) rows_partial_out<RB_COLS>(Ts, Wo, li, lk, i0, n, p.nout, p.opart + (int64_t)cq * n * OPW);
  // ---- 7. a critic's backward share of the block (dq = 1): wave w forms dh1 rows k in [64 w, 64 w + 64)
  //         of D(k, r) = sum_c W2[k][c0 + c] G(r, c), G = W3[c0 + c] (h2 > 0) (K = the block's 64
  //         columns), masked by h1 > 0.  F2, Q1 / Q2 at (s, pi(s)): then its partial of the action
  //         gradient sum_k dh1(r, k) W1[O + a][k], so the policy's backward needs no critic backward at
  //         (s, pi) in the next launch.  F1, Q1 / Q2(s, a): the masked tile itself (upart), which B1
  //         sums over the column blocks and scales by the row's dq (no W2 operand burst there).
  {
    if (p.dapart || p.upart) {
      const int kw = 64 * w;
      // A(m = k, K = c): lane (li, lk) holds W2[kw + 16 t + li][c0 + 16 s + 4 lk + u] (one b128 per (t, s))
      const auto dw2 = rsrc(p.w2, (int64_t)H * H);
      f32x4 wa2[4][4];
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
          const int k = kw + 16 * t + li, c = c0 + 16 * s2 + 4 * lk;
          wa2[t][s2] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                     dw2, ((k < H && c < H) ? k * H + c : -4) * 4, 0, 0));
        }
      // B(K = k, n = a) of the action contraction: W1[O + a = li][kw + 16 t + 4 lk .. + 3]
      const auto dwa = rsrc(p.w1a, p.w1a ? (int64_t)A * H : 0);
      f32x4 wb1[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int k = kw + 16 * t + 4 * lk;
        wb1[t] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                               dwa, ((p.w1a && li < A && k < H) ? li * H + k : -4) * 4, 0, 0));
      }
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
        const int k0 = kw + 16 * t + 4 * lk;
        if (p.upart && i0 + li < n && k0 < H)                // one b128 per lane: row li, k0 .. k0 + 3
          *reinterpret_cast<f32x4*>(p.upart + ((int64_t)cq * n + i0 + li) * H + k0) = um;
      }
      if (!p.dapart) goto done7;
#pragma unroll
      for (int i = 0; i < 4; ++i)                            // D: r = 4 lk + i, a = li
        if (li < 8) da_s[w][4 * lk + i][li] = da[i];
      lds_barrier();
      if (tid < 128) {                                       // waves' partials in wave order
        const int rr = tid >> 3, aa = tid & 7, orow = i0 + rr;
        const float v = da_s[0][rr][aa] + da_s[1][rr][aa] + da_s[2][rr][aa] + da_s[3][rr][aa];
        if (aa < A && orow < n) p.dapart[((int64_t)cq * n + orow) * OPW + aa] = v;
      }
    }
  }
done7:
  stamp(a.st, 4);
}

// ---- B1 -----------------------------------------------------------------------------------------
// The critics' per-row losses from the forward partials (mopo.py:361-404): q = sum of the column-block
// partials + b3, in column-block order.  Instances of the partial arrays: 0 Q1(s,a) 1 Q2(s,a)
// 2 Q1(s,pi) 3 Q2(s,pi) 4 Qt1(s',pi') 5 Qt2(s',pi').
struct LossRows {
  const float* qpart[6];             // [ncq][n][OPW] (element 0)
  const float* b3[6];
  const float* logp_s; const float* logp_n; const float* head_s; const float* rew; const float* term;
  const float* log_alpha;
  float gamma, rscale;
};

struct RowQ { float q[6]; float y, alpha; };

static __device__ __forceinline__ RowQ row_losses(const LossRows& L, int n, int ncq, int r) {
  RowQ o;
  float pv[6][MAX_NCQ];
#pragma unroll
  for (int i = 0; i < 6; ++i) {           // unconditional loads, then the sums in column-block order
    const auto dp = rsrc(L.qpart[i], (int64_t)ncq * n * OPW);
#pragma unroll
    for (int c = 0; c < MAX_NCQ; ++c) pv[i][c] = bload(dp, c < ncq ? (c * n + r) * OPW : -1);
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    float s = *L.b3[i];
#pragma unroll
    for (int c = 0; c < MAX_NCQ; ++c) s += pv[i][c];
    o.q[i] = s;
  }
  o.alpha = expf(*L.log_alpha);                                       // mopo.py:361
  const float qt = fminf(o.q[4], o.q[5]);                             // mopo.py:368
  o.y = L.rscale * L.rew[r] + L.gamma * ((1.f - L.term[r]) * (qt - o.alpha * L.logp_n[r]));  // :380-386
  return o;
}

struct Dh1Inst {
  const float* upart;                // F1's dh1 / dq partials [ncq][n][H] (then only dq, dh1 are formed here)
  const float* h1; const float* h2; const float* w2; const float* w3;
  int kind;                          // dq of the row: 0 (q1 - y) / n, 1 (q2 - y) / n, 2 min-select Q1, 3 Q2
  float* dh1;                        // stored when non-NULL
  float* dq;                         // stored by the column-block-0 workgroups when non-NULL
  const float* w1a;                  // (s, pi) instances: W1[O:] = the action rows [A][H]; NULL otherwise
  float* dapart;                     // [ncq1][n][OPW]: partial dh1 W1[O:]^T of the block's 128 columns
};

constexpr int B1_WAVES = 8, B1_COLS = 16 * B1_WAVES;   // B1 workgroups: 16 rows x 128 columns
constexpr int B1_TLD = B1_COLS + 4;

struct Dh1Args {
  int ninst, n, H, A;
  int ncq;                           // column blocks of the forward partials (64 wide)
  int ncq1;                          // B1's column blocks (128 wide): its action-gradient partials
  int nrb;
  Dh1Inst in[4];
  LossRows L;
  // the loss tail (last block): batch means -> logs, the alpha gradient + Adam, lr_t, beta powers, step
  AdamCtx ad;
  float tent, lr;
  float* logs; float* beta_pow; int64_t* iter;
  const int64_t* tctl;               // target schedule {base, n_train_repeat, interval} (sac.hip mopo_sac_set_target_schedule)
  // the policy's row-local backward chain (gemm_group.h policy_rows_block) as blocks z = ninst + 1 of
  // this launch: block (cq, rb) waits until the 2 ncq1 (s, pi) workgroups of row block rb published
  // their action-gradient partials (agent-scope counter rb_ready[rb], zeroed by the step's last launch)
  PolicyRows pr;
  int* rb_ready;
  Stamps st;
};

constexpr int PR_SPIN_LIMIT = 1 << 22;   // ~ 0.2 s of polling: a hang guard, never reached in a sane launch

// the extra block: per-row loss terms of all n rows (thread t: rows t, t + 256, ...), block sums in a
// fixed order (deterministic), then thread 0 applies the batch-level updates (loss_tail_block's tail)
static __device__ __forceinline__ void loss_tail_rows(const Dh1Args& a, float* sh) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, nw = blockDim.x >> 6;
  const int n = a.n, A = a.A;
  // the alpha Adam state and the beta powers, fetched up front (thread 0; used after the reduction)
  AdamIn al{0.f, 0.f, 0.f, 0.f};
  float b1p = 0.f, b2p = 0.f;
  if (tid == 0) {
    al = adam_load(a.ad, a.ad.total);                                 // log_alpha = the last parameter
    b1p = a.beta_pow[0];
    b2p = a.beta_pow[1];
  }
  float red[7] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int r = tid; r < n; r += blockDim.x) {
    const RowQ o = row_losses(a.L, n, a.ncq, r);
    const float q1 = o.q[0], q2 = o.q[1], q1p = o.q[2], q2p = o.q[3];
    const float lps = a.L.logp_s[r];
    float ent = 0.f;                                                  // pi_entropy terms (mopo.py:341)
    for (int j = 0; j < A; ++j) {
      const float ls = fminf(fmaxf(a.L.head_s[(int64_t)r * 2 * A + A + j], -20.f), 2.f);
      ent += logf(expf(ls) + 1e-8f) + 0.5f * logf(2.f * 3.14159265358979f * 2.718281828459045f);
    }
    red[0] += (q1 - o.y) * (q1 - o.y); red[1] += (q2 - o.y) * (q2 - o.y); red[2] += q1; red[3] += q2;
    red[4] += lps; red[5] += ent; red[6] += o.alpha * lps - fminf(q1p, q2p);
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
  const AdamCtx& ad = a.ad;
  const float fn = (float)n;
  const float l1 = red[0] / fn * 0.5f, l2 = red[1] / fn * 0.5f;       // mopo.py:403-404
  const float m1 = red[2] / fn, m2 = red[3] / fn, mlp = red[4] / fn, ment = red[5] / fn;
  const float pil = red[6] / fn;                                      // mopo.py:371-377
  const float ga = -(mlp + a.tent);                                   // d/dlog_alpha of -mean(la*(logp+H))
  const_cast<float*>(ad.G)[ad.total] = ga;
  float* logs = a.logs;
  logs[LOG_Q1_LOSS] = l1; logs[LOG_Q2_LOSS] = l2; logs[LOG_Q1] = m1; logs[LOG_Q2] = m2;
  logs[LOG_ALPHA] = expf(al.p); logs[LOG_ENTROPY] = ment; logs[LOG_LOGP] = mlp; logs[LOG_PI_LOSS] = pil;
  const float lr_t = a.lr * sqrtf(1.f - b2p) / (1.f - b1p);           // TF1 Adam step size
  a.beta_pow[2] = lr_t;
  a.beta_pow[0] = b1p * 0.9f;
  a.beta_pow[1] = b2p * 0.999f;
  {  // the step's timestep (mopo.py:780-799: n_train_repeat steps share one) and its target-update flag
    const int64_t rep = a.tctl[1] > 0 ? a.tctl[1] : 1, every = a.tctl[2] > 0 ? a.tctl[2] : 1;
    const int64_t ts = (*a.iter - a.tctl[0]) / rep;
    a.beta_pow[3] = ((ts % every) + every) % every == 0 ? 1.f : 0.f;
  }
  *a.iter += 1;
  adam_apply(ad, ad.total, ga, al, lr_t);
}

// Grid (column block, row block, 2 + ninst): z = 0, block (0, 0): the loss tail; z = 1 .. ninst: the
// instances; z = ninst + 1: the policy-row blocks (they wait on the (s, pi) instances' partials).
// B1 runs 8-wave workgroups (16 rows x 128 columns), one per CU: the 1 + 4 x 32 + 32 busy workgroups
// of a batch-256 step then all start at once on their own CUs -- the policy-row blocks prefetch their
// operands beside the producers instead of queueing for a CU or sharing one with them.
static __global__ __launch_bounds__(B1_WAVES * 64, 1) void sac_dh1_kernel(const Dh1Args a) {
  __shared__ __attribute__((aligned(16))) float As[RB_LDS_A];
  __shared__ __attribute__((aligned(16))) float Ts[16 * B1_TLD];
  __shared__ __attribute__((aligned(16))) float Wo[16 * B1_TLD];
  __shared__ float dqs[16];
  stamp(a.st, 0);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // grid (ncq1, nrb, ninst + 2): SGPR indices (see sac_fwd_kernel); z = 0 holds the loss tail (block
  // (0, 0, 0), dispatched first: its ~6 us chain runs beside the tiles instead of after them), the
  // instances are z = 1 .. ninst, the policy-row blocks z = ninst + 1
  if (blockIdx.z == 0) {
    if (blockIdx.x == 0 && blockIdx.y == 0) {
      loss_tail_rows(a, Ts);
      stamp(a.st, 4);
    }
    return;
  }
  if ((int)blockIdx.z > a.ninst) {    // the policy-row blocks
    const int rb = blockIdx.y, cq = blockIdx.x;
    if (a.pr.qpart[0]) {                // the action-gradient partials come from F2 (the previous launch)
      policy_rows_block<false, true>(a.pr, rb * a.ncq1 + cq, As, Ts, [] {}, a.st);
      stamp(a.st, 4);
      return;
    }
    const int need = 2 * a.ncq1;
    bool late = false;
    auto wait = [&] {
      if (threadIdx.x == 0) {
        int spins = 0;
        while (__hip_atomic_load(a.rb_ready + rb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
          __builtin_amdgcn_s_sleep(2);
          if (++spins > PR_SPIN_LIMIT) { late = true; break; }
        }
      }
      __syncthreads();   // a full fence: the partials' agent-scope loads must not move above it
    };
    policy_rows_block<true>(a.pr, rb * a.ncq1 + cq, As, Ts, wait, a.st);
    if (late) a.logs[LOG_HANDOFF] = 1.f;   // hand-off timed out: sac.py raises on the flag
    stamp(a.st, 4);
    return;
  }
  const int ii = blockIdx.z - 1, rb = blockIdx.y, cq = blockIdx.x;
  const Dh1Inst p = pick4(a.in, ii);
  const int n = a.n, H = a.H, A = a.A;
  const int i0 = rb * 16, c0 = cq * B1_COLS, jw = c0 + w * 16;
  const int li = lane & 15, lk = lane >> 4;
  if (p.upart) {
    // dh1 = dq * sum of F1's column-block partials (already masked by h1 > 0), in column-block order:
    // thread t owns row t / 32, columns c0 + 4 (t % 32) .. + 3 of the block (one b128 per partial)
    const int rr = tid >> 5, kq = c0 + 4 * (tid & 31), orow = i0 + rr;
    const auto du = rsrc(p.upart, (int64_t)a.ncq * n * H);
    f32x4 up[MAX_NCQ];
#pragma unroll
    for (int c = 0; c < MAX_NCQ; ++c)
      up[c] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                            du, ((c < a.ncq && orow < n && kq < H) ? (c * n + orow) * H + kq : -4) * 4, 0, 0));
    if (tid < 16) {
      const int r2 = i0 + tid;
      float dq = 0.f;
      if (r2 < n) {
        const RowQ o = row_losses(a.L, n, a.ncq, r2);
        dq = (p.kind == 0 ? o.q[0] : o.q[1]) - o.y;
        dq *= 1.f / (float)n;
        if (cq == 0 && p.dq) p.dq[r2] = dq;
      }
      dqs[tid] = dq;
    }
    lds_barrier();
    if (orow < n && kq < H) {
      f32x4 v = up[0];
#pragma unroll
      for (int c = 1; c < MAX_NCQ; ++c) v += up[c];
      *reinterpret_cast<f32x4*>(p.dh1 + (int64_t)orow * H + kq) = v * dqs[rr];
    }
    stamp(a.st, 4);
    return;
  }
  // ---- 1. operands up front: this wave's W2^T operand straight into MFMA registers (B(m, c) = W2[c][m]:
  //         lane (li, lk) holds W2[jw + li][64 lk + 4 s .. + 3]), the A slab's h2 rows and W3 (waves
  //         0-3), the h1 mask of this lane's outputs, W1[O:] columns of the block (the (s, pi) instances)
  const auto dw2 = rsrc(p.w2, (int64_t)H * H);
  f32x4 bp[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int m = 64 * lk + 4 * i, c = jw + li;
    bp[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                          dw2, ((m < H && c < H) ? c * H + m : -4) * 4, 0, 0));
  }
  // A slab: thread (m-quad tid % 64, rows 4 (tid / 64) .. + 3), waves 0-3
  const bool slab = w < 4;
  const int am = 4 * (tid & 63), ar = 4 * (w & 3);
  const auto dh2 = rsrc(p.h2, (int64_t)n * H);
  f32x4 h2v[4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
    h2v[q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                           dh2, ((slab && am < H && i0 + ar + q < n) ? (i0 + ar + q) * H + am : -4) * 4, 0, 0));
  const f32x4 w3v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                  rsrc(p.w3, H), ((slab && am < H) ? am : -4) * 4, 0, 0));
  float m1[4];
  {
    const auto dm1 = rsrc(p.h1, (int64_t)n * H);
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) m1[rr] = bload(dm1, (jw + li < H && i0 + 4 * lk + rr < n) ? (i0 + 4 * lk + rr) * H + jw + li : -1);
  }
  float wov[4] = {0.f, 0.f, 0.f, 0.f};
  if (p.w1a) {
    const auto d1 = rsrc(p.w1a, (int64_t)A * H);
#pragma unroll
    for (int q = 0; q < 4; ++q) {     // Wo[c][j] = W1[O + j][c0 + c]: element e = c * 16 + j
      const int e = tid + B1_WAVES * 64 * q, c = c0 + (e >> 4), j = e & 15;
      wov[q] = bload(d1, (c < H && j < A) ? j * H + c : -1);
    }
  }
  // ---- 2. dq of the block's 16 rows (one lane per row)
  if (tid < 16) {
    const int rr = i0 + tid;
    float dq = 0.f;
    if (rr < n) {
      const RowQ o = row_losses(a.L, n, a.ncq, rr);
      const float inv_n = 1.f / (float)n;
      const bool sel1 = o.q[2] <= o.q[3];                             // tf.minimum grad -> x where x <= y
      dq = p.kind == 0 ? (o.q[0] - o.y) * inv_n : p.kind == 1 ? (o.q[1] - o.y) * inv_n
         : p.kind == 2 ? (sel1 ? -inv_n : 0.f) : (sel1 ? 0.f : -inv_n);
      if (cq == 0 && p.dq) p.dq[rr] = dq;
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
#pragma unroll
  for (int q = 0; q < 4; ++q) {     // Wo[j][c]
    const int e = tid + B1_WAVES * 64 * q;
    Wo[(e & 15) * B1_TLD + (e >> 4)] = wov[q];
  }
  lds_barrier();
  stamp(a.st, 2);
  // ---- 4. dh1 tile of the wave: 16 rows x 16 columns over the whole K
  f32x4 acc[4];
  rows_contract(As, bp, li, lk, acc);
  stamp(a.st, 3);
  // ---- 5. relu mask from h1; store; the (s, pi) instances' action-gradient partials
  const int col = jw + li;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int orow = i0 + 4 * lk + rr;
    const float v = (col < H && orow < n && m1[rr] > 0.f) ? acc[0][rr] + acc[1][rr] + acc[2][rr] + acc[3][rr] : 0.f;
    if (p.dh1 && orow < n && col < H) p.dh1[(int64_t)orow * H + col] = v;
    Ts[(4 * lk + rr) * B1_TLD + w * 16 + li] = v;
  }
  if (p.w1a) {
    lds_barrier();
    if (w == 0) {
      // the policy-row blocks of this launch read these partials: agent-scope (sc1) stores, the wave's
      // vmcnt(0), then one lane's agent-scope counter add (MI355X_MICROARCH.md hand-off, row 1)
      rows_partial_out<B1_COLS, true>(Ts, Wo, li, lk, i0, n, A, p.dapart + (int64_t)cq * n * OPW);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_fetch_add(a.rb_ready + rb, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  stamp(a.st, 4);
}

}  // namespace mopo
