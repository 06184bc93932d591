// Row-block kernels of the ensemble training step (bnn_train.hip): one minibatch step in three launches
// instead of twelve.
//
//   train_fwd_rows_kernel, grid (row blocks, members): the minibatch gather (bootstrap rows, scaler:
//     utils.py:96), the four swish layers and the fused mean / log-var head of the member for its 16
//     rows (fc.py:84-106; pre-activations Z and activations H stored for the backward), the output
//     gradient of the Gaussian NLL through the soft log-var bounds (bnn.py:241-249, 669-701) and the
//     block's partial sums of the max/min log-var gradients and of the loss
//   train_bwd_rows_kernel, grid (row blocks, members + 1): row block (0, 0) reduces those partials in
//     a fixed order and applies the batch-level updates (the 0.01 (sum maxlv - sum minlv) terms, their
//     Adam, this step's lr_t, the TF1 beta powers, the minibatch counter); the others run the
//     activation-gradient chain dZ_{l-1} = (dY_l W_l^T) * swish'(Z_{l-1}), l = 4 .. 1
//   one gemm_group launch (bnn_train.hip): every weight gradient X_in^T dY (+ bias column sums, weight
//     decay, TF1 Adam in the epilogue) as 5 batched problems, one per layer, the members as the batch
//
// Every row-local quantity stays in its workgroup: the layer's 16 x K input sits in LDS, each of the 8
// waves contracts 2 output tiles of 16 columns over the whole K on v_mfma_f32_16x16x4_f32
// (exact f32 products, f32 accumulation), its weight columns streamed from L2 straight into MFMA B
// registers two k-groups ahead (b64 / b128 loads), and the layer's output goes back to LDS for the next layer.
// A member's row blocks share one XCD (tr_block), so its weights are fetched into one L2.
// Requires H, IN <= 256, 2D <= 256, H and 2D multiples of 4 (bnn_train.hip use_rows).
#pragma once
#include <type_traits>

#include "gemm_group.h"

namespace mopo {

constexpr int TR_NHID = 4;
#ifndef TR_LD_CFG
#define TR_LD_CFG 260
#endif
constexpr int TR_LD = TR_LD_CFG;   // LDS row stride (floats) of a 16-row activation block: K <= 256 (+4: b128 reads conflict-free)

struct TrainRows {
  int E, M, IN, H, D, nrb;
  // gather: row = rows[e * stride + (*bstep) * batch + r] (rows == NULL: r)
  const float* inputs; const float* targets; const int32_t* rows; int64_t stride; const int* bstep; int batch;
  const float* mu; const float* sigma;
  const float* P;                    // this step's parameters (training layout, bnn_train.hip)
  int64_t W[TR_NHID + 1], b[TR_NHID + 1], mx, mn;
  float* X; float* T; float* Z[TR_NHID]; float* Hh[TR_NHID]; float* OUT; float* dOUT; float* dZ[TR_NHID];
  // staged (graph-captured full minibatches): this step's rows are already gathered in X / T (by the
  // previous step, or the epoch's first gather), and the block gathers the NEXT step's rows into Xn / Tn,
  // its loads issued at the start and stored at the end (the gather's dependent chain off the step's path)
  int staged; float* Xn; float* Tn;
  float* lpart;                      // [E][nrb][D][4]: d loss / d maxlv, d loss / d minlv, loss (per row block)
  // the batch-level tail (train_bwd_rows_kernel's block (0, 0))
  float* logs; float* beta_pow; int* bstep_inc; float lr; float* G; AdamCtx ad;
};

static __device__ __forceinline__ f32x4 bload4(__amdgpu_buffer_rsrc_t d, int idx) {   // idx < 0: zeros
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(d, idx * 4, 0, 0));
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

static __device__ __forceinline__ f32x2 bload2(__amdgpu_buffer_rsrc_t d, int idx) {   // idx < 0: zeros
  return __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(d, idx * 4, 0, 0));
}

// W, K, N, ldw are wave-uniform but computed from a runtime layer index: forced into SGPRs here, since a
// buffer descriptor the compiler believes divergent is wrapped in a readfirstlane waterfall loop around
// every load (measured: the step's forward kernel 2x slower)
static __device__ __forceinline__ const float* uniform_ptr(const float* p) {
  const uint64_t v = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (const float*)(((uint64_t)hi << 32) | lo);
}

// Workgroups of TR_WAVES waves: wave w owns column block cb = w % 4 (64 columns) and TW = 16 / TR_WAVES
// of its 4 tiles (two waves per SIMD at 8: one wave's memory waits overlap the other's MFMAs; 16: one
// tile per wave, four waves per SIMD -- measured 10.07k -> 8.5k grad-steps/s, same-box A/B).
#ifndef TR_WAVES_CFG
#define TR_WAVES_CFG 8
#endif
constexpr int TR_WAVES = TR_WAVES_CFG, TR_TW = 16 / TR_WAVES;

// acc[q] = A[16 x K] x B over the whole K for tiles q < TW of the wave: tile q's column li is column
// c + q, c = 64 cb + 4 li + TW (w / 4), so a lane's B values of one k are one b64 / b128 load (KT = false)
// and its outputs of one row one b64 / b128 store.  A in LDS (row stride TR_LD, zero past K up to the
// next multiple of 16); B(k, c) = W[k * ldw + c] (KT = false) or W[c * ldw + k] (KT = true), zero outside
// k < K, c < N (N and, for KT, K multiples of 4).  Lane (li, lk) contracts k = 16 grp + 4 lk + u (one
// ds_read_b128 of A per k-group).  G = ceil(K / 16) at compile time: straight-line code with the loads
// two k-groups ahead (a runtime k-group loop made the compiler wait for all but 2 of the prefetched
// loads at its header).
#ifndef TR_PF_CFG
#define TR_PF_CFG 2
#endif
// k-groups of B loaded ahead of their MFMAs (4 / 7: 11.52k -> 11.41k / 11.10k grad-steps/s, same-box A/B)
constexpr int TR_PF = TR_PF_CFG;
#ifndef TR_PF_B_CFG
#define TR_PF_B_CFG TR_PF_CFG   // the fused rows kernel's backward (transposed weight reads)
#endif
constexpr int TR_PF_B = TR_PF_B_CFG, TR_PFM = TR_PF > TR_PF_B ? TR_PF : TR_PF_B;
template <bool KT, int G, int TW>
static __device__ __forceinline__ void rows_gemm(const float* As, const float* Wv, int Kv, int Nv, int ldwv, int c,
                                                 int lane, f32x4 (&acc)[TW]) {
  const float* W = uniform_ptr(Wv);
  const int K = __builtin_amdgcn_readfirstlane(Kv), N = __builtin_amdgcn_readfirstlane(Nv);
  const int ldw = __builtin_amdgcn_readfirstlane(ldwv);
  const int li = lane & 15, lk = lane >> 4;
  const auto d = rsrc(W, KT ? (int64_t)(N - 1) * ldw + K : (int64_t)(K - 1) * ldw + N);
#pragma unroll
  for (int q = 0; q < TW; ++q) acc[q] = zero4();
  if (__builtin_amdgcn_readfirstlane(c - 4 * li) >= N) return;   // no columns for this wave (wave-uniform)
  auto ld = [&](int grp, float (&bv)[4][TW]) {
    const int k0 = 16 * grp + 4 * lk;
    if constexpr (KT) {
#pragma unroll
      for (int q = 0; q < TW; ++q) {                    // column c + q, k0 .. k0 + 3
        const f32x4 v = bload4(d, ((c + q < N) & (k0 < K)) ? (c + q) * ldw + k0 : -1);
#pragma unroll
        for (int u = 0; u < 4; ++u) bv[u][q] = v[u];
      }
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) {                     // row k0 + u, columns c .. c + TW - 1
        const int idx = ((c < N) & (k0 + u < K)) ? (k0 + u) * ldw + c : -1;
        if constexpr (TW == 4) {
          const f32x4 v = bload4(d, idx);
#pragma unroll
          for (int q = 0; q < 4; ++q) bv[u][q] = v[q];
        } else if constexpr (TW == 2) {
          const f32x2 v = bload2(d, idx);
          bv[u][0] = v[0];
          bv[u][1] = v[1];
        } else {
          bv[u][0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(d, idx * 4, 0, 0));
        }
      }
    }
  };
  auto mm = [&](int grp, const float (&bv)[4][TW]) {
    const f32x4 a4 = ld4(As + li * TR_LD + 16 * grp + 4 * lk);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int q = 0; q < TW; ++q) acc[q] = mfma4(a4[u], bv[u][q], acc[q]);
  };
  float bq[G + TR_PF][4][TW];
#pragma unroll
  for (int grp = 0; grp < TR_PF && grp < G; ++grp) ld(grp, bq[grp]);
#pragma unroll
  for (int grp = 0; grp < G; ++grp) {
    if (grp + TR_PF < G) ld(grp + TR_PF, bq[grp + TR_PF]);   // TR_PF k-groups ahead
    // keep them there: left alone the scheduler sinks each load to just before its first use, leaving
    // one or two in flight
    __builtin_amdgcn_sched_barrier(0);
    mm(grp, bq[grp]);
  }
}

// rows_gemm with the layer's first TR_PF k-groups of B loaded ahead (rows_pre), by the fused kernel across
// the previous layer's epilogue and barrier: the weights do not depend on the activations, so a layer
// no longer starts on an exposed L2 round trip
#ifndef TR_LDOFF
#define TR_LDOFF 1   // rows_ld: plain offsets, bounds by the buffer range (0: per-load masks, measured slower)
#endif
struct RowsW {
  __amdgpu_buffer_rsrc_t d;
  int K, N, ldw;
};
template <bool KT>
static __device__ __forceinline__ RowsW rows_w(const float* Wv, int Kv, int Nv, int ldwv) {
  const float* W = uniform_ptr(Wv);
  RowsW r;
  r.K = __builtin_amdgcn_readfirstlane(Kv);
  r.N = __builtin_amdgcn_readfirstlane(Nv);
  r.ldw = __builtin_amdgcn_readfirstlane(ldwv);
  r.d = rsrc(W, KT ? (int64_t)(r.N - 1) * r.ldw + r.K : (int64_t)(r.K - 1) * r.ldw + r.N);
  return r;
}
template <bool KT, int TW>
static __device__ __forceinline__ void rows_ld(const RowsW& W, int grp, int c, int lane, float (&bv)[4][TW]) {
  const int lk = lane >> 4, k0 = 16 * grp + 4 * lk;
  const int K = W.K, N = W.N, ldw = W.ldw;
#if defined(TR_KNOB_NOB)   // timing-only builds: no weight loads
  for (int u = 0; u < 4; ++u)
    for (int q = 0; q < TW; ++q) bv[u][q] = 0.001f * (k0 + u + q);
  return;
#endif
#if TR_LDOFF
  // no per-load bounds arithmetic: rows past the operand (k >= K, or c >= N for KT) fall past the buffer
  // descriptor's range and read 0; the columns c >= N of a row read the next row's (finite) values, which
  // only reach output columns the epilogue zeroes / never stores, or meet the zero padding of A
  (void)K;
  if constexpr (KT) {
#pragma unroll
    for (int q = 0; q < TW; ++q) {
      const f32x4 v = __builtin_bit_cast(
          f32x4, __builtin_amdgcn_raw_buffer_load_b128(W.d, ((c + q) * ldw + 4 * lk) * 4 + 64 * grp, 0, 0));
#pragma unroll
      for (int u = 0; u < 4; ++u) bv[u][q] = v[u];
    }
  } else {
    // a lane whose columns are all past N (the padding of the last column block) reads nothing: its base
    // offset is pushed past the range (no L2 traffic for the 56 padding columns of a 200-wide layer)
    const int vb = c < N ? (4 * lk * ldw + c) * 4 : (1 << 30);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int off = vb + (16 * grp + u) * ldw * 4;
      if constexpr (TW == 4) {
        const f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(W.d, off, 0, 0));
#pragma unroll
        for (int q = 0; q < 4; ++q) bv[u][q] = v[q];
      } else if constexpr (TW == 2) {
        const f32x2 v = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(W.d, off, 0, 0));
        bv[u][0] = v[0];
        bv[u][1] = v[1];
      } else {
        bv[u][0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(W.d, off, 0, 0));
      }
    }
  }
  return;
#endif
  if constexpr (KT) {
#pragma unroll
    for (int q = 0; q < TW; ++q) {
      const f32x4 v = bload4(W.d, ((c + q < N) & (k0 < K)) ? (c + q) * ldw + k0 : -1);
#pragma unroll
      for (int u = 0; u < 4; ++u) bv[u][q] = v[u];
    }
  } else {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int idx = ((c < N) & (k0 + u < K)) ? (k0 + u) * ldw + c : -1;
      if constexpr (TW == 4) {
        const f32x4 v = bload4(W.d, idx);
#pragma unroll
        for (int q = 0; q < 4; ++q) bv[u][q] = v[q];
      } else if constexpr (TW == 2) {
        const f32x2 v = bload2(W.d, idx);
        bv[u][0] = v[0];
        bv[u][1] = v[1];
      } else {
        bv[u][0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(W.d, idx * 4, 0, 0));
      }
    }
  }
}
template <bool KT, int G, int TW>
static __device__ __forceinline__ void rows_pre(const RowsW& W, int c, int lane, float (&pre)[TR_PFM][4][TW]) {
  constexpr int PF = KT ? TR_PF_B : TR_PF;
  if (__builtin_amdgcn_readfirstlane(c - 4 * (lane & 15)) >= W.N) return;   // rows_gemm's no-column exit
#pragma unroll
  for (int grp = 0; grp < PF && grp < G; ++grp) rows_ld<KT, TW>(W, grp, c, lane, pre[grp]);
}
template <bool KT, int G, int TW>
static __device__ __forceinline__ void rows_gemm_pre(const float* As, const RowsW& W, int c, int lane,
                                                     const float (&pre)[TR_PFM][4][TW], f32x4 (&acc)[TW]) {
  constexpr int PF = KT ? TR_PF_B : TR_PF;
  const int li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int q = 0; q < TW; ++q) acc[q] = zero4();
  if (__builtin_amdgcn_readfirstlane(c - 4 * li) >= W.N) return;
  float bq[G + PF][4][TW];
#pragma unroll
  for (int grp = 0; grp < PF && grp < G; ++grp)
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int q = 0; q < TW; ++q) bq[grp][u][q] = pre[grp][u][q];
#pragma unroll
  for (int grp = 0; grp < G; ++grp) {
    if (grp + PF < G) rows_ld<KT, TW>(W, grp + PF, c, lane, bq[grp + PF]);
    __builtin_amdgcn_sched_barrier(0);
    const f32x4 a4 = ld4(As + li * TR_LD + 16 * grp + 4 * lk);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int q = 0; q < TW; ++q) {
#if defined(TR_KNOB_NOMFMA)   // timing-only builds: no MFMAs
        acc[q][u] = fmaf(a4[u], bq[grp][u][q], acc[q][u]);
#else
        acc[q] = mfma4(a4[u], bq[grp][u][q], acc[q]);
#endif
      }
  }
}

// a lane's TW consecutive floats at p (16-B / 8-B aligned)
template <int TW>
static __device__ __forceinline__ void st_tw(float* p, const float (&v)[TW]) {
  if constexpr (TW == 4) *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]};
  else if constexpr (TW == 2) *reinterpret_cast<f32x2*>(p) = f32x2{v[0], v[1]};
  else *p = v[0];
}
template <int TW>
static __device__ __forceinline__ void ld_tw(const float* p, float (&v)[TW]) {
  if constexpr (TW == 4) {
    const f32x4 x = *reinterpret_cast<const f32x4*>(p);
    v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
  } else if constexpr (TW == 1) {
    v[0] = *p;
  } else {
    const f32x2 x = *reinterpret_cast<const f32x2*>(p);
    v[0] = x[0]; v[1] = x[1];
  }
}

// Workgroup b -> (member, row block): workgroups are dealt round-robin over the 8 XCDs (b mod 8), so
// member e's row blocks all get b = e mod 8 (+ 8 per later row block): each member's weights are read
// into ONE XCD's L2 (grid 8 nrb ceil(E / 8); ids past E exit).
static __device__ __forceinline__ bool tr_block(int b, int nrb, int E, int& e, int& rb) {
  const int j = b >> 3;
  e = (b & 7) + 8 * (j / nrb);
  rb = j % nrb;
  return e < E;
}

// ---- forward + loss gradient ----------------------------------------------------------------------
// G0 / GH: k-groups of the inputs / the hidden width (rows_gemm)
template <int G0, int GH>
static __global__ __launch_bounds__(TR_WAVES * 64, 1) void train_fwd_rows_kernel(const TrainRows a) {
  __shared__ __attribute__((aligned(16))) float buf[2][16 * TR_LD];
  __shared__ float red[3][64][17];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 15, lk = lane >> 4;
  int e, rb;
  if (!tr_block(blockIdx.x, a.nrb, a.E, e, rb)) return;
  const int M = a.M, IN = a.IN, H = a.H, D = a.D, i0 = rb * 16;
  // ---- gather: X rows (scaled) into buf[0] (and HBM, for dW_0), targets into HBM; zero K padding
  {
    const int W = IN + D, KP = ((IN + 15) >> 4) << 4;
    const int64_t base = a.bstep ? (int64_t)(*a.bstep) * a.batch : 0;
    for (int i = tid; i < 16 * KP; i += TR_WAVES * 64) buf[0][(i / KP) * TR_LD + i % KP] = 0.f;
    lds_barrier();
    for (int i = tid; i < 16 * W; i += TR_WAVES * 64) {
      const int r = i / W, c = i % W, row = i0 + r;
      if (row >= M) continue;
      const int64_t src = a.rows ? a.rows[e * a.stride + base + row] : row;
      const int64_t er = (int64_t)e * M + row;
      if (c < IN) {
        const float x = (a.inputs[src * IN + c] - a.mu[c]) / a.sigma[c];   // utils.py:96
        a.X[er * IN + c] = x;
        buf[0][r * TR_LD + c] = x;
      } else {
        a.T[er * D + (c - IN)] = a.targets[src * D + (c - IN)];
      }
    }
    lds_barrier();
  }
  // ---- 4 swish layers + the fused heads; lane (li, lk) holds rows 4 lk + i, columns c0 .. c0 + 3
  const int c0 = 64 * (w & 3) + 4 * li + TR_TW * (w >> 2);   // this lane's first column
  auto layer = [&](auto gtag, int l) {
    constexpr int G = decltype(gtag)::value;
    const int K = l == 0 ? IN : H, N = l == TR_NHID ? 2 * D : H;
    const float* Wl = a.P + a.W[l] + (int64_t)e * K * N;
    float bias[TR_TW] = {};
    if (c0 < N) ld_tw<TR_TW>(a.P + a.b[l] + (int64_t)e * N + c0, bias);
    f32x4 acc[TR_TW];
    rows_gemm<false, G, TR_TW>(buf[l & 1], Wl, K, N, N, c0, lane, acc);
    float* out = buf[(l + 1) & 1];
    if (__builtin_amdgcn_readfirstlane(c0 - 4 * li) < N) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {                      // D: row 4 lk + i; tile q = column c0 + q
        const int r = 4 * lk + i, row = i0 + r;
        const bool ok = row < M && c0 < N;
        float v[TR_TW];
#pragma unroll
        for (int q = 0; q < TR_TW; ++q) v[q] = acc[q][i] + bias[q];
        if (l < TR_NHID) {
          const int64_t o = ((int64_t)e * M + row) * H + c0;
          if (ok) st_tw<TR_TW>(a.Z[l] + o, v);             // pre-activation (swish' in the backward)
#pragma unroll
          for (int q = 0; q < TR_TW; ++q) v[q] = swish_fast(v[q]);
          if (ok) st_tw<TR_TW>(a.Hh[l] + o, v);
        } else if (ok) {
          st_tw<TR_TW>(a.OUT + ((int64_t)e * M + row) * 2 * D + c0, v);
        }
        if (!ok)
#pragma unroll
          for (int q = 0; q < TR_TW; ++q) v[q] = 0.f;
        st_tw<TR_TW>(out + r * TR_LD + c0, v);
      }
    }
    lds_barrier();
  };
  layer(std::integral_constant<int, G0>{}, 0);
  for (int l = 1; l <= TR_NHID; ++l) layer(std::integral_constant<int, GH>{}, l);   // 3 swish layers + the heads
  // ---- output gradient (train_loss_kernel's math, per (row, d)) and the block's partial sums
  const float* o = buf[(TR_NHID + 1) & 1];
  const float s = 1.f / ((float)M * (float)D);
  for (int i = tid; i < 16 * D; i += TR_WAVES * 64) {
    const int r = i / D, d = i % D, row = i0 + r;
    float c_mx = 0.f, c_mn = 0.f, c_loss = 0.f;
    if (row < M) {
      const int64_t er = (int64_t)e * M + row;
      const float mx = a.P[a.mx + d], mn = a.P[a.mn + d];
      const float mean = o[r * TR_LD + d], raw = o[r * TR_LD + D + d], y = a.T[er * D + d];
      const float lv1 = mx - softplusf(mx - raw);
      const float lv = mn + softplusf(lv1 - mn);
      const float inv = expf(-lv);
      const float err = mean - y;
      const float dlv = (1.f - err * err * inv) * s;
      const float sb = 1.f / (1.f + expf(-(lv1 - mn))), sa = 1.f / (1.f + expf(-(mx - raw)));
      const float dlv1 = dlv * sb;
      a.dOUT[er * 2 * D + d] = 2.f * err * inv * s;
      a.dOUT[er * 2 * D + D + d] = dlv1 * sa;
      c_mn = dlv * (1.f - sb);
      c_mx = dlv1 * (1.f - sa);
      c_loss = (err * err * inv + lv) * s;
    }
    red[0][d][r] = c_mx;
    red[1][d][r] = c_mn;
    red[2][d][r] = c_loss;
  }
  lds_barrier();
  if (tid < D) {                                          // rows in order (deterministic)
    float t3[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 3; ++k)
      for (int r = 0; r < 16; ++r) t3[k] += red[k][tid][r];
    float* pp = a.lpart + (((int64_t)e * a.nrb + rb) * D + tid) * 4;
    pp[0] = t3[0]; pp[1] = t3[1]; pp[2] = t3[2];
  }
}

// ---- batch-level tail: the (member, row block) partial sums, then train_loss_kernel's tail ------------
constexpr int TR_TAIL_CH = 8;     // chunks per output column, at most
constexpr int TR_TAIL_SH = 512;   // floats of sh the tail may use (3 per (chunk, column))
// TR: TrainRows or TrainTail (the fields used here)
// KEEP_POW: leave the beta powers and the minibatch counter to the caller (train_step_kernel advances them
// once every workgroup of its launch has read them)
template <class TR, bool KEEP_POW = false>
static __device__ __forceinline__ void train_loss_tail(const TR& a, float* sh) {
  const int D = a.D, n = a.E * a.nrb;
  const float b1p = a.beta_pow[0], b2p = a.beta_pow[1];  // every thread reads them before thread 0 advances them
  const float lr_t = a.lr * sqrtf(1.f - b2p) / (1.f - b1p);
  __syncthreads();
  // the E nrb partials of each d in TR_TAIL_CH interleaved chunks (thread (j, d): partials j, j + CH, ...
  // in order, 8 independent loads in flight), then the chunk sums in chunk order: deterministic, and one
  // memory latency instead of E nrb dependent ones (a serial loop made the tail ~30 us)
  const int CH = max(1, min(TR_TAIL_CH, min(TR_TAIL_SH / (3 * D), (int)blockDim.x / D)));
  const int t = threadIdx.x;
  if (t < CH * D) {
    const int dd = t % D, j = t / D;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll 8
    for (int c = j; c < n; c += CH) {
      const float* pp = a.lpart + ((int64_t)c * D + dd) * 4;
      s0 += pp[0]; s1 += pp[1]; s2 += pp[2];
    }
    sh[(j * D + dd) * 3 + 0] = s0; sh[(j * D + dd) * 3 + 1] = s1; sh[(j * D + dd) * 3 + 2] = s2;
  }
  __syncthreads();
  float loss = 0.f;
  if (t < D) {
    const int dd = t;
    float gmx = 0.f, gmn = 0.f;
    for (int j = 0; j < CH; ++j) {
      gmx += sh[(j * D + dd) * 3 + 0]; gmn += sh[(j * D + dd) * 3 + 1]; loss += sh[(j * D + dd) * 3 + 2];
    }
    gmx += 0.01f;                                                   // 0.01 * sum(max_logvar)
    gmn -= 0.01f;                                                   // -0.01 * sum(min_logvar)
    a.G[a.mx + dd] = gmx;
    a.G[a.mn + dd] = gmn;
    adam_apply(a.ad, a.mx + dd, gmx, adam_load(a.ad, a.mx + dd), lr_t);
    adam_apply(a.ad, a.mn + dd, gmn, adam_load(a.ad, a.mn + dd), lr_t);
  }
  __syncthreads();                                                  // every chunk sum is read
  if (t < D) sh[t] = loss;
  __syncthreads();
  if (threadIdx.x == 0) {
    float loss = 0.f;
    for (int dd = 0; dd < D; ++dd) loss += sh[dd];
    a.logs[0] = loss;                                               // data term of the train loss
    if (!KEEP_POW) {
      a.beta_pow[2] = lr_t;
      a.beta_pow[0] = b1p * 0.9f;
      a.beta_pow[1] = b2p * 0.999f;
      if (a.bstep_inc) *a.bstep_inc += 1;
    }
  }
}

// ---- activation-gradient chain ------------------------------------------------------------------
// GD / GH: k-groups of the heads' width 2D / the hidden width
template <int GD, int GH>
static __global__ __launch_bounds__(TR_WAVES * 64, 1) void train_bwd_rows_kernel(const TrainRows a) {
  __shared__ __attribute__((aligned(16))) float buf[2][16 * TR_LD];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 15, lk = lane >> 4;
  if (blockIdx.x == gridDim.x - 1) {                      // the batch-level tail (last block)
    train_loss_tail(a, buf[0]);
    return;
  }
  int e, rb;
  if (!tr_block(blockIdx.x, a.nrb, a.E, e, rb)) return;  // the forward's placement: weights L2-warm
  const int M = a.M, H = a.H, D = a.D, i0 = rb * 16;
  {  // dY of the heads into buf[0], zero-padded to a multiple of 16 columns
    const int N = 2 * D, NP = ((N + 15) >> 4) << 4;
    for (int i = tid; i < 16 * NP; i += TR_WAVES * 64) {
      const int r = i / NP, c = i % NP, row = i0 + r;
      buf[0][r * TR_LD + c] = (row < M && c < N) ? a.dOUT[((int64_t)e * M + row) * N + c] : 0.f;
    }
    lds_barrier();
  }
  const int c0 = 64 * (w & 3) + 4 * li + TR_TW * (w >> 2);   // this lane's first column
  auto layer = [&](auto gtag, int l) {
    constexpr int G = decltype(gtag)::value;
    const int Kl = H, Nl = l == TR_NHID ? 2 * D : H;     // layer l: [Kl -> Nl]; dZ_{l-1} is 16 x Kl
    const float* Wl = a.P + a.W[l] + (int64_t)e * Kl * Nl;
    float zm[4][TR_TW];                                   // swish'(Z_{l-1}) operands, fetched up front
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = i0 + 4 * lk + i;
#pragma unroll
      for (int q = 0; q < TR_TW; ++q) zm[i][q] = 0.f;
      if (c0 < Kl && row < M) ld_tw<TR_TW>(a.Z[l - 1] + ((int64_t)e * M + row) * H + c0, zm[i]);
    }
    f32x4 acc[TR_TW];
    rows_gemm<true, G, TR_TW>(buf[(TR_NHID - l) & 1], Wl, Nl, Kl, Nl, c0, lane, acc);
    float* out = buf[(TR_NHID - l + 1) & 1];
    if (__builtin_amdgcn_readfirstlane(c0 - 4 * li) < Kl) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 4 * lk + i, row = i0 + r;
        const bool ok = row < M && c0 < Kl;
        float v[TR_TW];
#pragma unroll
        for (int q = 0; q < TR_TW; ++q) v[q] = ok ? acc[q][i] * dswish_fast(zm[i][q]) : 0.f;
        if (ok) st_tw<TR_TW>(a.dZ[l - 1] + ((int64_t)e * M + row) * H + c0, v);
        st_tw<TR_TW>(out + r * TR_LD + c0, v);
      }
    }
    lds_barrier();
  };
  layer(std::integral_constant<int, GD>{}, TR_NHID);
  for (int l = TR_NHID - 1; l >= 1; --l) layer(std::integral_constant<int, GH>{}, l);
}

// ---- forward + backward rows in ONE launch (MOPO_TRAIN_FUSED) -------------------------------------
// train_fwd_rows_kernel then train_bwd_rows_kernel's chain in the same workgroup: the pre-activations Z
// stay in LDS (zb, 66 KB; no HBM round trip), the heads' output gradient goes straight into the
// backward's input buffer, and the batch-level tail moves to the weight-gradient launch (bnn_train.hip
// train_wgrad_kernel), which only needs this step's lr_t -- block 0 writes it here (the tail advances
// the beta powers after every reader of them in this step).
#ifndef TR_XPF
#define TR_XPF 1   // the next layer's first weight k-groups issued before this layer's epilogue (rows_pre)
#endif
// The fused rows body of train_rows_kernel.
#ifndef MOPO_TRAIN_STAMPS
#define MOPO_TRAIN_STAMPS 0   // diagnostic builds: per-workgroup phase stamps of train_rows_kernel
#endif
#if MOPO_TRAIN_STAMPS
__device__ uint64_t g_train_stamps[2048 * 8];
#endif
// stamp i of this workgroup (wave 0; its lanes all store the same value); v: a value instead of the clock
static __device__ __forceinline__ void tstamp(int i, int64_t v = -1) {
#if MOPO_TRAIN_STAMPS
  if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 0 && blockIdx.x < 2048)
    __hip_atomic_store(&g_train_stamps[blockIdx.x * 8 + i], v < 0 ? __builtin_amdgcn_s_memrealtime() : (uint64_t)v,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
  (void)i; (void)v;
#endif
}
constexpr int TR_LDS_FLOATS = (2 + TR_NHID) * 16 * TR_LD + 3 * 64 * 17;
template <int G0, int GH, int GD>
static __device__ __forceinline__ void train_rows_body(const TrainRows& a, float* lds, int e, int rb) {
  float (*buf)[16 * TR_LD] = reinterpret_cast<float (*)[16 * TR_LD]>(lds);
  float (*zb)[16 * TR_LD] = reinterpret_cast<float (*)[16 * TR_LD]>(lds + 2 * 16 * TR_LD);
  float (*red)[64][17] = reinterpret_cast<float (*)[64][17]>(lds + (2 + TR_NHID) * 16 * TR_LD);
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6), li = lane & 15;
  const int M = a.M, IN = a.IN, H = a.H, D = a.D, i0 = rb * 16;
  const int c0 = 64 * (w & 3) + 4 * li + TR_TW * (w >> 2);   // this lane's first column
  auto wfwd = [&](int l) {
    const int K = l == 0 ? IN : H, N = l == TR_NHID ? 2 * D : H;
    return rows_w<false>(a.P + a.W[l] + (int64_t)e * K * N, K, N, N);
  };
  auto wbwd = [&](int l) {   // layer l: [H -> Nl], read transposed
    const int Nl = l == TR_NHID ? 2 * D : H;
    return rows_w<true>(a.P + a.W[l] + (int64_t)e * H * Nl, Nl, H, Nl);
  };
  float pre[TR_PFM][4][TR_TW];
  if (TR_XPF) rows_pre<false, G0, TR_TW>(wfwd(0), c0, lane, pre);   // in flight during the gather
  // the next step's rows (staged): two items per thread at most (host: 16 (IN + D) <= 2 TR_WAVES 64)
  constexpr int NPF = 2;
  float pf_v[NPF];
  int pf_src[NPF];
  const bool staged = a.staged;
  if (staged) {   // the indices now; the rows they name after layer 0; the stores at the end
    const int W = IN + D;
    const int64_t nb = (int64_t)(*a.bstep + 1) * a.batch;
    const auto drows = rsrc(reinterpret_cast<const float*>(a.rows), (int64_t)a.E * a.stride);
#pragma unroll
    for (int q = 0; q < NPF; ++q) {
      const int i = tid + q * TR_WAVES * 64, row = i0 + (i / W);
      // past the index array: row 0 (the last full step prefetches for a minibatch that does not come)
      // rows past the member's batch (batch % 16 != 0) are neither loaded nor stored
      pf_src[q] = i < 16 * W && row < M ? __builtin_bit_cast(int, __builtin_amdgcn_raw_buffer_load_b32(
                                              drows, (int)((e * a.stride + nb + row) * 4), 0, 0)) : 0;
    }
  }
  auto prefetch_rows = [&]() {
    if (!staged) return;
    const int W = IN + D;
#pragma unroll
    for (int q = 0; q < NPF; ++q) {
      const int i = tid + q * TR_WAVES * 64, c = i % W;
      const int64_t src = pf_src[q];
      pf_v[q] = i >= 16 * W || i0 + i / W >= M ? 0.f : c < IN ? (a.inputs[src * IN + c] - a.mu[c]) / a.sigma[c]   // utils.py:96
                                           : a.targets[src * D + (c - IN)];
    }
  };
  {  // gather (train_fwd_rows_kernel); staged: this step's rows from X
    const int W = IN + D, KP = ((IN + 15) >> 4) << 4;
    const int64_t base = a.bstep ? (int64_t)(*a.bstep) * a.batch : 0;
    for (int i = tid; i < 16 * KP; i += TR_WAVES * 64) buf[0][(i / KP) * TR_LD + i % KP] = 0.f;
    lds_barrier();
    if (staged) {
      for (int i = tid; i < 16 * IN; i += TR_WAVES * 64) {
        const int r = i / IN, c = i % IN;
        if (i0 + r < M) buf[0][r * TR_LD + c] = a.X[((int64_t)e * M + i0 + r) * IN + c];   // padding rows stay 0
      }
    } else
    for (int i = tid; i < 16 * W; i += TR_WAVES * 64) {
      const int r = i / W, c = i % W, row = i0 + r;
      if (row >= M) continue;
      const int64_t src = a.rows ? a.rows[e * a.stride + base + row] : row;
      const int64_t er = (int64_t)e * M + row;
      if (c < IN) {
        const float x = (a.inputs[src * IN + c] - a.mu[c]) / a.sigma[c];   // utils.py:96
        *(&a.X[er * IN + c]) = x;
        buf[0][r * TR_LD + c] = x;
      } else {
        a.T[er * D + (c - IN)] = a.targets[src * D + (c - IN)];
      }
    }
    lds_barrier();
  }
  const int lk = lane >> 4;
  auto fwd = [&](auto gtag, int l) {
    constexpr int G = decltype(gtag)::value;
    const int K = l == 0 ? IN : H, N = l == TR_NHID ? 2 * D : H;
    const float* Wl = a.P + a.W[l] + (int64_t)e * K * N;
    float bias[TR_TW] = {};
    if (c0 < N) ld_tw<TR_TW>(a.P + a.b[l] + (int64_t)e * N + c0, bias);
    f32x4 acc[TR_TW];
    if (TR_XPF) {
      rows_gemm_pre<false, G, TR_TW>(buf[l & 1], wfwd(l), c0, lane, pre, acc);
      if (l < TR_NHID) rows_pre<false, GH, TR_TW>(wfwd(l + 1), c0, lane, pre);
      else rows_pre<true, GD, TR_TW>(wbwd(TR_NHID), c0, lane, pre);   // the backward's first layer
    } else {
      rows_gemm<false, G, TR_TW>(buf[l & 1], Wl, K, N, N, c0, lane, acc);
    }
    float* out = buf[(l + 1) & 1];
    if (__builtin_amdgcn_readfirstlane(c0 - 4 * li) < N) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 4 * lk + i, row = i0 + r;
        const bool ok = row < M && c0 < N;
        float v[TR_TW];
#pragma unroll
        for (int q = 0; q < TR_TW; ++q) v[q] = acc[q][i] + bias[q];
        if (l < TR_NHID) {
          st_tw<TR_TW>(zb[l] + r * TR_LD + c0, v);             // pre-activation, for swish' below
#pragma unroll
          for (int q = 0; q < TR_TW; ++q) v[q] = swish_fast(v[q]);
          if (ok) st_tw<TR_TW>(a.Hh[l] + ((int64_t)e * M + row) * H + c0, v);
        } else if (ok) {
          st_tw<TR_TW>(a.OUT + ((int64_t)e * M + row) * 2 * D + c0, v);
        }
        if (!ok)
#pragma unroll
          for (int q = 0; q < TR_TW; ++q) v[q] = 0.f;
        st_tw<TR_TW>(out + r * TR_LD + c0, v);
      }
    }
    lds_barrier();
  };
  tstamp(1);
  fwd(std::integral_constant<int, G0>{}, 0);
  prefetch_rows();
  tstamp(2);
  for (int l = 1; l <= TR_NHID; ++l) fwd(std::integral_constant<int, GH>{}, l);
  tstamp(3);
  // ---- output gradient and the block's partial sums (train_fwd_rows_kernel); dY of the heads also into
  //      buf[0] (the backward's input; zero-padded to a multiple of 16 columns)
  const float* o = buf[(TR_NHID + 1) & 1];
  float* dy = buf[TR_NHID & 1];
  const int N2 = 2 * D, NP = ((N2 + 15) >> 4) << 4;
  const float s = 1.f / ((float)M * (float)D);
  for (int i = tid; i < 16 * D; i += TR_WAVES * 64) {
    const int r = i / D, d = i % D, row = i0 + r;
    float c_mx = 0.f, c_mn = 0.f, c_loss = 0.f, g_mean = 0.f, g_lv = 0.f;
    if (row < M) {
      const int64_t er = (int64_t)e * M + row;
      const float mx = a.P[a.mx + d], mn = a.P[a.mn + d];
      const float mean = o[r * TR_LD + d], raw = o[r * TR_LD + D + d], y = a.T[er * D + d];
      const float lv1 = mx - softplusf(mx - raw);
      const float lv = mn + softplusf(lv1 - mn);
      const float inv = expf(-lv);
      const float err = mean - y;
      const float dlv = (1.f - err * err * inv) * s;
      const float sb = 1.f / (1.f + expf(-(lv1 - mn))), sa = 1.f / (1.f + expf(-(mx - raw)));
      const float dlv1 = dlv * sb;
      g_mean = 2.f * err * inv * s;
      g_lv = dlv1 * sa;
      *(&a.dOUT[er * 2 * D + d]) = g_mean;
      *(&a.dOUT[er * 2 * D + D + d]) = g_lv;
      c_mn = dlv * (1.f - sb);
      c_mx = dlv1 * (1.f - sa);
      c_loss = (err * err * inv + lv) * s;
    }
    dy[r * TR_LD + d] = g_mean;
    dy[r * TR_LD + D + d] = g_lv;
    red[0][d][r] = c_mx;
    red[1][d][r] = c_mn;
    red[2][d][r] = c_loss;
  }
  for (int i = tid; i < 16 * (NP - N2); i += TR_WAVES * 64) dy[(i / (NP - N2)) * TR_LD + N2 + i % (NP - N2)] = 0.f;
  lds_barrier();
  if (tid < D) {                                          // rows in order (deterministic)
    float t3[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 3; ++k)
      for (int r = 0; r < 16; ++r) t3[k] += red[k][tid][r];
    float* pp = a.lpart + (((int64_t)e * a.nrb + rb) * D + tid) * 4;
    *(pp) = t3[0]; *(pp + 1) = t3[1]; *(pp + 2) = t3[2];
  }
  tstamp(4);
  // ---- the activation-gradient chain (train_bwd_rows_kernel), swish'(Z) from LDS; dY of layer l sits in
  //      buf[(TR_NHID - l) & 1] as in that kernel (dy = buf[TR_NHID & 1] = buf[0] for 4 hidden layers)
  static_assert((TR_NHID & 1) == 0, "the backward's first input buffer is buf[0]");
  auto bwd = [&](auto gtag, int l) {
    constexpr int G = decltype(gtag)::value;
    const int Kl = H, Nl = l == TR_NHID ? 2 * D : H;     // layer l: [Kl -> Nl]; dZ_{l-1} is 16 x Kl
    const float* Wl = a.P + a.W[l] + (int64_t)e * Kl * Nl;
    float zm[4][TR_TW];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int q = 0; q < TR_TW; ++q) zm[i][q] = 0.f;
      if (c0 < Kl) ld_tw<TR_TW>(zb[l - 1] + (4 * lk + i) * TR_LD + c0, zm[i]);
    }
    f32x4 acc[TR_TW];
    if (TR_XPF) {
      rows_gemm_pre<true, G, TR_TW>(buf[(TR_NHID - l) & 1], wbwd(l), c0, lane, pre, acc);
      if (l > 1) rows_pre<true, GH, TR_TW>(wbwd(l - 1), c0, lane, pre);
    } else {
      rows_gemm<true, G, TR_TW>(buf[(TR_NHID - l) & 1], Wl, Nl, Kl, Nl, c0, lane, acc);
    }
    float* out = buf[(TR_NHID - l + 1) & 1];
    if (__builtin_amdgcn_readfirstlane(c0 - 4 * li) < Kl) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 4 * lk + i, row = i0 + r;
        const bool ok = row < M && c0 < Kl;
        float v[TR_TW];
#pragma unroll
        for (int q = 0; q < TR_TW; ++q) v[q] = ok ? acc[q][i] * dswish_fast(zm[i][q]) : 0.f;
        if (ok) st_tw<TR_TW>(a.dZ[l - 1] + ((int64_t)e * M + row) * H + c0, v);
        st_tw<TR_TW>(out + r * TR_LD + c0, v);
      }
    }
    lds_barrier();
  };
  bwd(std::integral_constant<int, GD>{}, TR_NHID);
  tstamp(5);
  for (int l = TR_NHID - 1; l >= 1; --l) {
    bwd(std::integral_constant<int, GH>{}, l);
    if (l == 2) tstamp(6);
  }
  tstamp(7);
  if (staged) {   // the next step's rows, loaded at the start
    const int W = IN + D;
#pragma unroll
    for (int q = 0; q < NPF; ++q) {
      const int i = tid + q * TR_WAVES * 64, r = i / W, c = i % W;
      const int64_t er = (int64_t)e * M + i0 + r;
      if (i < 16 * W && i0 + r < M) {   // never into the next member's rows (or past the last member's)
        if (c < IN) a.Xn[er * IN + c] = pf_v[q];
        else a.Tn[er * D + (c - IN)] = pf_v[q];
      }
    }
  }
}

template <int G0, int GH, int GD>
static __global__ __launch_bounds__(TR_WAVES * 64, 1) void train_rows_kernel(const TrainRows a) {
  __shared__ __attribute__((aligned(16))) float lds[TR_LDS_FLOATS];
  int e, rb;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const float b1p = a.beta_pow[0], b2p = a.beta_pow[1];
    a.beta_pow[2] = a.lr * sqrtf(1.f - b2p) / (1.f - b1p);          // this step's TF1 Adam step size
  }
  if (!tr_block(blockIdx.x, a.nrb, a.E, e, rb)) return;
  tstamp(0);
  train_rows_body<G0, GH, GD>(a, lds, e, rb);
}

}  // namespace mopo
