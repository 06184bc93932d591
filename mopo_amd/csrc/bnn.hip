// Probabilistic ensemble (BNN) forward on CDNA4 MFMA.
//
// Replaces BNN._compile_outputs / BNN.predict (mopo/models/bnn.py:508-546, 631-675),
// TensorStandardScaler.transform (mopo/models/utils.py:96) and FC.compute_output_tensor
// (mopo/models/fc.py:84-106).
//
// Work decomposition: a workgroup of 4 waves owns one ensemble member and 64 rows (16 per wave)
// and runs all five layers with the activations held in VGPRs: every layer is the transposed
// product Out^T[n][m] = W^T[n][k] X^T[k][m] on v_mfma_f32_16x16x4_f32, whose accumulator layout
// (feature on the register axis, row on the lane axis) is exactly the B operand of the next layer,
// so activations never leave registers.  Weights stream HBM/L2 -> LDS as 1 KiB fragments with
// global_load_lds, double-buffered per 16-deep k-group and shared by the 4 waves (mlp_tile.h);
// each layer's bias rides along with its last slice.  Workgroups are member-major so the ones
// resident on an XCD share one member's weights in L2.
#include "mlp_tile.h"

// build-time knobs (defaults are the tuned configuration; scripts/micro/bnn_knobs.hip explores them)
#ifndef BNN_KPB
#define BNN_KPB 1  // k-groups staged per barrier in the hidden / head layers
#endif

#include <vector>
#include <cstring>
#include <type_traits>
#include <cmath>

namespace mopo {

// ---------------------------------------------------------------------------------------
// weight packing:  src W[E][K][N] (TF layout, x @ W)  ->  fragment-major (see internal.h);
// perm_k / perm_n: that side is a hidden/input width laid out by slot_feat (mlp_tile.h)
__global__ void pack_frags_kernel(const float* __restrict__ src, float* __restrict__ dst, int E, int K,
                                  int N, int KG, int NB, int perm_k, int perm_n) {
  int64_t total = (int64_t)E * KG * NB * 256;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int t = i & 3, lane = (i >> 2) & 63;
    int64_t f = i >> 8;
    int nb = f % NB;
    int kg = (f / NB) % KG;
    int e = f / ((int64_t)NB * KG);
    int k = kg * 16 + 4 * (lane >> 4) + t, n = nb * 16 + (lane & 15);
    if (perm_k) k = slot_feat(k, K);
    if (perm_n == 1) n = slot_feat(n, N);
    else if (perm_n == 2) n = head_col(n, N / 2);  // fused [mean | log-var] head, N = 2D
    dst[i] = (k >= 0 && n >= 0 && k < K && n < N) ? src[((int64_t)e * K + k) * N + n] : 0.f;
  }
}

// bf16 fragments for v_mfma_f32_16x16x32_bf16 (k-group of 32, permuted k order: mlp_tile.h):
// frag (kg, nb), lane l (n = l&15, g = l>>4), element j = W[e][32 kg + bf16_kperm(g, j)][16 nb + n]
// P > 1: fragment (kg, p, nb) holds part p of the split (split_bf16), laid out [e][kg][p][nb].
template <int P>
__global__ void pack_frags_bf16_kernel(const float* __restrict__ src, short* __restrict__ dst, int E, int K, int N,
                                       int KG, int NB, int perm_k, int perm_n) {
  int64_t total = (int64_t)E * KG * P * NB * 512;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int j = i & 7, lane = (i >> 3) & 63;
    int64_t f = i >> 9;
    int nb = f % NB;
    int p = (f / NB) % P;
    int kg = (f / ((int64_t)NB * P)) % KG;
    int e = f / ((int64_t)NB * P * KG);
    int k = kg * 32 + bf16_kperm(lane >> 4, j), n = nb * 16 + (lane & 15);
    if (perm_k) k = slot_feat(k, K);
    if (perm_n == 1) n = slot_feat(n, N);
    else if (perm_n == 2) n = head_col(n, N / 2);
    short parts[P];
    split_bf16<P>((k >= 0 && n >= 0 && k < K && n < N) ? src[((int64_t)e * K + k) * N + n] : 0.f, parts);
    short v = parts[0];
#pragma unroll
    for (int q = 1; q < P; ++q)
      if (q == p) v = parts[q];
    dst[i] = v;
  }
}

// f16x3 fragments: the bf16 fragment layout with P = 2 fp16 parts of W * 2^k_e (split_f16_scaled);
// scale[e] = 2^k_e puts member e's max |W| of this layer in [2^14, 2^15)
__global__ void pack_frags_f16s_kernel(const float* __restrict__ src, short* __restrict__ dst, int E, int K, int N,
                                       int KG, int NB, int perm_k, int perm_n, const float* __restrict__ scale) {
  constexpr int P = 2;
  int64_t total = (int64_t)E * KG * P * NB * 512;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int j = i & 7, lane = (i >> 3) & 63;
    int64_t f = i >> 9;
    int nb = f % NB;
    int p = (f / NB) % P;
    int kg = (f / ((int64_t)NB * P)) % KG;
    int e = f / ((int64_t)NB * P * KG);
    int k = kg * 32 + bf16_kperm(lane >> 4, j), n = nb * 16 + (lane & 15);
    if (perm_k) k = slot_feat(k, K);
    if (perm_n == 1) n = slot_feat(n, N);
    else if (perm_n == 2) n = head_col(n, N / 2);
    const F16Parts q = split_f16_scaled((k >= 0 && n >= 0 && k < K && n < N) ? src[((int64_t)e * K + k) * N + n] : 0.f,
                                        scale[e]);
    dst[i] = p == 0 ? q.hi : q.lo;
  }
}

// hidden biases in slot order (slot_feat)
// mul: the 16-bit kernels keep their hidden biases pre-multiplied by -log2(e) (see bnn_fwd_f16s_kernel)
__global__ void pack_bias_kernel(const float* __restrict__ src, float* __restrict__ dst, int E, int N,
                                 int NP, float mul) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= E * NP) return;
  int e = i / NP, n = slot_feat(i % NP, N);
  dst[i] = n >= 0 ? src[e * N + n] * mul : 0.f;
}

// ---------------------------------------------------------------------------------------
int pack_frags(const float* src, float* dst, int E, int K, int N, int KG, int NB, hipStream_t s, int perm_k) {
  const int64_t tot = (int64_t)E * KG * NB * 256;
  const int blocks = (int)std::min<int64_t>((tot + 255) / 256, 4096);
  hipLaunchKernelGGL(pack_frags_kernel, dim3(blocks), dim3(256), 0, s, src, dst, E, K, N, KG, NB, perm_k, 0);
  MOPO_HIP(hipGetLastError());
  return 0;
}

__device__ __forceinline__ float load_feat(const void* p, int f64, int64_t idx) {
  return f64 ? (float)reinterpret_cast<const double*>(p)[idx] : reinterpret_cast<const float*>(p)[idx];
}

// bias + swish, acc -> next-layer input (fc.py:21,99-106); the layer's bias was staged in LDS
template <int NB, int R>
__device__ __forceinline__ void bias_swish(const float* lds_bias, const f32x4 (&acc)[R][NB], f32x4 (&out)[R][NB],
                                           int g) {
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const f32x4 bb = *reinterpret_cast<const f32x4*>(lds_bias + nb * 16 + 4 * g);
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
#ifndef BNN_KNOB_NOSWISH
        out[r][nb][t] = swish_fast(acc[r][nb][t] + bb[t]);
#else
        out[r][nb][t] = acc[r][nb][t] + bb[t];
#endif
      }
  }
}

// heads -> outputs for one row per lane group (bnn.py:661-675; rollout mode: fake_env.py:66-81, 110)
// hx = the member's head aux block [bias | max_logvar | min_logvar] (NBO*16 each, in head_col slot
// order), staged in LDS by the head layer; sel_e = the row's selected member (rollout)
template <int NBO, int MODE>
__device__ __forceinline__ void head_epilogue(const BnnDev& w, const FwdArgs& a, const f32x4 (&hd)[NBO], int e,
                                              int64_t row, int64_t count, int g, const float* hx, int sel_e) {
  const int D = w.D, Q = (D + 3) >> 2;
  const bool ok = row < count;
  float ss = 0.f;  // sum of std^2 over D (learned-var penalty, fake_env.py:110)
  const bool selected = (MODE == FWD_ROLLOUT) && ok && sel_e == e;
#pragma unroll
  for (int nb = 0; nb < NBO; ++nb) {
    const f32x4 bb = *reinterpret_cast<const f32x4*>(hx + nb * 16 + 4 * g);
    const f32x4 bmx = *reinterpret_cast<const f32x4*>(hx + NBO * 16 + nb * 16 + 4 * g);
    const f32x4 bmn = *reinterpret_cast<const f32x4*>(hx + 2 * NBO * 16 + nb * 16 + 4 * g);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int j = 4 * nb + t;  // wave-uniform kind
      const float v = hd[nb][t] + bb[t];
      if (j < Q) {
        const int d = g + 4 * j;
        const bool valid = d < D;
        const float mx = bmx[t], mn = bmn[t];
        float lv = mx - softplus_fast(mx - v);  // bnn.py:669
        lv = mn + softplus_fast(lv - mn);       // bnn.py:670
        const float l2 = lv * 1.4426950408889634f;
        if (MODE == FWD_PREDICT) {
          const float var = __builtin_amdgcn_exp2f(l2);         // bnn.py:675
          if (ok && valid) a.var[((int64_t)e * a.B + row) * D + d] = var;
        } else {
          const float sd = __builtin_amdgcn_exp2f(0.5f * l2);   // sqrt(exp(lv)), fake_env.py:67
          if (valid) ss += sd * sd;
          if (selected && valid) a.std_sel[row * D + d] = sd;
          if (a.std_all && ok && valid) a.std_all[((int64_t)e * a.all_stride + row) * D + d] = sd;
        }
      } else if (j < 2 * Q) {
        const int d = g + 4 * (j - Q);
        if (d < D) {
          if (MODE == FWD_PREDICT) {
            if (ok) a.mean[((int64_t)e * a.B + row) * D + d] = v;
          } else {
            if (selected) a.mean_sel[row * D + d] = v;
            if (a.mean_all && ok) a.mean_all[((int64_t)e * a.all_stride + row) * D + d] = v;
          }
        }
      }
    }
  }
  if (MODE == FWD_ROLLOUT) {
    ss += __shfl_xor(ss, 16);
    ss += __shfl_xor(ss, 32);
    if (g == 0 && ok) atomicMax(a.pen_bits + row, __float_as_uint(sqrtf(ss)));  // >= 0: uint order
  }
}

// TQ0 / TQH: k-steps run in the last k-group of the inputs / hidden width (tail_steps; 4 = all)
template <int KG0, int NBH, int NBO, int R, int MODE, int WAVES, int TQ0 = 4, int TQH = 4>
#ifndef BNN_MINB_WIDE
#define BNN_MINB_WIDE 2  // workgroups per CU the H = 400 variant is compiled for
#endif
__global__ __launch_bounds__(WAVES * 64, (WAVES >= 8 || NBH > 16) ? BNN_MINB_WIDE : 2) void bnn_fwd_kernel(const BnnDev w,
                                                                                                   const FwdArgs a) {
  constexpr int NBMAX = NBH > NBO ? NBH : NBO;
  constexpr int KPB = BNN_KPB;                            // k-groups per barrier (hidden/head layers)
  constexpr int SLOT = (KPB * NBMAX + WAVES - 1) / WAVES * WAVES * 256;  // floats per buffer (stage_block)
  constexpr int BIASQ = NBH > 3 * NBO ? NBH * 4 : 3 * NBO * 4;  // quads: hidden bias / head aux
  // ONE __shared__ array (weight double buffer | bias): a second LDS object beside the
  // global_load_lds destination makes hipcc wait vmcnt(0) before the first ds_read of a k-group,
  // draining the next slice's copy instead of overlapping it with the MFMAs
  __shared__ __attribute__((aligned(16))) float lds[2 * SLOT + (BIASQ + 63) / 64 * 256];
  float* lds_bias = lds + 2 * SLOT;
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), m = lane & 15, g = lane >> 4;
  const int64_t count = a.d_count ? (int64_t)*a.d_count : a.B;
  const int groups = ceil_div(a.ntiles, WAVES);
  const int e = blockIdx.x / groups, grp = blockIdx.x % groups;
  const int tile = grp * WAVES + wv;
  const int64_t row0 = (int64_t)tile * 16 * R;
  if ((int64_t)grp * WAVES * 16 * R >= count) return;  // whole workgroup past the live rows
  const int IN = w.IN, O = w.O, D = w.D;
  int sel_e[R];  // the selected member of each row, fetched early (used by the head epilogue)
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t row = row0 + r * 16 + m;
    sel_e[r] = (MODE == FWD_ROLLOUT && a.sel && row < count) ? a.sel[row] : -1;
  }

  // ---- layer-0 input: scaler transform (utils.py:96), f64 inputs cast to f32 as TF's feed does
  f32x4 x0[R][KG0];
  if (a.xs) {  // rollout: the actor already wrote the scaled row in slot order
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int64_t row = row0 + r * 16 + m;
#pragma unroll
      for (int kg = 0; kg < KG0; ++kg) x0[r][kg] = row < count ? ld4(a.xs + row * XS_STRIDE + kg * 16 + 4 * g) : zero4();
    }
  } else
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t row = row0 + r * 16 + m;
    const bool ok = row < count;
#pragma unroll
    for (int kg = 0; kg < KG0; ++kg)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int k = slot_feat(kg * 16 + 4 * g + t, IN);
        float v = 0.f;
#ifndef BNN_KNOB_NOX0
        if (ok && k >= 0) {
          float raw = k < O ? load_feat(a.in.xa, a.in.xa_f64, row * a.in.sa + k)
                            : load_feat(a.in.xb, a.in.xb_f64, row * a.in.sb + (k - O));
          v = (raw - w.mu[k]) / w.sigma[k];
        }
#else
        v = ok && k >= 0 ? 0.01f * (float)(k + m) : 0.f;
#endif
        x0[r][kg][t] = v;
      }
  }
  f32x4 acc[R][NBH], hcur[R][NBH];
  const int64_t hp = w.BS;  // per-member bias stride
#ifndef BNN_KNOB_NOXPRE
  // each layer's first weight slice (block of KPB k-groups) is copied during the previous layer's
  // last block; parity: block b of a layer uses buffer (b + par) & 1
  constexpr int NBLKH = (NBH + KPB - 1) / KPB;
  const float* wh0 = w.wh + (int64_t)e * NBH * NBH * 256;
  layer_lds<KG0, NBH, R, WAVES, SLOT, NBH * 4, 1, TQ0, NBH, false, NBH, false, KPB, NBH>(
      w.w0 + (int64_t)e * KG0 * NBH * 256, x0, acc, lds, wv, lane, w.b0 + e * hp, lds_bias, 0, wh0);
  bias_swish<NBH, R>(lds_bias, acc, hcur, g);
  int par = KG0 & 1;
  for (int l = 0; l < 2; ++l) {  // hidden layers 1, 2 (constructor.py:31-33)
    layer_lds<NBH, NBH, R, WAVES, SLOT, NBH * 4, KPB, TQH, NBH, true, NBH, false, KPB, NBH>(
        w.wh + ((int64_t)l * w.E + e) * NBH * NBH * 256, hcur, acc, lds, wv, lane,
        w.bh + ((int64_t)l * w.E + e) * hp, lds_bias, par, w.wh + ((int64_t)(l + 1) * w.E + e) * NBH * NBH * 256);
    bias_swish<NBH, R>(lds_bias, acc, hcur, g);
    par = (par + NBLKH) & 1;
  }
  layer_lds<NBH, NBH, R, WAVES, SLOT, NBH * 4, KPB, TQH, NBO, true, NBH, false, KPB, NBO>(  // hidden layer 3
      w.wh + ((int64_t)2 * w.E + e) * NBH * NBH * 256, hcur, acc, lds, wv, lane, w.bh + ((int64_t)2 * w.E + e) * hp,
      lds_bias, par, w.whd + (int64_t)e * NBH * NBO * 256);
  bias_swish<NBH, R>(lds_bias, acc, hcur, g);
  par = (par + NBLKH) & 1;
  f32x4 hd[R][NBO];
  layer_lds<NBH, NBO, R, WAVES, SLOT, 3 * NBO * 4, KPB, TQH, 0, true>(w.whd + (int64_t)e * NBH * NBO * 256, hcur, hd,
                                                                     lds, wv, lane, w.bhd + (int64_t)e * 3 * NBO * 16,
                                                                     lds_bias, par);
#else
  layer_lds<KG0, NBH, R, WAVES, SLOT, NBH * 4, 1, TQ0>(w.w0 + (int64_t)e * KG0 * NBH * 256, x0, acc, lds, wv, lane,
                                                     w.b0 + e * hp, lds_bias);
  bias_swish<NBH, R>(lds_bias, acc, hcur, g);
  for (int l = 0; l < 3; ++l) {  // hidden layers 1..3 (constructor.py:31-33)
    layer_lds<NBH, NBH, R, WAVES, SLOT, NBH * 4, KPB, TQH>(w.wh + ((int64_t)l * w.E + e) * NBH * NBH * 256, hcur, acc, lds,
                                                     wv, lane, w.bh + ((int64_t)l * w.E + e) * hp, lds_bias);
    bias_swish<NBH, R>(lds_bias, acc, hcur, g);
  }
  // ---- heads on the 4th hidden output (bnn.py:661-667): n < D mean, D <= n < 2D log-var
  f32x4 hd[R][NBO];
  layer_lds<NBH, NBO, R, WAVES, SLOT, 3 * NBO * 4, KPB, TQH>(w.whd + (int64_t)e * NBH * NBO * 256, hcur, hd, lds, wv, lane,
                                                       w.bhd + (int64_t)e * 3 * NBO * 16, lds_bias);

#endif

#ifndef BNN_KNOB_NOHEAD
#pragma unroll
  for (int r = 0; r < R; ++r)
    head_epilogue<NBO, MODE>(w, a, hd[r], e, row0 + r * 16 + m, count, g, lds_bias, sel_e[r]);
#else
  if (hd[0][0][0] == 12345.f) a.pen_bits[0] = 1;
#endif
  (void)D;
}

// ---- bf16 forward: weights/activations as P bf16 parts, f32 accumulate and f32 epilogues.
// P = 1 (dtype 1): bf16.  P = 2 (dtype 2, "bf16x3"): 3 products per k-group, ~17 significand bits.
// P = 3 (dtype 3, "bf16x6"): 6 products, f32-accurate (mlp_tile.h split_bf16 / layer_lds_split).
// NB2 = hidden blocks rounded up to even (k-groups of 32 pair two accumulator blocks).
#ifndef BNN_SPLIT_HOLD_F32
#define BNN_SPLIT_HOLD_F32 1  // hold split activations in f32 (P = 3 scratch spill 64 -> 20 B/lane)
#endif
#ifndef BNN_SPLIT_MINB
#define BNN_SPLIT_MINB 3  // split kernels (P > 1): 4-wave workgroups per CU (3: 168 VGPRs; P = 3 spills 15, still 4 % faster than 2)
#endif
template <int NB2, int NBO, int MODE, int WAVES, int P = 1, int PS = 1, int NBU = NB2>
__global__ __launch_bounds__(WAVES * 64, P > 1 ? (NB2 > 16 ? 1 : BNN_SPLIT_MINB * 4 / WAVES) : 512 / (WAVES * 64)) void bnn_fwd_bf16_kernel(
    const BnnDev w, const FwdArgs a) {
  constexpr int KG = NB2 / 2;
  // 16-deep MFMAs for a half-padded last k-group (as the f16x3 kernel does) measured slower here: the
  // larger unrolled body stops the part loops from unrolling (C3 -4 %, bf16x6 70x via dynamic indexing)
  constexpr bool KH = false;
  constexpr int NBMAX = NB2 > NBO ? NB2 : NBO;
  constexpr int SLOT = Stage<PS * NBMAX, WAVES>::SLOTS * 256;
  constexpr int BIAS_LDS = (NB2 * 4 + 63) / 64 * 256;  // the layer's bias (stage_bias pieces)
  __shared__ __attribute__((aligned(16))) float lds[2 * SLOT + BIAS_LDS];  // one array (see layer_lds)
  float* lds_bias = lds + 2 * SLOT;
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), m = lane & 15, g = lane >> 4;
  const int64_t count = a.d_count ? (int64_t)*a.d_count : a.B;
  const int groups = ceil_div(a.ntiles, WAVES);
  // member-major over the grid; or (a.xcd_members, E % 8 == 0) XCD x owns members x, x + 8, ... (workgroup b
  // runs on XCD b mod 8), member-major within the XCD.  C5 bf16 (E = 32, H = 400, 125k rows): 20.45 vs 20.42M
  // transitions/s member-major over the grid; row-group-major within the XCD (a row group's inputs read once
  // per XCD) 19.3M (same box, profiles/r06_c5_bf16_order_ab.txt)
  int e, grp;
  if (a.xcd_members) {   // member-major within the XCD: each owned member's weights are fetched into ONE L2
    // a.xcd_members = IW > 1: the XCD's members run IW at a time, interleaved per row group (its inputs read
    // once per IW members instead of once per member)
    const int j = blockIdx.x >> 3, iw = a.xcd_members;
    const int ph = j / (iw * groups), r = j % (iw * groups);
    e = (blockIdx.x & 7) + 8 * (iw * ph + r % iw);
    grp = r / iw;
  } else {
    e = blockIdx.x / groups;
    grp = blockIdx.x % groups;
  }
  const int64_t row = (int64_t)(grp * WAVES + wv) * 16 + m;
  if (grp >= groups || (int64_t)grp * WAVES * 16 >= count) return;
  const int IN = w.IN, O = w.O;
  const bool ok = row < count;
  bf16x8 x0[P][1];
  auto put = [&](bf16x8 (&dst)[P][KG], int c, int j, float v) {
    short parts[P];
    split_bf16<P>(v, parts);
#pragma unroll
    for (int p = 0; p < P; ++p) dst[p][c][j] = parts[p];
  };
  (void)put;
  auto put0 = [&](int j, float v) {
    short parts[P];
    split_bf16<P>(v, parts);
#pragma unroll
    for (int p = 0; p < P; ++p) x0[p][0][j] = parts[p];
  };
  if (a.xs) {  // rollout: the actor already wrote the scaled row in slot order (bf16_kperm)
    const f32x4 lo = ok ? ld4(a.xs + row * XS_STRIDE + 4 * g) : zero4();
    const f32x4 hi = ok ? ld4(a.xs + row * XS_STRIDE + 16 + 4 * g) : zero4();
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      put0(t, lo[t]);
      put0(4 + t, hi[t]);
    }
  } else
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = slot_feat(bf16_kperm(g, j), IN);
    float v = 0.f;
    if (ok && k >= 0) {
      float raw = k < O ? load_feat(a.in.xa, a.in.xa_f64, row * a.in.sa + k)
                        : load_feat(a.in.xb, a.in.xb_f64, row * a.in.sb + (k - O));
      v = (raw - w.mu[k]) / w.sigma[k];
    }
    put0(j, v);
  }
  const int64_t bs = w.BS;
  f32x4 acc[NB2];
  bf16x8 hin[P][KG];
  // P = 3: split activations held in f32, parts made per k-group (P = 2's parts take no more VGPRs)
  constexpr bool HOLD = BNN_SPLIT_HOLD_F32 && P >= 3;
  float hf[KG][8];
  (void)hf;
  // Epilogue in the log2 domain, as in bnn_fwd_f16s_kernel: the packed biases carry -log2(e), a layer's
  // input is y' = -log2(e) y, so u = -log2(e) t = acc + b' (layer 0, whose input is x: acc * -log2(e) + b')
  // and the output y' = u / (1 + 2^u); the head's accumulators are taken back by -ln 2.
  auto to_input = [&](const float* b, float f) {  // bias + swish in f32, then the bf16 B operand parts
#pragma unroll
    for (int c = 0; c < KG; ++c) {
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(b + (2 * c) * 16 + 4 * g);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(b + (2 * c + 1) * 16 + 4 * g);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const bool pad = 2 * c + 1 >= NBU;  // padding block (odd hidden-block count): zero
        (void)pad;
        if constexpr (P > 1) {
          if constexpr (HOLD) {
            hf[c][t] = swish_log2(fmaf(acc[2 * c][t], f, b0[t]));
            hf[c][4 + t] = pad ? 0.f : swish_log2(fmaf(acc[2 * c + 1][t], f, b1[t]));
          } else {
            put(hin, c, t, swish_log2(fmaf(acc[2 * c][t], f, b0[t])));
            put(hin, c, 4 + t, pad ? 0.f : swish_log2(fmaf(acc[2 * c + 1][t], f, b1[t])));
          }
          continue;
        }
#if defined(BNN_KNOB_CHEAPSWISH)
        hin[0][c][t] = to_bf16(acc[2 * c][t] * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(acc[2 * c][t])));
        hin[0][c][4 + t] = to_bf16(acc[2 * c + 1][t] * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(acc[2 * c + 1][t])));
#elif !defined(BNN_KNOB_NOSWISH)
        hin[0][c][t] = to_bf16(swish_log2(fmaf(acc[2 * c][t], f, b0[t])));
        hin[0][c][4 + t] = pad ? (short)0 : to_bf16(swish_log2(fmaf(acc[2 * c + 1][t], f, b1[t])));
#else
        hin[0][c][t] = to_bf16(acc[2 * c][t] + b0[t]);
        hin[0][c][4 + t] = to_bf16(acc[2 * c + 1][t] + b1[t]);
#endif
      }
    }
  };
  constexpr float kNegLog2e = -1.4426950408889634f, kNegLn2 = -0.6931471805599453f;
  const float* b0g = w.b0 + e * bs;
  if constexpr (P == 1) {
    layer_lds_bf16<1, NB2, WAVES, SLOT, NBU>(w.w0b + (int64_t)e * NB2 * 256, x0[0], acc, lds, wv, lane, b0g, lds_bias);
  } else {
    layer_lds_split<1, NB2, WAVES, SLOT, P, PS, false, NBU>(w.w0b + (int64_t)e * P * NB2 * 256, x0, acc, lds, wv, lane,
                                                            b0g, lds_bias);
  }
  to_input(lds_bias, kNegLog2e);
  for (int l = 0; l < 3; ++l) {
    const float* wl = w.whb + ((int64_t)l * w.E + e) * KG * P * NB2 * 256;
    const float* bl = w.bh + ((int64_t)l * w.E + e) * bs;
    if constexpr (P == 1)
      layer_lds_bf16<KG, NB2, WAVES, SLOT, NBU, KH>(wl, hin[0], acc, lds, wv, lane, bl, lds_bias);
    else if constexpr (HOLD)
      layer_lds_split_f32<KG, NB2, WAVES, SLOT, P, PS, false, NBU, KH>(wl, hf, acc, lds, wv, lane, 1.f, bl, lds_bias);
    else
      layer_lds_split<KG, NB2, WAVES, SLOT, P, PS, false, NBU, KH>(wl, hin, acc, lds, wv, lane, bl, lds_bias);
    to_input(lds_bias, 1.f);
  }
  f32x4 hd[NBO];
  if constexpr (P == 1) {
    layer_lds_bf16<KG, NBO, WAVES, SLOT, NBO, KH>(w.whdb + (int64_t)e * KG * NBO * 256, hin[0], hd, lds, wv, lane);
  } else {
    if constexpr (HOLD)
      layer_lds_split_f32<KG, NBO, WAVES, SLOT, P, PS, false, NBO, KH>(w.whdb + (int64_t)e * KG * P * NBO * 256, hf, hd,
                                                                        lds, wv, lane);
    else
      layer_lds_split<KG, NBO, WAVES, SLOT, P, PS, false, NBO, KH>(w.whdb + (int64_t)e * KG * P * NBO * 256, hin, hd,
                                                                    lds, wv, lane);
  }
#pragma unroll
  for (int nb = 0; nb < NBO; ++nb) hd[nb] *= kNegLn2;  // the head's input is y' = -log2(e) y
  head_epilogue<NBO, MODE>(w, a, hd, e, row, count, g, w.bhd + (int64_t)e * 3 * NBO * 16,
                           (MODE == FWD_ROLLOUT && a.sel && ok) ? a.sel[row] : -1);
}

// ---- f16x3 forward: f32 operands as 2 fp16 parts under power-of-two scales (mlp_tile.h
// split_f16_scaled / row_scale), 3 products per k-group on v_mfma_f32_16x16x32_f16, f32 accumulate and
// f32 epilogues.  Each layer's output is acc * (2^-k_w / s_row): the weight scale of the layer and
// member, the row scale of the layer's input (both exact powers of two), folded into the bias add.
#ifndef BNN_F16_XCD
#define BNN_F16_XCD 1
#endif
#ifndef BNN_F16_MINB_WIDE
#define BNN_F16_MINB_WIDE 1  // H = 400 (NB2 = 26): workgroups per CU the f16s kernel's registers are capped for
#endif
#ifndef BNN_F16_MINB
#define BNN_F16_MINB 2  // 4-wave workgroups per CU: 2 (170 VGPRs, no scratch) measured 0.5 % faster than 3 (28 B/lane spill)
#endif
template <int NB2, int NBO, int MODE, int WAVES, int PS = 1, int NBU = NB2>
__global__ __launch_bounds__(WAVES * 64, NB2 > 16 ? BNN_F16_MINB_WIDE : BNN_F16_MINB * 4 / WAVES) void bnn_fwd_f16s_kernel(
    const BnnDev w, const FwdArgs a) {
  constexpr int P = 2, KG = NB2 / 2;
  constexpr bool KH = NBU < NB2;  // the hidden layers' last k-group is half padding: 16-deep MFMAs there
  constexpr int NBMAX = NB2 > NBO ? NB2 : NBO;
  constexpr int SLOT = Stage<PS * NBMAX, WAVES>::SLOTS * 256;
  constexpr int BIAS_LDS = (NB2 * 4 + 63) / 64 * 256;  // the layer's bias (stage_bias pieces)
  __shared__ __attribute__((aligned(16))) float lds[2 * SLOT + BIAS_LDS];  // one array (see layer_lds)
  float* lds_bias = lds + 2 * SLOT;
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), m = lane & 15, g = lane >> 4;
  const int64_t count = a.d_count ? (int64_t)*a.d_count : a.B;
  const int groups = ceil_div(a.ntiles, WAVES);
#if BNN_F16_XCD
  // XCD-aware order: workgroups are dealt round-robin over the 8 XCDs; XCD x takes row groups
  // [x C, (x + 1) C) of every member, member-major, so a row group's input is fetched from HBM once
  // and re-read from that XCD's L2 by the other members (grid = 8 C E, see launch_f16s)
  const int C = ceil_div(groups, 8);
  const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
  const int e = j / C, grp = xcd * C + j % C;
  if (grp >= groups) return;
#else
  const int e = blockIdx.x / groups, grp = blockIdx.x % groups;
#endif
  const int64_t row = (int64_t)(grp * WAVES + wv) * 16 + m;
  if ((int64_t)grp * WAVES * 16 >= count) return;
  const int IN = w.IN, O = w.O, E = w.E;
  const bool ok = row < count;
  // the row's max |v| over the lane group's 8-per-k-group values -> the 4 lanes of row m (g = 0..3)
  auto row_max = [&](float mx) {
    mx = fmaxf(mx, __shfl_xor(mx, 16));
    return fmaxf(mx, __shfl_xor(mx, 32));
  };

  float xv[8];
  if (a.xs) {  // rollout: the actor already wrote the scaled row in slot order (bf16_kperm)
    const f32x4 lo = ok ? ld4(a.xs + row * XS_STRIDE + 4 * g) : zero4();
    const f32x4 hi = ok ? ld4(a.xs + row * XS_STRIDE + 16 + 4 * g) : zero4();
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      xv[t] = lo[t];
      xv[4 + t] = hi[t];
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = slot_feat(bf16_kperm(g, j), IN);
      float v = 0.f;
      if (ok && k >= 0) {
        float raw = k < O ? load_feat(a.in.xa, a.in.xa_f64, row * a.in.sa + k)
                          : load_feat(a.in.xb, a.in.xb_f64, row * a.in.sb + (k - O));
        v = (raw - w.mu[k]) / w.sigma[k];
      }
      xv[j] = v;
    }
  }
  float mx = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) mx = fmaxf(mx, fabsf(xv[j]));
  float sc, inv_row;
  row_scale(row_max(mx), sc, inv_row);
  bf16x8 x0[P][1];
  {
    u32x4v h4, l4;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const F16Pair pr = split_f16_pair(xv[2 * q], xv[2 * q + 1], sc);
      h4[q] = pr.hi;
      l4[q] = pr.lo;
    }
    x0[0][0] = __builtin_bit_cast(bf16x8, h4);
    x0[1][0] = __builtin_bit_cast(bf16x8, l4);
  }
  const int64_t bs = w.BS;
  f32x4 acc[NB2];
  // the activations are held in f32 and each k-group's fp16 parts made when it is consumed
  // (layer_lds_split_f32): holding both parts would take 168 VGPRs and spill at H = 200
  float hf[KG][8];
  float s_in = 1.f;  // the held activations' row scale
  // Epilogue in the log2 domain: u = -log2(e) t = acc * f + b' (f and the packed biases b' carry the
  // factor), and the layer output is held as y' = u / (1 + 2^u) = -log2(e) swish(t) (fc.py:21); the next
  // layer's scale takes the -ln 2 back (its f has no -log2(e) factor, the head's f gets -ln 2), which
  // saves one multiply per value.  Then the row scale of y' (the next layer's input).
  auto to_input = [&](const float* b, float f) {
    float mx = 0.f;
#pragma unroll
    for (int c = 0; c < KG; ++c) {
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(b + (2 * c) * 16 + 4 * g);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(b + (2 * c + 1) * 16 + 4 * g);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        hf[c][t] = swish_log2(fmaf(acc[2 * c][t], f, b0[t]));
        // an odd hidden-block count leaves the last block all padding: zero, not computed
        hf[c][4 + t] = 2 * c + 1 < NBU ? swish_log2(fmaf(acc[2 * c + 1][t], f, b1[t])) : 0.f;
        mx = fmaxf(mx, fmaxf(fabsf(hf[c][t]), fabsf(hf[c][4 + t])));
      }
    }
    row_scale(row_max(mx), s_in, inv_row);
  };
  // the bias of each hidden layer rides into LDS with the layer's first slice (lds_bias)
  layer_lds_split<1, NB2, WAVES, SLOT, P, PS, true, NBU>(w.w0b + (int64_t)e * P * NB2 * 256, x0, acc, lds, wv, lane,
                                                         w.b0 + e * bs, lds_bias);
  constexpr float kNegLog2e = -1.4426950408889634f, kNegLn2 = -0.6931471805599453f;
  to_input(lds_bias, inv_row * w.wscale[e] * kNegLog2e);  // layer 0's input is x itself
  for (int l = 0; l < 3; ++l) {
    layer_lds_split_f32<KG, NB2, WAVES, SLOT, P, PS, true, NBU, KH>(w.whb + ((int64_t)l * E + e) * KG * P * NB2 * 256, hf, acc,
                                                                lds, wv, lane, s_in, w.bh + ((int64_t)l * E + e) * bs,
                                                                lds_bias);
    to_input(lds_bias, inv_row * w.wscale[(1 + l) * E + e]);
  }
  f32x4 hd[NBO];
  layer_lds_split_f32<KG, NBO, WAVES, SLOT, P, PS, true, NBO, KH>(w.whdb + (int64_t)e * KG * P * NBO * 256, hf, hd, lds,
                                                                  wv, lane, s_in);
  const float f = inv_row * w.wscale[4 * E + e] * kNegLn2;  // the head's input is y' = -log2(e) y
#pragma unroll
  for (int nb = 0; nb < NBO; ++nb) hd[nb] *= f;
  head_epilogue<NBO, MODE>(w, a, hd, e, row, count, g, w.bhd + (int64_t)e * 3 * NBO * 16,
                           (MODE == FWD_ROLLOUT && a.sel && ok) ? a.sel[row] : -1);
}

// ---- f16x3 forward at H = 400 in column halves (bnn_fwd_f16h_kernel): bnn_fwd_f16s_kernel's arithmetic, product
// for product, with every layer's output blocks computed in two passes over the layer's input (blocks [0, NHA)
// then [NHA, NB2), each pass streaming its half of every weight slice), so only one half's accumulators are
// live beside the other's results: 2 workgroups per CU (256 registers) instead of 1 (376).  The input row's
// split is the same split_f16_pair under the same row scale (made inside the layer as for the hidden layers).
#ifndef BNN_F16_HALF
#define BNN_F16_HALF 1  // 1: H = 400 f16x3 runs bnn_fwd_f16h_kernel; 0: bnn_fwd_f16s_kernel
#endif
#ifndef BNN_F16H_MINB
#define BNN_F16H_MINB 2
#endif
#ifndef BNN_BF16_XCDMEM
#define BNN_BF16_XCDMEM 1  // bnn_fwd_bf16_kernel, E % 8 == 0: XCD-owned members (member-major within the XCD; > 1: that many interleaved)
#endif
#ifndef BNN_F16H_XCDMEM
#define BNN_F16H_XCDMEM 1  // E % 8 == 0: each XCD owns E / 8 members (their weights fetched into one L2)
#endif
template <int NB2, int NBO, int MODE, int WAVES, int NBU>
__global__ __launch_bounds__(WAVES * 64, BNN_F16H_MINB * 4 / WAVES) void bnn_fwd_f16h_kernel(const BnnDev w,
                                                                                          const FwdArgs a) {
  constexpr int P = 2, KG = NB2 / 2;
  constexpr bool KH = NBU < NB2;  // the hidden layers' last k-group is half padding: 16-deep MFMAs there
  constexpr int NHA = NB2 / 2, NHB = NB2 - NHA, NHBU = NBU - NHA;
  constexpr int NBMAX = NHB > NBO ? NHB : NBO;
  constexpr int SLOT = Stage<NBMAX, WAVES>::SLOTS * 256;
  constexpr int BIAS_LDS = (NB2 * 4 + 63) / 64 * 256;
  __shared__ __attribute__((aligned(16))) float lds[2 * SLOT + BIAS_LDS];  // one array (see layer_lds)
  float* lds_bias = lds + 2 * SLOT;
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), g = lane >> 4;
  const int m = lane & 15;
  const int64_t count = a.d_count ? (int64_t)*a.d_count : a.B;
  const int groups = ceil_div(a.ntiles, WAVES);
  const int IN = w.IN, O = w.O, E = w.E;
  // XCD-owned members (E % 8 == 0, launch_f16s): XCD x runs members x, x + 8, ... over EVERY row group,
  // member-major, so each member's weights are fetched into ONE XCD's L2 (the row groups stream past them).
  // Otherwise the XCD-aware order of bnn_fwd_f16s_kernel: XCD x takes row groups [x C, (x + 1) C) of every
  // member.  (A workgroup looping over its XCD's members with the rows in registers spilled 145-197 VGPRs.)
  const bool own = a.xcd_members != 0;
  const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
  const int C = ceil_div(groups, 8);
  const int e = own ? xcd + 8 * (j / groups) : j / C;
  const int grp = own ? j % groups : xcd * C + j % C;
  if (grp >= groups || e >= E) return;
  const int row = (grp * WAVES + wv) * 16 + m;   // < 2^31 (B <= max_batch)
  if ((int64_t)grp * WAVES * 16 >= count) return;
  const bool ok = row < count;
  auto row_max = [&](float mx) {
    mx = fmaxf(mx, __shfl_xor(mx, 16));
    return fmaxf(mx, __shfl_xor(mx, 32));
  };
  float s_in, inv_row;
  const int64_t bs = w.BS;
  f32x4 accA[NHA], accB[NHB];
  float hf[KG][8];
  // the two passes of a layer (the bias, all NB2 * 16 values, rides with pass A's first slice)
  auto layer2 = [&](const float* wl, const auto& in, auto kgc, const float* bias) {
    constexpr int KGL = decltype(kgc)::value;
    constexpr bool KHL = KGL > 1 && KH;
    layer_lds_split_f32<KGL, NHA, WAVES, SLOT, P, 1, true, NHA, KHL, NB2, NB2 * 4>(wl, in, accA, lds, wv, lane, s_in,
                                                                                  bias, lds_bias);
    layer_lds_split_f32<KGL, NHB, WAVES, SLOT, P, 1, true, NHBU, KHL, NB2>(wl + NHA * 256, in, accB, lds, wv, lane,
                                                                           s_in);
  };
  // block bi of the layer's output -> values (bi & 1) * 4 + t of k-group bi / 2 of the next input
  auto to_input = [&](const float* b, float f) {
    float mxv = 0.f;
#pragma unroll
    for (int bi = 0; bi < NHA; ++bi) {
      const f32x4 bb = *reinterpret_cast<const f32x4*>(b + bi * 16 + 4 * g);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float y = swish_log2(fmaf(accA[bi][t], f, bb[t]));
        hf[bi / 2][(bi & 1) * 4 + t] = y;
        mxv = fmaxf(mxv, fabsf(y));
      }
    }
#pragma unroll
    for (int bi = NHA; bi < NB2; ++bi) {
      const f32x4 bb = *reinterpret_cast<const f32x4*>(b + bi * 16 + 4 * g);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        // an odd hidden-block count leaves the last block all padding: zero, not computed
        const float y = bi < NBU ? swish_log2(fmaf(accB[bi - NHA][t], f, bb[t])) : 0.f;
        hf[bi / 2][(bi & 1) * 4 + t] = y;
        mxv = fmaxf(mxv, fabsf(y));
      }
    }
    row_scale(row_max(mxv), s_in, inv_row);
  };
  constexpr float kNegLog2e = -1.4426950408889634f, kNegLn2 = -0.6931471805599453f;
  float x1[1][8];
  if (a.xs) {
    const f32x4 lo = ok ? ld4(a.xs + (int64_t)row * XS_STRIDE + 4 * g) : zero4();
    const f32x4 hi = ok ? ld4(a.xs + (int64_t)row * XS_STRIDE + 16 + 4 * g) : zero4();
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      x1[0][t] = lo[t];
      x1[0][4 + t] = hi[t];
    }
  } else {
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const int k = slot_feat(bf16_kperm(g, jj), IN);
      float v = 0.f;
      if (ok && k >= 0) {
        float raw = k < O ? load_feat(a.in.xa, a.in.xa_f64, (int64_t)row * a.in.sa + k)
                          : load_feat(a.in.xb, a.in.xb_f64, (int64_t)row * a.in.sb + (k - O));
        v = (raw - w.mu[k]) / w.sigma[k];
      }
      x1[0][jj] = v;
    }
  }
  float mx = 0.f;
#pragma unroll
  for (int jj = 0; jj < 8; ++jj) mx = fmaxf(mx, fabsf(x1[0][jj]));
  row_scale(row_max(mx), s_in, inv_row);
  layer2(w.w0b + (int64_t)e * P * NB2 * 256, x1, std::integral_constant<int, 1>{}, w.b0 + e * bs);
  to_input(lds_bias, inv_row * w.wscale[e] * kNegLog2e);  // layer 0's input is x itself
  for (int l = 0; l < 3; ++l) {
    layer2(w.whb + ((int64_t)l * E + e) * KG * P * NB2 * 256, hf, std::integral_constant<int, KG>{},
           w.bh + ((int64_t)l * E + e) * bs);
    to_input(lds_bias, inv_row * w.wscale[(1 + l) * E + e]);
  }
  f32x4 hd[NBO];
  layer_lds_split_f32<KG, NBO, WAVES, SLOT, P, 1, true, NBO, KH>(w.whdb + (int64_t)e * KG * P * NBO * 256, hf, hd,
                                                                 lds, wv, lane, s_in);
  const float f = inv_row * w.wscale[4 * E + e] * kNegLn2;  // the head's input is y' = -log2(e) y
#pragma unroll
  for (int nb = 0; nb < NBO; ++nb) hd[nb] *= f;
  // the row index again from a fresh lane id (v_mbcnt in volatile asm: not merged with the one at the top), so
  // no row value lives across the layers -- kept live, it was the value spilled (8 B per lane in rollout mode)
  int lane_e;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane_e));
  const int64_t row_e = (int64_t)((grp * WAVES + __builtin_amdgcn_readfirstlane(wv)) * 16 + (lane_e & 15));
  const bool ok_e = row_e < count;
  head_epilogue<NBO, MODE>(w, a, hd, e, row_e, count, g, w.bhd + (int64_t)e * 3 * NBO * 16,
                           (MODE == FWD_ROLLOUT && a.sel && ok_e) ? a.sel[row_e] : -1);
}

// ---- f16x3 forward over R row blocks per wave (R = 2: 32 rows per wave, 128 per 4-wave workgroup, one
// workgroup per CU with the accumulators in AGPRs): bnn_fwd_f16s_kernel's arithmetic, product for
// product, with each LDS weight fragment feeding R row blocks (layer_f16_rows).
#ifndef BNN_F16_R
#define BNN_F16_R 0  // 0: bnn_fwd_f16s_kernel; R >= 1: bnn_fwd_f16r_kernel<R> (H <= 256)
#endif
#ifndef BNN_F16R_WAVES
#define BNN_F16R_WAVES 4
#endif
template <int NB2, int NBO, int MODE, int WAVES, int R, int NBU = NB2>
__global__ __launch_bounds__(WAVES * 64, R == 1 ? 2 : 1) void bnn_fwd_f16r_kernel(const BnnDev w, const FwdArgs a) {
  constexpr int KG = NB2 / 2;
  constexpr bool KH = NBU < NB2;
  constexpr int NBMAX = NB2 > NBO ? NB2 : NBO;
  constexpr int SLOT = Stage<NBMAX, WAVES>::SLOTS * 256;
  constexpr int BIAS_LDS = (NB2 * 4 + 63) / 64 * 256;
  __shared__ __attribute__((aligned(16))) float lds[2 * SLOT + BIAS_LDS];
  float* lds_bias = lds + 2 * SLOT;
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), m = lane & 15, g = lane >> 4;
  const int64_t count = a.d_count ? (int64_t)*a.d_count : a.B;
  const int groups = ceil_div(a.ntiles, WAVES);  // ntiles: tiles of 16 R rows
  const int C = ceil_div(groups, 8);             // XCD-aware order (bnn_fwd_f16s_kernel)
  const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
  const int e = j / C, grp = xcd * C + j % C;
  if (grp >= groups) return;
  const int64_t row0 = (int64_t)(grp * WAVES + wv) * 16 * R + m;  // row block r: row0 + 16 r
  if ((int64_t)grp * WAVES * 16 * R >= count) return;
  const int IN = w.IN, E = w.E, O = w.O;
  auto row_max = [&](float mx) {
    mx = fmaxf(mx, __shfl_xor(mx, 16));
    return fmaxf(mx, __shfl_xor(mx, 32));
  };
  float xin[R][1][8], sc[R], inv[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t row = row0 + 16 * r;
    const bool ok = row < count;
    if (a.xs) {
      const f32x4 lo = ok ? ld4(a.xs + row * XS_STRIDE + 4 * g) : zero4();
      const f32x4 hi = ok ? ld4(a.xs + row * XS_STRIDE + 16 + 4 * g) : zero4();
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        xin[r][0][t] = lo[t];
        xin[r][0][4 + t] = hi[t];
      }
    } else {
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const int k = slot_feat(bf16_kperm(g, jj), IN);
        float v = 0.f;
        if (ok && k >= 0) {
          float raw = k < O ? load_feat(a.in.xa, a.in.xa_f64, row * a.in.sa + k)
                            : load_feat(a.in.xb, a.in.xb_f64, row * a.in.sb + (k - O));
          v = (raw - w.mu[k]) / w.sigma[k];
        }
        xin[r][0][jj] = v;
      }
    }
    float mx = 0.f;
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) mx = fmaxf(mx, fabsf(xin[r][0][jj]));
    row_scale(row_max(mx), sc[r], inv[r]);
  }
  const int64_t bs = w.BS;
  f32x4 acc[R][NB2];
  float hf[R][KG][8];
  constexpr float kNegLog2e = -1.4426950408889634f, kNegLn2 = -0.6931471805599453f;
  // bias + swish_log2 (bnn_fwd_f16s_kernel's to_input) of row block r, then its new row scale
  auto to_input = [&](int r, const float* b, float f) {
    float mx = 0.f;
#pragma unroll
    for (int c = 0; c < KG; ++c) {
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(b + (2 * c) * 16 + 4 * g);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(b + (2 * c + 1) * 16 + 4 * g);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        hf[r][c][t] = swish_log2(fmaf(acc[r][2 * c][t], f, b0[t]));
        hf[r][c][4 + t] = 2 * c + 1 < NBU ? swish_log2(fmaf(acc[r][2 * c + 1][t], f, b1[t])) : 0.f;
        mx = fmaxf(mx, fmaxf(fabsf(hf[r][c][t]), fabsf(hf[r][c][4 + t])));
      }
    }
    row_scale(row_max(mx), sc[r], inv[r]);
  };
  // each layer's first slice is prefetched during the previous layer's last one (every layer has an
  // even slice count: the prefetch lands in buffer 0, where the next layer starts)
  auto whl = [&](int l) { return w.whb + ((int64_t)l * E + e) * KG * 2 * NB2 * 256; };
  const float* whd = w.whdb + (int64_t)e * KG * 2 * NBO * 256;
  layer_f16_rows<1, NB2, R, WAVES, SLOT, NBU, false, NB2>(w.w0b + (int64_t)e * 2 * NB2 * 256, xin, acc, lds, wv, lane, sc,
                                                          w.b0 + e * bs, lds_bias, whl(0));
#pragma unroll
  for (int r = 0; r < R; ++r) to_input(r, lds_bias, inv[r] * w.wscale[e] * kNegLog2e);
#pragma unroll
  for (int l = 0; l < 2; ++l) {
    layer_f16_rows<KG, NB2, R, WAVES, SLOT, NBU, KH, NB2, true>(whl(l), hf, acc, lds, wv, lane, sc,
                                                                w.bh + ((int64_t)l * E + e) * bs, lds_bias, whl(l + 1));
#pragma unroll
    for (int r = 0; r < R; ++r) to_input(r, lds_bias, inv[r] * w.wscale[(1 + l) * E + e]);
  }
  layer_f16_rows<KG, NB2, R, WAVES, SLOT, NBU, KH, NBO, true>(whl(2), hf, acc, lds, wv, lane, sc,
                                                              w.bh + ((int64_t)2 * E + e) * bs, lds_bias, whd);
#pragma unroll
  for (int r = 0; r < R; ++r) to_input(r, lds_bias, inv[r] * w.wscale[3 * E + e]);
  f32x4 hd[R][NBO];
  layer_f16_rows<KG, NBO, R, WAVES, SLOT, NBO, KH, 0, true>(whd, hf, hd, lds, wv, lane, sc);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t row = row0 + 16 * r;
    const float f = inv[r] * w.wscale[4 * E + e] * kNegLn2;
#pragma unroll
    for (int nb = 0; nb < NBO; ++nb) hd[r][nb] *= f;
    head_epilogue<NBO, MODE>(w, a, hd[r], e, row, count, g, w.bhd + (int64_t)e * 3 * NBO * 16,
                             (MODE == FWD_ROLLOUT && a.sel && row < count) ? a.sel[row] : -1);
  }
}

// ---- ensemble forward over an LDS ring (bnn_fwd_ring_kernel): P = 2 is bnn_fwd_f16s_kernel's f16x3
// arithmetic (BNN_F16_RING), P = 1 bnn_fwd_bf16_kernel's single-bf16 arithmetic (BNN_BF16_RING), product
// for product, with the weight slices of all five layers as ONE stream (layer 0: P slices, each hidden
// layer and the head: P KG; a slice is one weight part of one 32-deep k-group).  Slice j + DEPTH - 1 is
// copied while slice j is consumed, so DEPTH - 1 slices are in flight across every barrier: the barrier is
// a raw s_barrier behind a counted `s_waitcnt vmcnt(N)` that retires only slice j's copies (N = the later
// slices' copies per wave; __syncthreads() would drain vmcnt(0)), and no layer starts on an exposed copy
// (the layer_lds_split_f32 path stages each layer's first slice behind a barrier of its own).  Layer 0's
// bias goes out ahead of the first slices, layer L's (L = 1..3) at the top of layer L - 1's first slice,
// into one of two bias slots (a layer of slice waits and barriers behind it at any depth).
#ifndef BNN_F16_RING
#define BNN_F16_RING 1
#endif
#ifndef BNN_BF16_RING
#define BNN_BF16_RING 0
#endif
#ifndef BNN_RING_DEPTH_F16
#define BNN_RING_DEPTH_F16 3  // 3 x 16 KB slots: 3 workgroups per CU
#endif
#ifndef BNN_RING_DEPTH_BF16
#define BNN_RING_DEPTH_BF16 3
#endif
#ifndef BNN_BF16X6_RING
#define BNN_BF16X6_RING 1   // bf16x6 (the exact 3-part split) on the ring kernel at H <= 256
#endif
#ifndef BNN_F16_FOLD
#define BNN_F16_FOLD 1   // with BNN_F16Q_DEFER: the ring kernel's row scale folded into the swish (bnn_fwd_ring_kernel)
#endif
#ifndef BNN_F16Q_DEFER
// 1: the swish of k-group c in the MFMA gaps of k-group c - 1 (see below).  Alone within noise of 0; with
// the folded scale (BNN_F16_FOLD) +1.4 % on the headline rollout (131.2 vs 129.4M/s, ensemble 0.331 vs
// 0.334 ms, same-box A/B, profiles/r04_ens_ab_fold.txt), so both are on
#define BNN_F16Q_DEFER 1
#endif

#ifndef BNN_RING_HEAD_MERGE
#define BNN_RING_HEAD_MERGE 1   // the head's weight parts of a k-group in one ring slice (bnn_fwd_ring_kernel)
#endif

#ifndef BNN_RING_PF
#define BNN_RING_PF 3   // ring kernel: fragment reads in flight ahead of the MFMAs (P = 1, 2)
#endif
#ifndef BNN_RING_PF_X6
#define BNN_RING_PF_X6 3   // the same for bf16x6 (5 and more spill at its 168-VGPR cap)
#endif
#ifndef BNN_RING_PIN
#define BNN_RING_PIN 1
#endif

#ifndef BNN_RING_WAVES
#define BNN_RING_WAVES 4  // waves per workgroup (16 rows each) sharing one ring
#endif
#ifndef BNN_RING_MINB
#define BNN_RING_MINB 3  // 4-wave workgroups per CU the ring kernel's registers are capped for (LDS admits 3)
#endif
#ifndef BNN_RING_MINB_X6
#define BNN_RING_MINB_X6 3  // the same for bf16x6 (P = 3)
#endif
template <int NB2, int NBO, int MODE, int WAVES, int P, int DEPTH, int NBU = NB2>
__global__ __launch_bounds__(WAVES * 64, ((P == 3 ? BNN_RING_MINB_X6 : BNN_RING_MINB) * 4 / WAVES > 0)
                                             ? (P == 3 ? BNN_RING_MINB_X6 : BNN_RING_MINB) * 4 / WAVES : 1) void bnn_fwd_ring_kernel(const BnnDev w,
                                                                                            const FwdArgs a) {
  static_assert(P == 1 || P == 2 || P == 3, "1: bf16, 2: f16x3, 3: bf16x6 (the exact 3-part bf16 split)");
  static_assert(DEPTH >= 3, "ring of at least 3 slots");
  constexpr bool F16 = P == 2;
  // the head's slices carry HPS weight parts each: all P of a k-group where they fit a hidden layer's slot
  // (its P NBO fragments are contiguous in the packing), so the narrow head runs behind KG barriers, not P KG
  constexpr int HPS = BNN_RING_HEAD_MERGE && Stage<P * NBO, WAVES>::SLOTS <= Stage<NB2, WAVES>::SLOTS ? P : 1;
  constexpr int KG = NB2 / 2, NS = P + 3 * KG * P + KG * (P / HPS);
  constexpr int JHEAD = P + 3 * KG * P;  // the head's first slice
  constexpr bool KH = NBU < NB2;
  constexpr int SLOT = Stage<(NB2 > HPS * NBO ? NB2 : HPS * NBO), WAVES>::SLOTS * 256;
  constexpr int BIAS_LDS = (NB2 * 4 + 63) / 64 * 256;
  // two bias slots: layer L's bias (slot L & 1) goes out at the top of layer L - 1's first slice, so it
  // has a whole layer of slice waits behind it whatever the depth
  __shared__ __attribute__((aligned(16))) float lds[DEPTH * SLOT + 2 * BIAS_LDS];  // one array (see layer_lds)
  float* lds_bias0 = lds + DEPTH * SLOT;
  // the wave index in an SGPR (uniform): it and the row base computed from it hold no VGPRs
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), m = lane & 15, g = lane >> 4;
  const int64_t count = a.d_count ? (int64_t)*a.d_count : a.B;
  const int groups = ceil_div(a.ntiles, WAVES);
  const int C = ceil_div(groups, 8);  // XCD-aware order (bnn_fwd_f16s_kernel)
  const int xcd = blockIdx.x & 7, jb = blockIdx.x >> 3;
  // uniform (SGPR) member: its weight scales come in by scalar loads, which leave vmcnt alone
  const int e = __builtin_amdgcn_readfirstlane(jb / C), grp = __builtin_amdgcn_readfirstlane(xcd * C + jb % C);
  if (grp >= groups) return;
  const int64_t row = (int64_t)(grp * WAVES + wv) * 16 + m;
  if ((int64_t)grp * WAVES * 16 >= count) return;
  const int IN = w.IN, O = w.O, E = w.E;
  const bool ok = row < count;
  auto row_max = [&](float mx) {
    mx = fmaxf(mx, __shfl_xor(mx, 16));
    return fmaxf(mx, __shfl_xor(mx, 32));
  };
  // slice stream: layer L (0 input, 1..3 hidden, 4 head) owns slices [P + P KG (L - 1), ...) (layer 0: [0, P))
  const float* src[5];
  src[0] = w.w0b + (int64_t)e * P * NB2 * 256;
#pragma unroll
  for (int l = 0; l < 3; ++l) src[1 + l] = w.whb + ((int64_t)l * E + e) * KG * P * NB2 * 256;
  src[4] = w.whdb + (int64_t)e * KG * P * NBO * 256;
  auto issue = [&](auto jc) {  // every wave's copies of slice J (PER per wave, pads re-read a fragment)
    constexpr int J = decltype(jc)::value;
    if constexpr (J < NS) {
      constexpr int L = J < P ? 0 : 1 + (J - P) / (P * KG);
      constexpr int NF = L == 4 ? HPS * NBO : NB2;
      constexpr int s = J - (L == 0 ? 0 : P + P * KG * (L - 1));
      stage_slice<NF, WAVES>(src[L] + s * NF * 256, lds + (J % DEPTH) * SLOT, wv, lane);
    }
  };
  const int64_t bs = w.BS;

  float xv[8];
  if (a.xs) {  // rollout: the actor already wrote the scaled row in slot order (bf16_kperm)
    const f32x4 lo = ok ? ld4(a.xs + row * XS_STRIDE + 4 * g) : zero4();
    const f32x4 hi = ok ? ld4(a.xs + row * XS_STRIDE + 16 + 4 * g) : zero4();
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      xv[t] = lo[t];
      xv[4 + t] = hi[t];
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = slot_feat(bf16_kperm(g, j), IN);
      float v = 0.f;
      if (ok && k >= 0) {
        float raw = k < O ? load_feat(a.in.xa, a.in.xa_f64, row * a.in.sa + k)
                          : load_feat(a.in.xb, a.in.xb_f64, row * a.in.sb + (k - O));
        v = (raw - w.mu[k]) / w.sigma[k];
      }
      xv[j] = v;
    }
  }
  // f16x3: the five layers' weight scales, loaded with the row and kept in SGPRs (a vector load of one
  // later would be waited for with vmcnt(0), draining the slices in flight); the input row's scale
  float wsc[5] = {1.f, 1.f, 1.f, 1.f, 1.f};
  float s_in = 1.f, inv_row = 1.f;
  if constexpr (F16) {
#pragma unroll
    for (int l = 0; l < 5; ++l) wsc[l] = w.wscale[l * E + e];
#pragma unroll
    for (int l = 0; l < 5; ++l) wsc[l] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(wsc[l])));
    float mx0 = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) mx0 = fmaxf(mx0, fabsf(xv[j]));
    row_scale(row_max(mx0), s_in, inv_row);
  }
  // the row is in registers before the first copies go out (a later first use of its loads would wait
  // for the copies too: vmcnt is in order)
  wait_vm_lgkm0<0>();
  __builtin_amdgcn_sched_barrier(0);
  stage_bias<NB2 * 4, WAVES>(w.b0 + e * bs, lds_bias0, wv, lane);   // layer 0's bias (slot 0), ahead of every slice
  RingRun<0, DEPTH - 1>::run([&](auto jc) { issue(jc); });

  constexpr float kNegLog2e = -1.4426950408889634f, kNegLn2 = -0.6931471805599453f;
  f32x4 acc[NB2 > NBO ? NB2 : NBO];
  float hf[KG][8];
  bf16x8 cur[P];
  // the bias is read with the fragments' type: read as f32x4, hipcc drained vmcnt(0) in front of it (the
  // slices in flight) as if it might alias the pending LDS-DMA writes
  const float* lds_bias = lds_bias0;   // the slot of the layer whose epilogue runs next
  auto bias4 = [&](int off) { return __builtin_bit_cast(f32x4, *reinterpret_cast<const bf16x8*>(lds_bias + off)); };
  // Deferred swish (BNN_F16Q_DEFER): the epilogue right after a layer only forms u = -log2(e) t = acc f + b'
  // (f16x3: and the row scale from max |u|; |y'| = |u| / (1 + 2^u) <= |u|, so y' s stays below 2^15), and
  // the activation y' = u / (1 + 2^u) of k-group c is made during the MFMAs of k-group c - 1 of the next
  // layer (its exp / rcp in the MFMA issue gaps).
  constexpr bool DEF = BNN_F16Q_DEFER;
  // Folded scale (BNN_F16_FOLD with the deferred swish, f16x3): the row scale already comes from max |u|
  // (|y'| = |u| / (1 + 2^u) <= |u|, so y' s stays below 2^15), so the swish produces y' s directly as
  // u / ((1 + 2^u) / s) -- its 1 + 2^u add becomes an fma with 1 / s -- and the split needs no multiply:
  // one VALU op per value less, in a kernel whose vector issue, not its MFMAs, is the bound
  constexpr bool FOLD = F16 && DEF && BNN_F16_FOLD;
  auto to_input = [&](float f) {
    float mx = 0.f;
#pragma unroll
    for (int c = 0; c < KG; ++c) {
      const f32x4 b0 = bias4((2 * c) * 16 + 4 * g);
      const f32x4 b1 = bias4((2 * c + 1) * 16 + 4 * g);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float u0 = fmaf(acc[2 * c][t], f, b0[t]);
        const float u1 = 2 * c + 1 < NBU ? fmaf(acc[2 * c + 1][t], f, b1[t]) : 0.f;
        hf[c][t] = DEF ? u0 : swish_log2(u0);
        // an odd hidden-block count leaves the last block all padding: zero, not computed
        hf[c][4 + t] = DEF || 2 * c + 1 >= NBU ? u1 : swish_log2(u1);
        if constexpr (F16) mx = fmaxf(mx, fmaxf(fabsf(hf[c][t]), fabsf(hf[c][4 + t])));
      }
    }
    if constexpr (F16) row_scale(row_max(mx), s_in, inv_row);
  };
  auto act = [&](int c, int j) {  // y' (FOLD: y' s) of value j of k-group c (the padding block stays 0)
    if (j < 4 || 2 * c + 1 < NBU) {
      const float u = hf[c][j];
      hf[c][j] = FOLD ? u * __builtin_amdgcn_rcpf(fmaf(__builtin_amdgcn_exp2f(u), inv_row, inv_row)) : swish_log2(u);
    }
  };
  // the operand parts of k-group kg of `in`: f16x3 the two scaled fp16 parts, bf16 the RN bf16 values
  // half: only values 0..3 feed the half-K MFMA of a layer's last k-group (KH); the rest are not split
  auto parts = [&](const float (&v)[8], auto prescaled, auto half) {
    if constexpr (F16) {
      u32x4v h4, l4;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (decltype(half)::value && q >= 2) {
          h4[q] = l4[q] = 0u;
          continue;
        }
        const F16Pair pr = decltype(prescaled)::value ? split_f16_pair_prescaled(v[2 * q], v[2 * q + 1])
                                                      : split_f16_pair(v[2 * q], v[2 * q + 1], s_in);
        h4[q] = pr.hi;
        l4[q] = pr.lo;
      }
      cur[0] = __builtin_bit_cast(bf16x8, h4);
      cur[P - 1] = __builtin_bit_cast(bf16x8, l4);
    } else if constexpr (P == 3) {   // the exact RN split (mlp_tile.h split_bf16_pair): x0 + x1 + x2 == x
      u32x4v p4[3];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (decltype(half)::value && q >= 2) {
#pragma unroll
          for (int k = 0; k < 3; ++k) p4[k][q] = 0u;
          continue;
        }
        uint32_t pr[3];
        split_bf16_pair<3>(v[2 * q], v[2 * q + 1], pr);
#pragma unroll
        for (int k = 0; k < 3; ++k) p4[k][q] = pr[k];
      }
#pragma unroll
      for (int k = 0; k < 3; ++k) cur[k] = __builtin_bit_cast(bf16x8, p4[k]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) cur[0][j] = to_bf16(v[j]);
    }
  };
  // layer L: NBL output blocks (NBUL used), KGL k-groups of input `in`, slices [J0, J0 + P KGL)
  auto layer = [&](auto Lc, auto& in) {
    constexpr int L = decltype(Lc)::value;
    constexpr int KGL = L == 0 ? 1 : KG, NBL = L == 4 ? NBO : NB2, NBUL = L == 4 ? NBO : NBU;
    constexpr bool KHL = L > 0 && KH;
    constexpr bool DEFER = DEF && L > 0;   // `in` holds u; y' made one k-group ahead
    constexpr int J0 = L == 0 ? 0 : P + P * KG * (L - 1);
    constexpr int PPS = L == 4 ? HPS : 1, SPK = P / PPS;   // weight parts per slice, slices per k-group
#pragma unroll
    for (int nb = 0; nb < NBL; ++nb) acc[nb] = zero4();
    if constexpr (DEFER) {
#pragma unroll
      for (int j = 0; j < 8; ++j) act(0, j);
    }
    RingRun<J0, J0 + SPK * KGL>::run([&](auto jc) {
      constexpr int J = decltype(jc)::value, s = J - J0, kg = s / SPK, p0 = (s % SPK) * PPS;
      // made when the k-group is first consumed (layers > 0 under FOLD hold y' s already)
      if constexpr (p0 == 0)
        parts(in[kg], std::integral_constant<bool, FOLD && (L > 0)>{}, std::integral_constant<bool, KHL && kg + 1 == KGL>{});
      // slice J landed (every later slice still in flight may stay so) ... for every wave, and every wave
      // is done with the buffer slice J + DEPTH - 1 goes into (slice J - 1's)
      constexpr int N = [] {
        int n = 0;
        for (int i = 1; i <= DEPTH - 2; ++i) n += (J + i >= NS ? 0 : (((J + i >= JHEAD) ? HPS * NBO : NB2) + WAVES - 1) / WAVES);
        return n;
      }();
      wait_vm_lgkm0<N>();
      __builtin_amdgcn_s_barrier();
      // the next layer's bias into slot (L + 1) & 1: every wave is past layer L - 1's epilogue, the last
      // reader of that slot
      if constexpr (s == 0 && L < 3)
        stage_bias<NB2 * 4, WAVES>(w.bh + ((int64_t)L * E + e) * bs, lds_bias0 + ((L + 1) & 1) * BIAS_LDS, wv, lane);
      issue(std::integral_constant<int, J + DEPTH - 1>{});
      __builtin_amdgcn_sched_barrier(0);
      const float* b = lds + (J % DEPTH) * SLOT;
      // fragment i = pp NBL + nb of the slice: weight part p0 + pp, output block nb
      auto frag = [&](int i) { return *reinterpret_cast<const bf16x8*>(b + (((i / NBUL) * NBL + i % NBUL) * 64 + lane) * 4); };
      // fragments read BNN_RING_PF ahead of their MFMAs, each read pinned ahead of the MFMAs that follow it
      // (left to itself the scheduler sinks it to just before its use: an exposed LDS latency per pair)
      constexpr int PF = P == 3 ? BNN_RING_PF_X6 : BNN_RING_PF, NFR = PPS * NBUL;
      bf16x8 fq[PF];
#pragma unroll
      for (int k = 0; k < PF; ++k)
        if (k < NFR) fq[k] = frag(k);
#pragma unroll
      for (int i = 0; i < NFR; ++i) {
        const int p = p0 + i / NBUL, nb = i % NBUL;
        const bf16x8 fr = fq[i % PF];
        if (i + PF < NFR) fq[i % PF] = frag(i + PF);
        if constexpr (BNN_RING_PIN) __builtin_amdgcn_sched_barrier(0x0406);   // VALU, SALU, transcendentals may cross
        // part p of W meets the activation parts q < P - p, the lowest first (the product order of
        // layer_lds_split_f32; bf16x6 with x0 first measured the same: 91.4-91.6 vs 91.2-91.6M/s)
#pragma unroll
        for (int q = P - 1 - p; q >= 0; --q)
          acc[nb] = (KHL && kg + 1 == KGL) ? mfma_16x16x16_lo<F16>(fr, cur[q], acc[nb])
                                           : mfma_16x16x32<F16>(fr, cur[q], acc[nb]);
        // the next k-group's activations, spread over this k-group's P slices: values V p .. V p + V - 1,
        // value v after fragment max((v + 1) NBUL / V - 1, 0) (V = ceil(8 / P) per slice)
        if constexpr (DEFER && kg + 1 < KGL) {
          constexpr int V = (8 + P - 1) / P;
#pragma unroll
          for (int v = 0; v < V; ++v)
            if (V * p + v < 8 && nb == ((v + 1) * NBUL / V - 1 > 0 ? (v + 1) * NBUL / V - 1 : 0)) act(kg + 1, V * p + v);
        }
      }
    });
  };
  {
    float x1[1][8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x1[0][j] = xv[j];
    layer(std::integral_constant<int, 0>{}, x1);
  }
  to_input(inv_row * wsc[0] * kNegLog2e);  // layer 0's input is x itself
  layer(std::integral_constant<int, 1>{}, hf);
  lds_bias = lds_bias0 + BIAS_LDS;
  to_input(inv_row * wsc[1]);
  layer(std::integral_constant<int, 2>{}, hf);
  lds_bias = lds_bias0;
  to_input(inv_row * wsc[2]);
  layer(std::integral_constant<int, 3>{}, hf);
  lds_bias = lds_bias0 + BIAS_LDS;
  to_input(inv_row * wsc[3]);
  layer(std::integral_constant<int, 4>{}, hf);
  f32x4 hd[NBO];
  const float f = inv_row * wsc[4] * kNegLn2;  // the head's input is y' = -log2(e) y
#pragma unroll
  for (int nb = 0; nb < NBO; ++nb) hd[nb] = acc[nb] * f;
  // the row index again from a fresh lane id (volatile asm: not merged with the one at the top), so no 64-bit
  // row value lives across the layers (bnn_fwd_f16h_kernel: it was the value spilled there)
  int lane_e;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane_e));
  const int64_t row_e = (int64_t)(grp * WAVES + wv) * 16 + (lane_e & 15);
  const bool ok_e = row_e < count;
  head_epilogue<NBO, MODE>(w, a, hd, e, row_e, count, g, w.bhd + (int64_t)e * 3 * NBO * 16,
                           (MODE == FWD_ROLLOUT && a.sel && ok_e) ? a.sel[row_e] : -1);
}

template <int NB2, int NBO, int P, int DEPTH>
static int launch_ring(const Bnn* h, int mode, FwdArgs a, hipStream_t s) {
  constexpr int WV = BNN_RING_WAVES;
  a.ntiles = (int)ceil_div((int)a.B, 16);
  if (a.ntiles == 0) return 0;
  dim3 grid(8 * ceil_div(ceil_div(a.ntiles, WV), 8) * h->E), block(64 * WV);
  // NB2 = 14 is H = 200 only: an odd hidden-block count, the last block is padding (NBU = 13); the
  // whole-block NB2 = 14 form (H = 209..224, no config) is not instantiated (it spilled 8-12 B)
  constexpr int NBU = NB2 == 14 ? NB2 - 1 : NB2;
  if (mode == FWD_PREDICT) {
    hipLaunchKernelGGL((bnn_fwd_ring_kernel<NB2, NBO, FWD_PREDICT, WV, P, DEPTH, NBU>), grid, block, 0, s, h->dev, a);
  } else {
    hipLaunchKernelGGL((bnn_fwd_ring_kernel<NB2, NBO, FWD_ROLLOUT, WV, P, DEPTH, NBU>), grid, block, 0, s, h->dev, a);
  }
  MOPO_HIP(hipGetLastError());
  return 0;
}
// the ring kernel's shapes: H = 200 (NB2 14, 13 used), or a whole even block count (NBH = NB2) other than 14
template <int NB2>
static bool ring_shape(const Bnn* h) { return NB2 <= 16 && (NB2 == 14 ? h->dev.NBH == 13 : h->dev.NBH == NB2); }

#ifndef BNN_R13
#define BNN_R13 1  // row blocks per wave at H = 200
#endif
#ifndef BNN_FWD_WAVES
#define BNN_FWD_WAVES 4
#endif
constexpr int FWD_WAVES = BNN_FWD_WAVES;

template <int KG0, int NBH, int NBO, int R, int TQ0 = 4, int TQH = 4>
static int launch_fwd_t(const Bnn* h, int mode, FwdArgs a, hipStream_t s) {
  a.ntiles = (int)ceil_div((int)a.B, 16 * R);
  if (a.ntiles == 0) return 0;
  dim3 grid(ceil_div(a.ntiles, FWD_WAVES) * h->E), block(64 * FWD_WAVES);
  if (mode == FWD_PREDICT)
    hipLaunchKernelGGL((bnn_fwd_kernel<KG0, NBH, NBO, R, FWD_PREDICT, FWD_WAVES, TQ0, TQH>), grid, block, 0, s, h->dev,
                       a);
  else
    hipLaunchKernelGGL((bnn_fwd_kernel<KG0, NBH, NBO, R, FWD_ROLLOUT, FWD_WAVES, TQ0, TQH>), grid, block, 0, s, h->dev,
                       a);
  MOPO_HIP(hipGetLastError());
  return 0;
}

template <int KG0, int NBO>
static int launch_fwd_h(const Bnn* h, int mode, const FwdArgs& a, hipStream_t s) {
  switch (h->dev.NBH) {
    case 2: return launch_fwd_t<KG0, 2, NBO, 2>(h, mode, a, s);
    case 4: return launch_fwd_t<KG0, 4, NBO, 2>(h, mode, a, s);
    case 13:  // H = 200 with 17 + 6 inputs (every halfcheetah / walker2d config): skip the padding k-steps
      if (KG0 == 2 && NBO == 3 && tail_steps(h->dev.IN) <= 2 && tail_steps(h->H) <= 2)
        return launch_fwd_t<KG0, 13, NBO, BNN_R13, 2, 2>(h, mode, a, s);
      return launch_fwd_t<KG0, 13, NBO, BNN_R13>(h, mode, a, s);
    case 25:
      if (KG0 == 2 && NBO == 3 && tail_steps(h->dev.IN) <= 2) return launch_fwd_t<KG0, 25, NBO, 1, 2, 4>(h, mode, a, s);
      return launch_fwd_t<KG0, 25, NBO, 1>(h, mode, a, s);
  }
  return fail("bnn: unsupported hidden size (supported: 32, 64, 200, 400; got H=" +
              std::to_string(h->H) + ")");
}

// split kernels (P > 1): one slice per k-group holding all P weight parts (every slice then feeds
// P (P + 1) / 2 MFMAs per block, so the copy of the next slice hides behind uniform work), 8 waves
// per workgroup sharing the 2 x P * NB KiB of LDS
#ifndef BNN_SPLIT_WAVES
#define BNN_SPLIT_WAVES 4
#endif
#ifndef BNN_SPLIT_PS
#define BNN_SPLIT_PS 1  // parts per slice; 0: all P
#endif

template <int NB2, int NBO, int P>
static int launch_bf16_p(const Bnn* h, int mode, FwdArgs a, hipStream_t s) {
  if constexpr (P == 1 && BNN_BF16_RING && NB2 <= 16)
    if (ring_shape<NB2>(h)) return launch_ring<NB2, NBO, 1, BNN_RING_DEPTH_BF16>(h, mode, a, s);
  if constexpr (P == 3 && BNN_BF16X6_RING && NB2 <= 16)
    if (ring_shape<NB2>(h)) return launch_ring<NB2, NBO, 3, BNN_RING_DEPTH_BF16>(h, mode, a, s);
  constexpr int WV = P == 1 ? FWD_WAVES : BNN_SPLIT_WAVES;
  constexpr int PS = P == 1 ? 1 : (BNN_SPLIT_PS == 0 ? P : BNN_SPLIT_PS);
  a.ntiles = (int)ceil_div((int)a.B, 16);
  if (a.ntiles == 0) return 0;
  dim3 grid(ceil_div(a.ntiles, WV) * h->E), block(64 * WV);   // = 8 groups (E / 8) when the XCDs own members
  a.xcd_members = (BNN_BF16_XCDMEM && h->E % (8 * BNN_BF16_XCDMEM) == 0) ? BNN_BF16_XCDMEM : 0;
  // odd hidden-block count (e.g. H = 200): the last block is padding and is skipped (NBU = NB2 - 1); not at
  // H = 400 (25 of 26), where the skipping variant takes 256 VGPRs and spills
  // NB2 = 14: H = 200 only (13 blocks used); the whole-block form is not instantiated (it spilled 8-12 B)
  if constexpr (NB2 == 14) {
    if (h->dev.NBH != NB2 - 1) return fail("bnn bf16: unsupported hidden size (H in (192, 224] runs at H <= 208 only)");
    if (mode == FWD_PREDICT)
      hipLaunchKernelGGL((bnn_fwd_bf16_kernel<NB2, NBO, FWD_PREDICT, WV, P, PS, NB2 - 1>), grid, block, 0, s, h->dev, a);
    else
      hipLaunchKernelGGL((bnn_fwd_bf16_kernel<NB2, NBO, FWD_ROLLOUT, WV, P, PS, NB2 - 1>), grid, block, 0, s, h->dev, a);
  } else if (NB2 <= 16 && h->dev.NBH == NB2 - 1) {
    if constexpr (NB2 <= 16) {
      if (mode == FWD_PREDICT)
        hipLaunchKernelGGL((bnn_fwd_bf16_kernel<NB2, NBO, FWD_PREDICT, WV, P, PS, NB2 - 1>), grid, block, 0, s, h->dev, a);
      else
        hipLaunchKernelGGL((bnn_fwd_bf16_kernel<NB2, NBO, FWD_ROLLOUT, WV, P, PS, NB2 - 1>), grid, block, 0, s, h->dev, a);
    }
  } else if (mode == FWD_PREDICT) {
    hipLaunchKernelGGL((bnn_fwd_bf16_kernel<NB2, NBO, FWD_PREDICT, WV, P, PS>), grid, block, 0, s, h->dev, a);
  } else {
    hipLaunchKernelGGL((bnn_fwd_bf16_kernel<NB2, NBO, FWD_ROLLOUT, WV, P, PS>), grid, block, 0, s, h->dev, a);
  }
  MOPO_HIP(hipGetLastError());
  return 0;
}

template <int NB2, int NBO, int R>
static int launch_f16r(const Bnn* h, int mode, FwdArgs a, hipStream_t s) {
  constexpr int WV = BNN_F16R_WAVES;
  a.ntiles = (int)ceil_div((int)a.B, 16 * R);
  if (a.ntiles == 0) return 0;
  dim3 grid(8 * ceil_div(ceil_div(a.ntiles, WV), 8) * h->E), block(64 * WV);
  if (NB2 <= 16 && h->dev.NBH == NB2 - 1) {
    if (mode == FWD_PREDICT)
      hipLaunchKernelGGL((bnn_fwd_f16r_kernel<NB2, NBO, FWD_PREDICT, WV, R, NB2 - 1>), grid, block, 0, s, h->dev, a);
    else
      hipLaunchKernelGGL((bnn_fwd_f16r_kernel<NB2, NBO, FWD_ROLLOUT, WV, R, NB2 - 1>), grid, block, 0, s, h->dev, a);
  } else if (mode == FWD_PREDICT) {
    hipLaunchKernelGGL((bnn_fwd_f16r_kernel<NB2, NBO, FWD_PREDICT, WV, R>), grid, block, 0, s, h->dev, a);
  } else {
    hipLaunchKernelGGL((bnn_fwd_f16r_kernel<NB2, NBO, FWD_ROLLOUT, WV, R>), grid, block, 0, s, h->dev, a);
  }
  MOPO_HIP(hipGetLastError());
  return 0;
}

template <int NB2, int NBO>
static int launch_f16s(const Bnn* h, int mode, FwdArgs a, hipStream_t s) {
  if constexpr (BNN_F16_R > 0 && NB2 <= 16) return launch_f16r<NB2, NBO, BNN_F16_R>(h, mode, a, s);
  constexpr int WV = BNN_SPLIT_WAVES, PS = BNN_SPLIT_PS == 0 ? 2 : BNN_SPLIT_PS;
  a.ntiles = (int)ceil_div((int)a.B, 16);
  if (a.ntiles == 0) return 0;
#if BNN_F16_XCD
  dim3 grid(8 * ceil_div(ceil_div(a.ntiles, WV), 8) * h->E), block(64 * WV);
#else
  dim3 grid(ceil_div(a.ntiles, WV) * h->E), block(64 * WV);
#endif
  // NBU: hidden blocks in use (NB2 - 1 when the block count is odd, e.g. H = 200 -> 13 of 14).  Not at
  // H = 400 (25 of 26): the register allocation it gets there (VGPR + AGPR split) measured 17 % slower.
  // H <= 256 runs the ring kernel (every supported hidden size there has a ring shape); the f16s kernel
  // is compiled for H = 400 only (and for H <= 256 in BNN_F16_RING = 0 A/B builds)
  if constexpr (BNN_F16_RING && NB2 <= 16) {
    if (ring_shape<NB2>(h)) return launch_ring<NB2, NBO, 2, BNN_RING_DEPTH_F16>(h, mode, a, s);
    return fail("bnn f16x3: unsupported hidden size");
  }
  if constexpr (BNN_F16_HALF && NB2 == 26) {   // H = 400: the column-half kernel (two workgroups per CU)
    if (h->dev.NBH == NB2 - 1) {
      a.xcd_members = (BNN_F16H_XCDMEM && h->E % 8 == 0) ? 1 : 0;
      if (a.xcd_members) grid = dim3(8 * ceil_div(a.ntiles, WV) * (h->E / 8));   // (XCD, member, row group)
      if (mode == FWD_PREDICT)
        hipLaunchKernelGGL((bnn_fwd_f16h_kernel<NB2, NBO, FWD_PREDICT, WV, NB2 - 1>), grid, block, 0, s, h->dev, a);
      else
        hipLaunchKernelGGL((bnn_fwd_f16h_kernel<NB2, NBO, FWD_ROLLOUT, WV, NB2 - 1>), grid, block, 0, s, h->dev, a);
      MOPO_HIP(hipGetLastError());
      return 0;
    }
  }
  if constexpr (NB2 <= 16) {
    if (h->dev.NBH == NB2 - 1) {
      if (mode == FWD_PREDICT)
        hipLaunchKernelGGL((bnn_fwd_f16s_kernel<NB2, NBO, FWD_PREDICT, WV, PS, NB2 - 1>), grid, block, 0, s, h->dev, a);
      else
        hipLaunchKernelGGL((bnn_fwd_f16s_kernel<NB2, NBO, FWD_ROLLOUT, WV, PS, NB2 - 1>), grid, block, 0, s, h->dev, a);
      MOPO_HIP(hipGetLastError());
      return 0;
    }
  }
  if (mode == FWD_PREDICT) {
    hipLaunchKernelGGL((bnn_fwd_f16s_kernel<NB2, NBO, FWD_PREDICT, WV, PS>), grid, block, 0, s, h->dev, a);
  } else {
    hipLaunchKernelGGL((bnn_fwd_f16s_kernel<NB2, NBO, FWD_ROLLOUT, WV, PS>), grid, block, 0, s, h->dev, a);
  }
  MOPO_HIP(hipGetLastError());
  return 0;
}

template <int NB2, int NBO>
static int launch_bf16_t(const Bnn* h, int mode, const FwdArgs& a, hipStream_t s) {
  if (h->dtype == DT_F16X3) return launch_f16s<NB2, NBO>(h, mode, a, s);
  switch (bf16_parts(h->dtype)) {
    case 2: return launch_bf16_p<NB2, NBO, 2>(h, mode, a, s);
    case 3:
      // bf16x6 at H > 256: its 39-slice layer loop does not unroll (the part index goes dynamic: 432 B of
      // scratch per lane, a ~70x cliff) -- f16x3 is the f32-accurate 16-bit mode there
      if constexpr (NB2 > 16) return fail("bnn bf16x6: hidden sizes <= 256 only (use f16x3 or fp32 at H = 400)");
      else return launch_bf16_p<NB2, NBO, 3>(h, mode, a, s);
  }
  return launch_bf16_p<NB2, NBO, 1>(h, mode, a, s);
}

static int launch_bf16(const Bnn* h, int mode, const FwdArgs& a, hipStream_t s) {
  if (h->dev.IN > 32) return fail("bnn bf16: obs_dim + act_dim must be <= 32");
  if (h->dev.NBO == 3) {
    switch (h->dev.NB2) {
      case 2: return launch_bf16_t<2, 3>(h, mode, a, s);
      case 4: return launch_bf16_t<4, 3>(h, mode, a, s);
      case 14: return launch_bf16_t<14, 3>(h, mode, a, s);
      case 26: return launch_bf16_t<26, 3>(h, mode, a, s);
    }
  } else if (h->dev.NBO == 2) {
    switch (h->dev.NB2) {
      case 4: return launch_bf16_t<4, 2>(h, mode, a, s);
      case 14: return launch_bf16_t<14, 2>(h, mode, a, s);
    }
  }
  return fail("bnn bf16: unsupported hidden/output size");
}

int launch_bnn_fwd(const Bnn* h, int mode, const FwdArgs& a, hipStream_t s) {
  if (!h->has_params) return fail("bnn: parameters not set (mopo_bnn_set_params)");
  if (h->dtype != 0) return launch_bf16(h, mode, a, s);
  if (h->dev.KG0 != 1 && h->dev.KG0 != 2) return fail("bnn: obs_dim + act_dim must be <= 32");
  const bool k1 = h->dev.KG0 == 1;  // hopper: 11 + 3 inputs
  switch (h->dev.NBO) {
    case 3: return k1 ? launch_fwd_h<1, 3>(h, mode, a, s) : launch_fwd_h<2, 3>(h, mode, a, s);
    case 2: return k1 ? launch_fwd_h<1, 2>(h, mode, a, s) : launch_fwd_h<2, 2>(h, mode, a, s);
  }
  return fail("bnn: unsupported output dim");
}

}  // namespace mopo

using namespace mopo;

// ---------------------------------------------------------------------------------------- C ABI
extern "C" int mopo_bnn_create(mopo_bnn_t* out, int E, int obs_dim, int act_dim, int hidden, int smv,
                               int dtype) {
  MOPO_REQUIRE(out != nullptr, "mopo_bnn_create: out is NULL");
  MOPO_REQUIRE(E >= 1 && E <= 256, "mopo_bnn_create: num_networks must be in [1, 256]");
  MOPO_REQUIRE(obs_dim >= 1 && act_dim >= 1, "mopo_bnn_create: bad obs/act dims");
  MOPO_REQUIRE(dtype >= 0 && dtype <= 4,
               "mopo_bnn_create: dtype must be 0 (fp32), 1 (bf16), 2 (bf16x3), 3 (bf16x6) or 4 (f16x3)");
  Bnn* h = new Bnn();
  h->E = E; h->O = obs_dim; h->A = act_dim; h->H = hidden; h->smv = smv; h->dtype = dtype;
  BnnDev& d = h->dev;
  d.E = E; d.O = obs_dim; d.A = act_dim; d.IN = obs_dim + act_dim; d.H = hidden; d.D = obs_dim + 1;
  d.KG0 = ceil_div(d.IN, 16);
  d.NBH = ceil_div(hidden, 16);
  d.NBO = ceil_div(2 * d.D, 16);
  d.NB2 = (d.NBH + 1) / 2 * 2;
  d.BS = d.NB2 * 16;
  if (dtype != 0 && d.NB2 == 14 && d.NBH != 13) {   // the 16-bit kernels' NB2 = 14 shape is H = 200's 13 blocks
    delete h;
    return fail("mopo_bnn_create: the 16-bit dtypes do not support hidden sizes 209..224 (got " +
                std::to_string(hidden) + "; use fp32)");
  }
  if (dtype == 3 && d.NB2 > 16) {   // launch_bf16_t: no bf16x6 kernel above H = 256
    delete h;
    return fail("mopo_bnn_create: bf16x6 supports hidden sizes <= 256 (use f16x3 or fp32)");
  }
  *out = reinterpret_cast<mopo_bnn_t>(h);
  return 0;
}

extern "C" int mopo_bnn_destroy(mopo_bnn_t hh) {
  Bnn* h = reinterpret_cast<Bnn*>(hh);
  if (!h) return 0;
  if (h->buf) (void)hipFree(h->buf);
  if (h->bbuf) (void)hipFree(h->bbuf);
  delete h;
  return 0;
}

extern "C" int mopo_bnn_set_params(mopo_bnn_t hh, const float* const* arrs, int n) {
  Bnn* h = reinterpret_cast<Bnn*>(hh);
  MOPO_REQUIRE(h != nullptr, "mopo_bnn_set_params: NULL handle");
  MOPO_REQUIRE(n == (h->smv ? 16 : 14), "mopo_bnn_set_params: expected 16 (smv) or 14 arrays (.mat keys)");
  BnnDev& d = h->dev;
  const int E = h->E, IN = d.IN, H = h->H, D = d.D;
  const int KG0 = d.KG0, NBH = d.NBH, NBO = d.NBO;
  const int64_t hp = d.BS;  // bias stride (covers the bf16 path's even block count)
  // sizes (floats) of the packed regions
  const int64_t s_w0 = (int64_t)E * KG0 * NBH * 256, s_wh = 3LL * E * NBH * NBH * 256,
                s_whd = (int64_t)E * NBH * NBO * 256, s_b0 = E * hp, s_bh = 3 * E * hp,
                s_bhd = (int64_t)E * 3 * NBO * 16;
  const int64_t s_ws = (5LL * E + 63) / 64 * 64;  // f16x3 inverse weight scales [5][E]
  const int64_t total = s_w0 + s_wh + s_whd + s_b0 + s_bh + s_bhd + 2 * 64 + 2 * 64 + s_ws;
  if (!h->buf) MOPO_HIP(hipMalloc(&h->buf, total * sizeof(float)));
  h->buf_bytes = total * (int64_t)sizeof(float);
  float* base = h->buf;
  float* w0 = base; float* wh = w0 + s_w0; float* whd = wh + s_wh;
  float* b0 = whd + s_whd; float* bh = b0 + s_b0; float* bhd = bh + s_bh;
  float* mu = bhd + s_bhd; float* sg = mu + 64; float* mx = sg + 64; float* mn = mx + 64;
  float* wsc = mn + 64;

  // stage raw arrays on the device, then pack there (same code path as on-device repacking)
  const int n_layers = 5;
  std::vector<const float*> W(n_layers), Bv(n_layers);
  for (int i = 0; i < n_layers; ++i) { W[i] = arrs[2 + 2 * i]; Bv[i] = arrs[3 + 2 * i]; }
  // combined head raw [E][H][2D] : mean columns then log-var columns
  std::vector<float> head((size_t)E * H * 2 * D), headb((size_t)E * 2 * D);
  for (int e = 0; e < E; ++e)
    for (int k = 0; k < H; ++k)
      for (int j = 0; j < 2 * D; ++j) {
        float v;
        if (h->smv) v = j < D ? W[4][((size_t)e * H + k) * D + j] : arrs[12][((size_t)e * H + k) * D + (j - D)];
        else v = W[4][((size_t)e * H + k) * 2 * D + j];
        head[((size_t)e * H + k) * 2 * D + j] = v;
      }
  for (int e = 0; e < E; ++e)
    for (int j = 0; j < 2 * D; ++j)
      headb[(size_t)e * 2 * D + j] = h->smv ? (j < D ? Bv[4][e * D + j] : arrs[13][e * D + (j - D)])
                                            : Bv[4][e * 2 * D + j];
  const float* maxlv = arrs[h->smv ? 14 : 12];
  const float* minlv = arrs[h->smv ? 15 : 13];

  size_t stage_n = std::max((size_t)E * H * H, head.size());
  stage_n = std::max(stage_n, (size_t)E * IN * H);
  float* stage = nullptr;
  MOPO_HIP(hipMalloc(&stage, stage_n * sizeof(float)));
  struct DevFree {  // frees the staging buffers on every return path
    float*& p;
    ~DevFree() { if (p) (void)hipFree(p); }
  } stage_guard{stage};
  auto pack = [&](const float* src, size_t nsrc, float* dst, int K, int N, int KG, int NB, int perm_n) -> int {
    MOPO_HIP(hipMemcpy(stage, src, nsrc * sizeof(float), hipMemcpyHostToDevice));
    int64_t tot = (int64_t)E * KG * NB * 256;
    int blocks = (int)std::min<int64_t>((tot + 255) / 256, 4096);
    hipLaunchKernelGGL(pack_frags_kernel, dim3(blocks), dim3(256), 0, 0, stage, dst, E, K, N, KG, NB, 1, perm_n);
    MOPO_HIP(hipGetLastError());
    MOPO_HIP(hipDeviceSynchronize());
    return 0;
  };
  auto packb = [&](const float* src, float* dst, int N, int NP) -> int {
    MOPO_HIP(hipMemcpy(stage, src, (size_t)E * N * sizeof(float), hipMemcpyHostToDevice));
    const float mul = h->dtype != DT_FP32 ? -1.4426950408889634f : 1.f;  // 16-bit kernels: log2 domain
    hipLaunchKernelGGL(pack_bias_kernel, dim3(ceil_div(E * NP, 256)), dim3(256), 0, 0, stage, dst, E, N, NP, mul);
    MOPO_HIP(hipGetLastError());
    MOPO_HIP(hipDeviceSynchronize());
    return 0;
  };
  int rc = pack(W[0], (size_t)E * IN * H, w0, IN, H, KG0, NBH, 1);  // each step runs only if all before succeeded
  if (rc == 0) rc = packb(Bv[0], b0, H, (int)hp);
  for (int l = 0; l < 3 && rc == 0; ++l) {
    rc = pack(W[1 + l], (size_t)E * H * H, wh + (int64_t)l * E * NBH * NBH * 256, H, H, NBH, NBH, 1);
    if (rc == 0) rc = packb(Bv[1 + l], bh + l * E * hp, H, (int)hp);
  }
  if (rc == 0) rc = pack(head.data(), head.size(), whd, H, 2 * D, NBH, NBO, 2);  // head outputs: head_col slots
  if (rc) return rc;
  {  // head aux [E][bias | max_logvar | min_logvar], NBO*16 each, in head_col slot order
    std::vector<float> aux((size_t)s_bhd, 0.f);
    for (int e = 0; e < E; ++e) {
      float* x = aux.data() + (size_t)e * 3 * NBO * 16;
      for (int sl = 0; sl < NBO * 16; ++sl) {
        const int c = head_col(sl, D);
        if (c < 0) continue;
        x[sl] = headb[(size_t)e * 2 * D + c];
        if (c >= D) {
          x[NBO * 16 + sl] = arrs[h->smv ? 14 : 12][c - D];
          x[2 * NBO * 16 + sl] = arrs[h->smv ? 15 : 13][c - D];
        }
      }
    }
    MOPO_HIP(hipMemcpy(bhd, aux.data(), aux.size() * sizeof(float), hipMemcpyHostToDevice));
  }
  if (h->dtype != 0 && rc == 0) {
    // bf16 fragments: [E][1][P][NB2] | [3][E][KG][P][NB2] | [E][KG][P][NBO], 256 floats (= 512 bf16) each
    const int NB2 = d.NB2, KG = NB2 / 2, P = bf16_parts(h->dtype);
    const int64_t f0 = (int64_t)E * P * NB2, fh = 3LL * E * KG * P * NB2, fd = (int64_t)E * KG * P * NBO;
    if (!h->bbuf) MOPO_HIP(hipMalloc(&h->bbuf, (f0 + fh + fd) * 256 * sizeof(float)));
    h->bbuf_bytes = (f0 + fh + fd) * 256 * (int64_t)sizeof(float);
    float* b0f = reinterpret_cast<float*>(h->bbuf);
    float* bhf = b0f + f0 * 256;
    float* bdf = bhf + fh * 256;
    // f16x3: per layer and member, 2^k with max |W| 2^k in [2^14, 2^15) (mlp_tile.h split_f16_scaled)
    std::vector<float> scale_h(5 * E), inv_h(5 * E, 1.f);
    float* scale_d = nullptr;
    DevFree scale_guard{scale_d};
    if (h->dtype == DT_F16X3) MOPO_HIP(hipMalloc(&scale_d, E * sizeof(float)));
    auto member_scales = [&](const float* src, int K, int N, int layer) {
      for (int e = 0; e < E; ++e) {
        float m = 0.f;
        for (int64_t i = 0; i < (int64_t)K * N; ++i) m = std::max(m, std::fabs(src[(int64_t)e * K * N + i]));
        int ex = 0;
        if (m > 0.f && std::isfinite(m)) std::frexp(m, &ex);  // m in [2^(ex-1), 2^ex)
        const int k = m > 0.f && std::isfinite(m) ? 15 - ex : 0;
        scale_h[layer * E + e] = std::ldexp(1.f, k);
        inv_h[layer * E + e] = std::ldexp(1.f, -k);
      }
    };
    int layer_idx = 0;
    auto packh = [&](const float* src, size_t nsrc, float* dst, int K, int N, int KGb, int NB, int perm_n) -> int {
      MOPO_HIP(hipMemcpy(stage, src, nsrc * sizeof(float), hipMemcpyHostToDevice));
      int64_t tot = (int64_t)E * KGb * P * NB * 512;
      int blocks = (int)std::min<int64_t>((tot + 255) / 256, 4096);
      if (h->dtype == DT_F16X3) {
        member_scales(src, K, N, layer_idx);
        MOPO_HIP(hipMemcpy(scale_d, scale_h.data() + layer_idx * E, E * sizeof(float), hipMemcpyHostToDevice));
        hipLaunchKernelGGL(pack_frags_f16s_kernel, dim3(blocks), dim3(256), 0, 0, stage, (short*)dst, E, K, N, KGb, NB,
                           1, perm_n, (const float*)scale_d);
      } else if (P == 3)
        hipLaunchKernelGGL(pack_frags_bf16_kernel<3>, dim3(blocks), dim3(256), 0, 0, stage, (short*)dst, E, K, N, KGb,
                           NB, 1, perm_n);
      else if (P == 2)
        hipLaunchKernelGGL(pack_frags_bf16_kernel<2>, dim3(blocks), dim3(256), 0, 0, stage, (short*)dst, E, K, N, KGb,
                           NB, 1, perm_n);
      else
        hipLaunchKernelGGL(pack_frags_bf16_kernel<1>, dim3(blocks), dim3(256), 0, 0, stage, (short*)dst, E, K, N, KGb,
                           NB, 1, perm_n);
      MOPO_HIP(hipGetLastError());
      MOPO_HIP(hipDeviceSynchronize());
      ++layer_idx;
      return 0;
    };
    if (rc == 0) rc = packh(W[0], (size_t)E * IN * H, b0f, IN, H, 1, NB2, 1);
    for (int l = 0; l < 3 && rc == 0; ++l)
      rc = packh(W[1 + l], (size_t)E * H * H, bhf + (int64_t)l * E * KG * P * NB2 * 256, H, H, KG, NB2, 1);
    if (rc == 0) rc = packh(head.data(), head.size(), bdf, H, 2 * D, KG, NBO, 2);
    if (rc == 0 && h->dtype == DT_F16X3)
      rc = hipMemcpy(wsc, inv_h.data(), 5 * E * sizeof(float), hipMemcpyHostToDevice) == hipSuccess ? 0
                                                                                                 : fail("bnn: scale copy");
    d.w0b = b0f; d.whb = bhf; d.whdb = bdf; d.wscale = wsc;
  }
  if (rc) return -1;
  MOPO_HIP(hipMemcpy(mu, arrs[0], IN * sizeof(float), hipMemcpyHostToDevice));
  MOPO_HIP(hipMemcpy(sg, arrs[1], IN * sizeof(float), hipMemcpyHostToDevice));
  MOPO_HIP(hipMemcpy(mx, maxlv, D * sizeof(float), hipMemcpyHostToDevice));
  MOPO_HIP(hipMemcpy(mn, minlv, D * sizeof(float), hipMemcpyHostToDevice));
  d.w0 = w0; d.wh = wh; d.whd = whd; d.b0 = b0; d.bh = bh; d.bhd = bhd;
  d.mu = mu; d.sigma = sg; d.maxlv = mx; d.minlv = mn;
  h->has_params = true;
  return 0;
}

extern "C" int mopo_bnn_predict(mopo_bnn_t hh, const void* x, int x_f64, int64_t B, float* mean,
                                float* var, void* stream) {
  Bnn* h = reinterpret_cast<Bnn*>(hh);
  MOPO_REQUIRE(h != nullptr, "mopo_bnn_predict: NULL handle");
  MOPO_REQUIRE(B >= 0 && B < (1LL << 31) / 32, "mopo_bnn_predict: batch too large");
  if (B == 0) return 0;
  MOPO_REQUIRE(x && mean && var, "mopo_bnn_predict: NULL pointer");
  FwdArgs a{};
  const int IN = h->dev.IN;
  const size_t es = x_f64 ? 8 : 4;
  a.in = FwdIn{x, x_f64, IN, (const char*)x + es * h->O, x_f64, IN};
  a.B = B;
  a.mean = mean;
  a.var = var;
  return launch_bnn_fwd(h, FWD_PREDICT, a, (hipStream_t)stream);
}

extern "C" int64_t mopo_bnn_packed_bytes(mopo_bnn_t hh) {
  const Bnn* h = reinterpret_cast<const Bnn*>(hh);
  if (!h || !h->has_params) return -1;
  return h->buf_bytes + h->bbuf_bytes;
}

extern "C" int mopo_bnn_packed_copy(mopo_bnn_t hh, int to_handle, void* d_buf, int64_t nbytes, void* stream) {
  Bnn* h = reinterpret_cast<Bnn*>(hh);
  MOPO_REQUIRE(h != nullptr, "mopo_bnn_packed_copy: NULL handle");
  MOPO_REQUIRE(h->has_params, "mopo_bnn_packed_copy: parameters not set (the packed layout comes from set_params)");
  MOPO_REQUIRE(d_buf != nullptr && nbytes == h->buf_bytes + h->bbuf_bytes,
               "mopo_bnn_packed_copy: buffer must hold exactly mopo_bnn_packed_bytes() bytes");
  hipStream_t s = (hipStream_t)stream;
  char* b = static_cast<char*>(d_buf);
  if (to_handle) {
    MOPO_HIP(hipMemcpyAsync(h->buf, b, h->buf_bytes, hipMemcpyDeviceToDevice, s));
    if (h->bbuf_bytes) MOPO_HIP(hipMemcpyAsync(h->bbuf, b + h->buf_bytes, h->bbuf_bytes, hipMemcpyDeviceToDevice, s));
  } else {
    MOPO_HIP(hipMemcpyAsync(b, h->buf, h->buf_bytes, hipMemcpyDeviceToDevice, s));
    if (h->bbuf_bytes) MOPO_HIP(hipMemcpyAsync(b + h->buf_bytes, h->bbuf, h->bbuf_bytes, hipMemcpyDeviceToDevice, s));
  }
  return 0;
}
