// Squashed-Gaussian policy forward (rollout actions).
//
// Replaces MOPO.get_action_meta -> mlp_gaussian_policy + apply_squashing_func
// (mopo/algorithms/mopo.py:468-485, 275-308, 286-296):
//   net = relu(relu(s W1 + b1) W2 + b2); mu = net Wmu + bmu; log_std = clip(net Wls + bls, -20, 2)
//   pi = tanh(mu + eps * exp(log_std)),  mu_out = tanh(mu)
// Same register-resident transposed-MFMA scheme and LDS-staged weight slices as the ensemble
// forward (mlp_tile.h).  The policy changes every SAC step, so its weights are repacked into
// fragment-major order once per rollout (pack_actor, ~0.3 MB) from the SAC parameter buffer.
#include "actor.h"
#include "mlp_tile.h"

namespace mopo {

// packed layout: W1 frags | W2 frags | head frags | b1 [NB*16] | b2 [NB*16] | [bmu | bls] [16]
// (biases zero-padded to whole 16-blocks so the kernel stages them into LDS with global_load_lds)
// f16 (f16x3): W1 [1][2][NB] | W2 [NB/2][2][NB] | head [NB/2][2][1] fragments of 64 lanes x 8 fp16
// (256 floats each, the ensemble's bf16 fragment layout with its k permutation), then the same biases,
// then 3 inverse weight scales (+5 spare floats) and actor_wmax_kernel's WMAX_BLOCKS x 3 partial max-|W|
constexpr int WMAX_BLOCKS = 64;   // actor_wmax_kernel's grid (<= 64: one wave reduces the partials)

// split: 0 f32 fragments, 1 f16x3 (2 scaled fp16 parts), 2 bf16x6 (the exact 3-part bf16 split, no scales):
// W1 [1][3][NB] | W2 [NB/2][3][NB] | head [NB/2][3][1] fragments, then the biases
__host__ __device__ int64_t actor_packed_floats(int O, int Hp, int split) {
  const int KG0 = (O + 15) / 16, NB = (Hp + 15) / 16;
  if (split == 2) return (int64_t)(3 * NB + 3 * (NB / 2) * NB + 3 * (NB / 2)) * 256 + 2LL * NB * 16 + 16;
  if (split) return (int64_t)(2 * NB + NB * NB + NB) * 256 + 2LL * NB * 16 + 16 + 8 + 3 * WMAX_BLOCKS;
  return (int64_t)KG0 * NB * 256 + (int64_t)NB * NB * 256 + (int64_t)NB * 256 + 2LL * NB * 16 + 16;
}

// max |W| of the three weight matrices (W1, W2, [Wmu | Wls]): block b's maxima -> wpart[3 b + q] (plain
// stores: no zeroing launch before it, no atomics; pack_actor_f16_kernel reduces the WMAX_BLOCKS partials)
__global__ __launch_bounds__(256) void actor_wmax_kernel(const float* __restrict__ P, int O, int A, int Hp,
                                                         float* __restrict__ wpart) {
  __shared__ float sm[4][3];
  const float* W1 = P;
  const float* W2 = W1 + O * Hp + Hp;
  const float* Wm = W2 + Hp * Hp + Hp;
  const float* Wl = Wm + Hp * A + A;
  const int64_t n1 = (int64_t)O * Hp, n2 = (int64_t)Hp * Hp, nh = 2LL * Hp * A;
  float m[3] = {0.f, 0.f, 0.f};
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n1 + n2 + nh; i += (int64_t)gridDim.x * blockDim.x) {
    if (i < n1) m[0] = fmaxf(m[0], fabsf(W1[i]));
    else if (i < n1 + n2) m[1] = fmaxf(m[1], fabsf(W2[i - n1]));
    else {
      const int64_t j = i - n1 - n2;
      m[2] = fmaxf(m[2], fabsf(j < (int64_t)Hp * A ? Wm[j] : Wl[j - (int64_t)Hp * A]));
    }
  }
  for (int q = 0; q < 3; ++q) {
    float v = m[q];
    for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6][q] = v;
  }
  __syncthreads();
  if (threadIdx.x < 3)
    wpart[3 * blockIdx.x + threadIdx.x] =
        fmaxf(fmaxf(sm[0][threadIdx.x], sm[1][threadIdx.x]), fmaxf(sm[2][threadIdx.x], sm[3][threadIdx.x]));
}

// f16x3 packing: fp16 parts of W * 2^k (k per matrix from wmax: max |W| 2^k in [2^14, 2^15)), the
// biases as in the f32 packing, and the 3 inverse scales
__global__ void pack_actor_f16_kernel(const float* __restrict__ P, int O, int A, int Hp, float* __restrict__ dst,
                                      const float* __restrict__ wpart) {
  const int NB = ceil_div(Hp, 16), KG = NB / 2;
  const float* W1 = P;
  const float* W2 = W1 + O * Hp + Hp;
  const float* Wm = W2 + Hp * Hp + Hp;
  const float* Wl = Wm + Hp * A + A;
  __shared__ float smax[3];
  if (threadIdx.x < 64) {   // the max over actor_wmax_kernel's per-block partials (exact in any order)
    float v[3];
    for (int q = 0; q < 3; ++q) v[q] = threadIdx.x < WMAX_BLOCKS ? wpart[3 * threadIdx.x + q] : 0.f;
    for (int q = 0; q < 3; ++q)
      for (int o = 32; o >= 1; o >>= 1) v[q] = fmaxf(v[q], __shfl_xor(v[q], o));
    if (threadIdx.x == 0)
      for (int q = 0; q < 3; ++q) smax[q] = v[q];
  }
  __syncthreads();
  float sc[3], inv[3];
  for (int q = 0; q < 3; ++q) row_scale(smax[q], sc[q], inv[q]);
  const int64_t f1 = 2LL * NB, f2 = (int64_t)KG * 2 * NB, fh = (int64_t)KG * 2;
  const int64_t nfrag = (f1 + f2 + fh) * 512;  // fp16 elements
  short* d16 = reinterpret_cast<short*>(dst);
  float* tail = dst + (f1 + f2 + fh) * 256;
  const int64_t total = nfrag + 2LL * NB * 16 + 16 + 3;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    if (i < nfrag) {
      const int j = i & 7, lane = (int)((i >> 3) & 63), g = lane >> 4, r = lane & 15;
      int64_t f = i >> 9;
      int which, nbs;
      if (f < f1) { which = 0; nbs = NB; }
      else if (f < f1 + f2) { which = 1; f -= f1; nbs = NB; }
      else { which = 2; f -= f1 + f2; nbs = 1; }
      const int nb = (int)(f % nbs), p = (int)((f / nbs) % 2), kg = (int)(f / (2 * nbs));
      int k = kg * 32 + bf16_kperm(g, j);
      const int n = nb * 16 + r;
      float v = 0.f;
      if (which == 0) {
        k = slot_feat(k, O);
        if (k >= 0 && n < Hp) v = W1[k * Hp + n];
      } else if (which == 1) {
        if (k < Hp && n < Hp) v = W2[k * Hp + n];
      } else if (k < Hp) {
        v = r < A ? Wm[k * A + r] : (r < 2 * A ? Wl[k * A + (r - A)] : 0.f);
      }
      const F16Parts q = split_f16_scaled(v, sc[which]);
      d16[i] = p == 0 ? q.hi : q.lo;
    } else {
      const int j = (int)(i - nfrag);  // b1 | b2 | [bmu | bls] | inverse scales
      float v;
      if (j < NB * 16) v = j < Hp ? W1[O * Hp + j] : 0.f;
      else if (j < 2 * NB * 16) v = j - NB * 16 < Hp ? W2[Hp * Hp + j - NB * 16] : 0.f;
      else if (j < 2 * NB * 16 + 16) {
        const int q = j - 2 * NB * 16;
        v = q < A ? Wm[Hp * A + q] : (q < 2 * A ? Wl[Hp * A + q - A] : 0.f);
      } else {
        v = inv[j - 2 * NB * 16 - 16];
      }
      tail[j] = v;
    }
  }
}

// bf16x6 packing: part p of the exact split (split_bf16<3>) of each weight in the bf16 fragment layout
// (k permutation of the ensemble's), [kg][p][nb] per matrix; the biases as in the f32 packing
__global__ void pack_actor_x6_kernel(const float* __restrict__ P, int O, int A, int Hp, float* __restrict__ dst) {
  constexpr int NP = 3;
  const int NB = ceil_div(Hp, 16), KG = NB / 2;
  const float* W1 = P;
  const float* W2 = W1 + O * Hp + Hp;
  const float* Wm = W2 + Hp * Hp + Hp;
  const float* Wl = Wm + Hp * A + A;
  const int64_t f1 = (int64_t)NP * NB, f2 = (int64_t)KG * NP * NB, fh = (int64_t)KG * NP;
  const int64_t nfrag = (f1 + f2 + fh) * 512;  // bf16 elements
  short* d16 = reinterpret_cast<short*>(dst);
  float* tail = dst + (f1 + f2 + fh) * 256;
  const int64_t total = nfrag + 2LL * NB * 16 + 16;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    if (i < nfrag) {
      const int j = i & 7, lane = (int)((i >> 3) & 63), g = lane >> 4, r = lane & 15;
      int64_t f = i >> 9;
      int which, nbs;
      if (f < f1) { which = 0; nbs = NB; }
      else if (f < f1 + f2) { which = 1; f -= f1; nbs = NB; }
      else { which = 2; f -= f1 + f2; nbs = 1; }
      const int nb = (int)(f % nbs), p = (int)((f / nbs) % NP), kg = (int)(f / (NP * nbs));
      int k = kg * 32 + bf16_kperm(g, j);
      const int n = nb * 16 + r;
      float v = 0.f;
      if (which == 0) {
        k = slot_feat(k, O);
        if (k >= 0 && n < Hp) v = W1[k * Hp + n];
      } else if (which == 1) {
        if (k < Hp && n < Hp) v = W2[k * Hp + n];
      } else if (k < Hp) {
        v = r < A ? Wm[k * A + r] : (r < 2 * A ? Wl[k * A + (r - A)] : 0.f);
      }
      short parts[NP];
      split_bf16<NP>(v, parts);
      d16[i] = p == 0 ? parts[0] : (p == 1 ? parts[1] : parts[2]);
    } else {
      const int j = (int)(i - nfrag);  // b1 | b2 | [bmu | bls]
      float v;
      if (j < NB * 16) v = j < Hp ? W1[O * Hp + j] : 0.f;
      else if (j < 2 * NB * 16) v = j - NB * 16 < Hp ? W2[Hp * Hp + j - NB * 16] : 0.f;
      else {
        const int q = j - 2 * NB * 16;
        v = q < A ? Wm[Hp * A + q] : (q < 2 * A ? Wl[Hp * A + q - A] : 0.f);
      }
      tail[j] = v;
    }
  }
}

// One launch packs the whole policy (it is repacked at every rollout, after the SAC updates):
// W1 (observation side in slot_feat order), W2, the combined head (n < A -> Wmu[:, n],
// A <= n < 2A -> Wls[:, n - A]) fragment-major (mlp_tile.h), then the zero-padded biases.
__global__ void pack_actor_kernel(const float* __restrict__ P, int O, int A, int Hp, float* __restrict__ dst) {
  const int KG0 = ceil_div(O, 16), NB = ceil_div(Hp, 16);
  const float* W1 = P;
  const float* W2 = W1 + O * Hp + Hp;
  const float* Wm = W2 + Hp * Hp + Hp;
  const float* Wl = Wm + Hp * A + A;
  const int64_t n1 = (int64_t)KG0 * NB * 256, n2 = (int64_t)NB * NB * 256, nh = (int64_t)NB * 256;
  const int64_t total = actor_packed_floats(O, Hp);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int t = i & 3, lane = (i >> 2) & 63, g = lane >> 4, r = lane & 15;
    float v = 0.f;
    if (i < n1 + n2) {  // trunk layers: fragment f = kg * NB + nb
      const bool l1 = i < n1;
      const int64_t f = (l1 ? i : i - n1) >> 8;
      const int kg = (int)(f / NB), nb = (int)(f % NB);
      int k = kg * 16 + 4 * g + t;
      const int n = nb * 16 + r;
      if (l1) {
        k = slot_feat(k, O);
        if (k >= 0 && n < Hp) v = W1[k * Hp + n];
      } else if (k < Hp && n < Hp) {
        v = W2[k * Hp + n];
      }
    } else if (i < n1 + n2 + nh) {
      const int kg = (int)((i - n1 - n2) >> 8);
      const int k = kg * 16 + 4 * g + t;
      if (k < Hp) v = r < A ? Wm[k * A + r] : (r < 2 * A ? Wl[k * A + (r - A)] : 0.f);
    } else {
      const int j = (int)(i - n1 - n2 - nh);  // b1 | b2 | [bmu | bls]
      if (j < NB * 16) v = j < Hp ? W1[O * Hp + j] : 0.f;
      else if (j < 2 * NB * 16) v = j - NB * 16 < Hp ? W2[Hp * Hp + j - NB * 16] : 0.f;
      else {
        const int q = j - 2 * NB * 16;
        v = q < A ? Wm[Hp * A + q] : (q < 2 * A ? Wl[Hp * A + q - A] : 0.f);
      }
    }
    dst[i] = v;
  }
}

int pack_actor(const float* P, int O, int A, int Hp, float* dst, hipStream_t s, int split) {
  if (split == 2) {
    MOPO_REQUIRE(Hp % 32 == 0, "actor bf16x6: hidden width must be a multiple of 32");
    MOPO_REQUIRE(O <= 32 && 2 * A <= 16, "actor bf16x6: obs_dim <= 32, act_dim <= 8");
    const int64_t tot = actor_packed_floats(O, Hp, 2) * 2;   // upper bound on the elements the kernel walks
    hipLaunchKernelGGL(pack_actor_x6_kernel, dim3((int)std::min<int64_t>((tot + 255) / 256, 1024)), dim3(256), 0, s,
                       P, O, A, Hp, dst);
    MOPO_HIP(hipGetLastError());
    return 0;
  }
  const int f16 = split;
  if (f16) {
    MOPO_REQUIRE(Hp % 32 == 0, "actor f16x3: hidden width must be a multiple of 32");
    MOPO_REQUIRE(O <= 32 && 2 * A <= 16, "actor f16x3: obs_dim <= 32, act_dim <= 8");
    const int NB = Hp / 16;
    float* wpart = dst + (2LL * NB + NB * NB + NB) * 256 + 2LL * NB * 16 + 16 + 8;
    hipLaunchKernelGGL(actor_wmax_kernel, dim3(WMAX_BLOCKS), dim3(256), 0, s, P, O, A, Hp, wpart);
    MOPO_HIP(hipGetLastError());
    const int64_t tot = (2LL * NB + NB * NB + NB) * 512 + 2LL * NB * 16 + 16 + 3;
    hipLaunchKernelGGL(pack_actor_f16_kernel, dim3((int)std::min<int64_t>((tot + 255) / 256, 1024)), dim3(256), 0, s,
                       P, O, A, Hp, dst, (const float*)wpart);
    MOPO_HIP(hipGetLastError());
    return 0;
  }
  const int64_t tot = actor_packed_floats(O, Hp);
  hipLaunchKernelGGL(pack_actor_kernel, dim3((int)std::min<int64_t>((tot + 255) / 256, 1024)), dim3(256), 0, s, P, O,
                     A, Hp, dst);
  MOPO_HIP(hipGetLastError());
  return 0;
}

// bias (staged in LDS by layer_lds) + relu
template <int NB>
__device__ __forceinline__ void bias_relu(const float* b, const f32x4 (&acc)[1][NB], f32x4 (&out)[1][NB], int g) {
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const f32x4 bb = *reinterpret_cast<const f32x4*>(b + nb * 16 + 4 * g);
#pragma unroll
    for (int t = 0; t < 4; ++t) out[0][nb][t] = fmaxf(acc[0][nb][t] + bb[t], 0.f);
  }
}

// Four N(0, 1) policy-noise draws (actions 4 blk .. 4 blk + 3) of row ``uid``: one Philox block.
__device__ __forceinline__ void actor_noise4(uint64_t seed, uint32_t step, int64_t uid, int blk, float (&zz)[4]) {
  u32x4 c{(uint32_t)uid, (uint32_t)((uint64_t)uid >> 32) ^ ((uint32_t)blk << 20), step, RNG_ACT};
  u32x4 r = philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  box_muller(r.x, r.y, zz[0], zz[1]);
  box_muller(r.z, r.w, zz[2], zz[3]);
}

// Four U[-1, 1) random actions (np.random.uniform(-1, 1, act.shape), mopo.py:738), 24-bit uniforms.
__device__ __forceinline__ void actor_uniform4(uint64_t seed, uint32_t step, int64_t uid, int blk, float (&uu)[4]) {
  u32x4 c{(uint32_t)uid, (uint32_t)((uint64_t)uid >> 32) ^ ((uint32_t)blk << 20), step, RNG_ACT_UNIFORM};
  const u32x4 r = philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  uu[0] = -1.0f + 2.0f * ((float)(r.x >> 8) * 5.9604645e-8f);
  uu[1] = -1.0f + 2.0f * ((float)(r.y >> 8) * 5.9604645e-8f);
  uu[2] = -1.0f + 2.0f * ((float)(r.z >> 8) * 5.9604645e-8f);
  uu[3] = -1.0f + 2.0f * ((float)(r.w >> 8) * 5.9604645e-8f);
}

#ifndef ACT_WAVES_CFG
#define ACT_WAVES_CFG 4  // waves (16-row tiles) per workgroup
#endif
constexpr int ACT_WAVES = ACT_WAVES_CFG;

// Actions from the head outputs head[wv][m][0, 16) (mu | log_std) of the wave's 16 rows: noise or
// uniform actions, tanh squash, pool row / member pick (lane group 0), the ensemble's scaled input row.
__device__ __forceinline__ void actor_finish(const ActorArgs& a, float (&head)[ACT_WAVES][16][25], int wv, int m,
                                             int g, int64_t row, bool ok) {
  const int O = a.O, A = a.A;
  if (g == 0 && ok) {
    const int64_t uid = a.d_uid ? a.d_uid[row] : row + a.uid_offset;
    int64_t pos = -1;
    if (a.pool_act) pos = a.stage_base >= 0 ? a.stage_base + row : (a.pool_state[0] + a.pool_off + row) % a.pool_max;
    // four actions per Philox block; the per-block arrays are indexed by constants only (registers)
    for (int blk = 0; blk * 4 < A; ++blk) {
      float zz[4], uu[4];
      if (a.eps) {
#pragma unroll
        for (int i = 0; i < 4; ++i) zz[i] = blk * 4 + i < A ? a.eps[row * A + blk * 4 + i] : 0.f;
      } else {
#ifndef ACT_KNOB_LITE_FINISH   // timing-only builds (scripts/build_variant_actor.sh): no noise draws
        actor_noise4(a.seed, a.step, uid, blk, zz);
#else
        zz[0] = zz[1] = zz[2] = zz[3] = 0.f;
#endif
      }
      if (a.rand_act) {  // np.random.uniform(low=-1, high=1, size=act.shape) (mopo.py:738)
        if (a.act_uni) {
#pragma unroll
          for (int i = 0; i < 4; ++i) uu[i] = blk * 4 + i < A ? a.act_uni[row * A + blk * 4 + i] : 0.f;
        } else {
          actor_uniform4(a.seed, a.step, uid, blk, uu);
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int j = blk * 4 + i;
        if (j < A) {
          const float mu = head[wv][m][j];
          const float ls = fminf(fmaxf(head[wv][m][A + j], -20.f), 2.f);  // mopo.py:304
          const float sd = expf(ls);                                      // mopo.py:305
          const float u = mu + zz[i] * sd;                                // mopo.py:306
          const float act = a.rand_act ? uu[i] : tanhf(u);                // mopo.py:295 / 738
          head[wv][m][16 + j] = act;
          if (a.act) a.act[row * A + j] = act;
          if (a.mu) a.mu[row * A + j] = tanhf(mu);                        // mopo.py:294
          if (pos >= 0) a.pool_act[pos * A + j] = act;
        }
      }
    }
#ifdef ACT_KNOB_LITE_FINISH
    pos = -1;
#endif
    if (pos >= 0) {  // the observation half of the pool row (mopo.py:750), stored f32
      for (int k = 0; k < O; ++k)
        a.pool_obs[pos * O + k] = a.obs_f64 ? (float)reinterpret_cast<const double*>(a.obs)[row * O + k]
                                            : reinterpret_cast<const float*>(a.obs)[row * O + k];
    }
    if (a.pen_zero) a.pen_zero[row] = 0u;
    if (a.sel_out) {
      int32_t sel;
      if (a.sel_in) {
        sel = a.sel_in[row];
      } else {  // perf mode of np.random.choice(elites, B) (bnn.py:343)
        u32x4 c{(uint32_t)uid, (uint32_t)((uint64_t)uid >> 32), a.step, RNG_MODEL};
        u32x4 r = philox(c, (uint32_t)a.seed, (uint32_t)(a.seed >> 32));
        sel = a.elites[(int)(((uint64_t)r.x * (uint64_t)a.n_elites) >> 32)];
      }
      a.sel_out[row] = sel;
    }
  }
  if (a.xs) {  // the ensemble's layer-0 input, scaled exactly as bnn_fwd_kernel would; lane g: 8 slots
    __syncthreads();
    if (ok) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        f32x4 v;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int k = slot_feat(8 * g + 4 * q + t, a.xs_in);
          float x = 0.f;
          if (k >= 0) {
            const float raw = k < O ? (a.obs_f64 ? (float)reinterpret_cast<const double*>(a.obs)[row * O + k]
                                                  : reinterpret_cast<const float*>(a.obs)[row * O + k])
                                    : head[wv][m][16 + k - O];
            x = (raw - a.xs_mu[k]) / a.xs_sigma[k];
          }
          v[t] = x;
        }
        *reinterpret_cast<f32x4*>(a.xs + row * XS_STRIDE + 8 * g + 4 * q) = v;
      }
    }
  }
}

// TQ0: k-steps in the last k-group of the observation (tail_steps(O); 4 = all)
template <int KG0, int NBP, int TQ0 = 4>
#ifndef ACT_F32_OCC
// fp32 actor waves per SIMD at H = 256 (launch bound).  4 caps the kernel at 128 VGPRs and spilled 22-26 of
// them (88 B of scratch per lane); 3 (168 VGPRs) still spills 10-11 (44-48 B); 2 holds its 178 VGPRs with
// no scratch.  Measured at 4 / 3: 0.092 / 0.101 ms per 50k rows alone, the fp32 rollout 58.9 / 59.2M
// transitions/s (same-box A/B, profiles/r04_actor_ab.txt)
#define ACT_F32_OCC 2
#endif
__global__ __launch_bounds__(ACT_WAVES * 64, NBP == 16 ? ACT_F32_OCC : 2) void actor_kernel(const ActorArgs a) {
  constexpr int SLOT = Stage<NBP, ACT_WAVES>::SLOTS * 256;
  __shared__ float head[ACT_WAVES][16][25];  // head outputs [0, 16), then the actions [16, 16 + A)
  __shared__ __attribute__((aligned(16))) float lds[2 * SLOT + (NBP * 4 + 63) / 64 * 256];  // one array (bnn.hip)
  float* lds_bias = lds + 2 * SLOT;
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), m = lane & 15, g = lane >> 4;
  const int64_t count = a.d_count ? (int64_t)*a.d_count : a.B;
  if ((int64_t)blockIdx.x * ACT_WAVES * 16 >= count) return;  // whole workgroup past the live rows
  const int64_t row0 = ((int64_t)blockIdx.x * ACT_WAVES + wv) * 16;
  const int O = a.O, Hp = a.Hp;
  const float* w1f = a.Wpk;
  const float* w2f = w1f + KG0 * NBP * 256;
  const float* whf = w2f + NBP * NBP * 256;
  const float* b1 = whf + NBP * 256;  // padded biases (pack_actor)
  const float* b2 = b1 + NBP * 16;
  const float* bh = b2 + NBP * 16;
  (void)Hp;
  const int64_t row = row0 + m;
  const bool ok = row < count;
  f32x4 x0[1][KG0];
#pragma unroll
  for (int kg = 0; kg < KG0; ++kg)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int k = slot_feat(kg * 16 + 4 * g + t, O);
      float v = 0.f;
      if (ok && k >= 0)
        v = a.obs_f64 ? (float)reinterpret_cast<const double*>(a.obs)[row * O + k]
                      : reinterpret_cast<const float*>(a.obs)[row * O + k];
      x0[0][kg][t] = v;
    }
  f32x4 hd[1][1];
  if constexpr (NBP == 16) {
    // Hp = 256: the second layer runs as two passes of 8 output tiles, each folded into the head
    // right away, so a wave holds h1 (64 VGPRs) + 8 accumulator tiles (32) instead of 16 + 16:
    // <= 128 VGPRs = 4 waves/SIMD, and B = 50k (782 workgroups) fits one round of 1,024 slots
    // instead of spilling 14 workgroups into a second round of 768.  Staged bytes are unchanged
    // (each pass copies its half of every k-group slice); each layer's first slice is copied
    // during the previous pass's last k-group (mlp_tile.h).
    // (measured: staging 2 k-groups per barrier in the 8-tile passes is 3 % slower)
    f32x4 h1[1][NBP];  // accumulators, then (in place) the activations
    layer_lds<KG0, NBP, 1, ACT_WAVES, SLOT, NBP * 4, 1, TQ0, 8>(w1f, x0, h1, lds, wv, lane, b1, lds_bias, 0,
                                                               w2f);  // hidden 1 (:277-278)
    bias_relu<NBP>(lds_bias, h1, h1, g);
    constexpr int P = KG0 & 1;  // buffer parity of block 0 of every later pass (16 and 8 blocks: even)
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      f32x4 h2[1][8];  // accumulators, then (in place) the activations
      // hidden 2, relu (:301), output tiles [8 half, 8 half + 8); prefetch: this half's head slice
      layer_lds<NBP, 8, 1, ACT_WAVES, SLOT, 32, 1, 4, 1, true, NBP>(w2f + half * 8 * 256, h1, h2, lds, wv, lane,
                                                                   b2 + half * 128, lds_bias, P, whf + half * 8 * 256);
      bias_relu<8>(lds_bias, h2, h2, g);
      // mu | log_std (:302-303) over k in this half; prefetch: the second half's first slice
      if (half == 0)
        layer_lds<8, 1, 1, ACT_WAVES, SLOT, 4, 1, 4, 8, true, 1, false, 1, NBP>(whf, h2, hd, lds, wv, lane, nullptr,
                                                                               nullptr, P, w2f + 8 * 256);
      else
        layer_lds<8, 1, 1, ACT_WAVES, SLOT, 4, 1, 4, 0, true, 1, true>(whf + 8 * 256, h2, hd, lds, wv, lane, bh,
                                                                      lds_bias, P);
    }
  } else {
    f32x4 acc[1][NBP], h[1][NBP];
    layer_lds<KG0, NBP, 1, ACT_WAVES, SLOT, NBP * 4, 1, TQ0, NBP>(w1f, x0, acc, lds, wv, lane, b1, lds_bias, 0,
                                                                 w2f);  // hidden 1 (:277-278)
    bias_relu<NBP>(lds_bias, acc, h, g);
    constexpr int P2 = KG0 & 1, P3 = (KG0 + NBP) & 1;  // buffer parity of each layer's block 0
    layer_lds<NBP, NBP, 1, ACT_WAVES, SLOT, NBP * 4, 1, 4, 1, true>(w2f, h, acc, lds, wv, lane, b2, lds_bias, P2,
                                                                    whf);  // hidden 2, relu (:301)
    bias_relu<NBP>(lds_bias, acc, h, g);
    layer_lds<NBP, 1, 1, ACT_WAVES, SLOT, 4, 1, 4, 0, true>(whf, h, hd, lds, wv, lane, bh, lds_bias, P3);  // mu | log_std
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int n = 4 * g + t;
    head[wv][m][n] = hd[0][0][t] + lds_bias[n];
  }
  __syncthreads();
  actor_finish(a, head, wv, m, g, row, ok);
}

// f16x3 policy forward (mlp_tile.h split_f16_pair / row_scale): observation row scaled per row, each
// layer's output acc * (2^-k_W / s_row) + bias, relu; 16x16x32 f16 MFMAs, 3 products per k-group.
#ifndef ACT_F16_PS
#define ACT_F16_PS 1  // weight parts per staged slice (2: both parts of a k-group per barrier)
#endif
template <int NBP>
__global__ __launch_bounds__(ACT_WAVES * 64, 2) void actor_f16_kernel(const ActorArgs a) {
  constexpr int P = 2, KG = NBP / 2, PS = ACT_F16_PS;
  constexpr int SLOT = Stage<PS * NBP, ACT_WAVES>::SLOTS * 256;
  __shared__ float head[ACT_WAVES][16][25];
  __shared__ __attribute__((aligned(16))) float lds[2 * SLOT];
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), m = lane & 15, g = lane >> 4;
  const int64_t count = a.d_count ? (int64_t)*a.d_count : a.B;
  if ((int64_t)blockIdx.x * ACT_WAVES * 16 >= count) return;  // whole workgroup past the live rows
  const int64_t row = ((int64_t)blockIdx.x * ACT_WAVES + wv) * 16 + m;
  const bool ok = row < count;
  const int O = a.O;
  const float* w1f = a.Wpk;
  const float* w2f = w1f + 2 * NBP * 256;
  const float* whf = w2f + KG * 2 * NBP * 256;
  const float* b1 = whf + KG * 2 * 256;
  const float* b2 = b1 + NBP * 16;
  const float* bh = b2 + NBP * 16;
  const float* inv_w = bh + 16;
  auto row_max = [&](float mx) {
    mx = fmaxf(mx, __shfl_xor(mx, 16));
    return fmaxf(mx, __shfl_xor(mx, 32));
  };
  float xv[8], mx = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = slot_feat(bf16_kperm(g, j), O);
    float v = 0.f;
    if (ok && k >= 0)
      v = a.obs_f64 ? (float)reinterpret_cast<const double*>(a.obs)[row * O + k]
                    : reinterpret_cast<const float*>(a.obs)[row * O + k];
    xv[j] = v;
    mx = fmaxf(mx, fabsf(v));
  }
  float s_in, inv_row;
  row_scale(row_max(mx), s_in, inv_row);
  bf16x8 x0[P][1];
  {
    u32x4v h4, l4;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const F16Pair pr = split_f16_pair(xv[2 * q], xv[2 * q + 1], s_in);
      h4[q] = pr.hi;
      l4[q] = pr.lo;
    }
    x0[0][0] = __builtin_bit_cast(bf16x8, h4);
    x0[1][0] = __builtin_bit_cast(bf16x8, l4);
  }
  f32x4 acc[NBP];
  float hf[KG][8];
  auto to_input = [&](const float* b, float f) {  // acc * f + bias, relu (mopo.py:277-278, 301), row scale
    float mx = 0.f;
#pragma unroll
    for (int c = 0; c < KG; ++c) {
      const f32x4 b0 = ld4(b + (2 * c) * 16 + 4 * g), bb1 = ld4(b + (2 * c + 1) * 16 + 4 * g);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        hf[c][t] = fmaxf(fmaf(acc[2 * c][t], f, b0[t]), 0.f);
        hf[c][4 + t] = fmaxf(fmaf(acc[2 * c + 1][t], f, bb1[t]), 0.f);
        mx = fmaxf(mx, fmaxf(hf[c][t], hf[c][4 + t]));
      }
    }
    row_scale(row_max(mx), s_in, inv_row);
  };
  layer_lds_split<1, NBP, ACT_WAVES, SLOT, P, PS, true>(w1f, x0, acc, lds, wv, lane);
  to_input(b1, inv_row * inv_w[0]);
#ifndef ACT_KNOB_NOL2
  layer_lds_split_f32<KG, NBP, ACT_WAVES, SLOT, P, PS, true>(w2f, hf, acc, lds, wv, lane, s_in);
  to_input(b2, inv_row * inv_w[1]);
#endif
  f32x4 hd[1];
#ifndef ACT_KNOB_NOHEADL
  layer_lds_split_f32<KG, 1, ACT_WAVES, SLOT, P, PS, true>(whf, hf, hd, lds, wv, lane, s_in);
#else
  hd[0] = zero4();
  for (int c = 0; c < KG; ++c) hd[0][0] += hf[c][0];
#endif
  const float f = inv_row * inv_w[2];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int n = 4 * g + t;
    head[wv][m][n] = fmaf(hd[0][t], f, bh[n]);   // mu | log_std (mopo.py:302-303)
  }
  __syncthreads();
  actor_finish(a, head, wv, m, g, row, ok);
}

// bf16x6 policy forward: every f32 operand split EXACTLY into 3 RN bf16 parts (mlp_tile.h split_bf16), the 6
// products p + q < 3 per k-group on the bf16 MFMA, f32 accumulate and f32 epilogues -- the reference's f32
// operands, like the bf16x6 ensemble beside it; the f16x3 kernel's structure without scales
#ifndef ACT_X6_HEAD_PS
#define ACT_X6_HEAD_PS 3
#endif
template <int NBP>
__global__ __launch_bounds__(ACT_WAVES * 64, 2) void actor_x6_kernel(const ActorArgs a) {
  constexpr int P = 3, KG = NBP / 2;
  constexpr int SLOT = Stage<NBP, ACT_WAVES>::SLOTS * 256;
  __shared__ float head[ACT_WAVES][16][25];
  __shared__ __attribute__((aligned(16))) float lds[2 * SLOT];
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), m = lane & 15, g = lane >> 4;
  const int64_t count = a.d_count ? (int64_t)*a.d_count : a.B;
  if ((int64_t)blockIdx.x * ACT_WAVES * 16 >= count) return;  // whole workgroup past the live rows
  const int64_t row = ((int64_t)blockIdx.x * ACT_WAVES + wv) * 16 + m;
  const bool ok = row < count;
  const int O = a.O;
  const float* w1f = a.Wpk;
  const float* w2f = w1f + P * NBP * 256;
  const float* whf = w2f + KG * P * NBP * 256;
  const float* b1 = whf + KG * P * 256;
  const float* b2 = b1 + NBP * 16;
  const float* bh = b2 + NBP * 16;
  bf16x8 x0[P][1];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = slot_feat(bf16_kperm(g, j), O);
    float v = 0.f;
    if (ok && k >= 0)
      v = a.obs_f64 ? (float)reinterpret_cast<const double*>(a.obs)[row * O + k]
                    : reinterpret_cast<const float*>(a.obs)[row * O + k];
    short parts[P];
    split_bf16<P>(v, parts);
#pragma unroll
    for (int p = 0; p < P; ++p) x0[p][0][j] = parts[p];
  }
  f32x4 acc[NBP];
  float hf[KG][8];
  auto to_input = [&](const float* b) {  // acc + bias, relu (mopo.py:277-278, 301)
#pragma unroll
    for (int c = 0; c < KG; ++c) {
      const f32x4 b0 = ld4(b + (2 * c) * 16 + 4 * g), bb1 = ld4(b + (2 * c + 1) * 16 + 4 * g);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        hf[c][t] = fmaxf(acc[2 * c][t] + b0[t], 0.f);
        hf[c][4 + t] = fmaxf(acc[2 * c + 1][t] + bb1[t], 0.f);
      }
    }
  };
  layer_lds_split<1, NBP, ACT_WAVES, SLOT, P, 1, false>(w1f, x0, acc, lds, wv, lane);
  to_input(b1);
  layer_lds_split_f32<KG, NBP, ACT_WAVES, SLOT, P, 1, false>(w2f, hf, acc, lds, wv, lane);
  to_input(b2);
  f32x4 hd[1];
  // the head's P parts of a k-group as one slice (3 fragments, contiguous in the packing): KG barriers, not P KG
  layer_lds_split_f32<KG, 1, ACT_WAVES, SLOT, P, ACT_X6_HEAD_PS, false>(whf, hf, hd, lds, wv, lane);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int n = 4 * g + t;
    head[wv][m][n] = hd[0][t] + bh[n];   // mu | log_std (mopo.py:302-303)
  }
  __syncthreads();
  actor_finish(a, head, wv, m, g, row, ok);
}

// f16x3 policy forward over R row blocks per wave (layer_f16_rows): actor_f16_kernel's arithmetic,
// product for product, with layer 2's first slice prefetched during layer 1's last one and the whole
// head ([mu | log_std], 2 KG fragments) prefetched during layer 2's last slice, so no layer starts on
// an exposed copy and the head runs behind ONE barrier instead of 2 KG.
#ifndef ACT_F16_R
#define ACT_F16_R 0  // 0: actor_f16_kernel; R >= 1: actor_f16r_kernel<R> (A/B builds only: not compiled at 0)
#endif
#if ACT_F16_R > 0
template <int NBP, int R>
__global__ __launch_bounds__(ACT_WAVES * 64, R == 1 ? 2 : 1) void actor_f16r_kernel(const ActorArgs a) {
  constexpr int KG = NBP / 2;
  constexpr int SLOT = Stage<NBP, ACT_WAVES>::SLOTS * 256;   // also holds the head's 2 KG = NBP fragments
  __shared__ float head[ACT_WAVES][16][25];
  __shared__ __attribute__((aligned(16))) float lds[2 * SLOT];
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), m = lane & 15, g = lane >> 4;
  const int64_t count = a.d_count ? (int64_t)*a.d_count : a.B;
  if ((int64_t)blockIdx.x * ACT_WAVES * 16 * R >= count) return;  // whole workgroup past the live rows
  const int64_t row0 = ((int64_t)blockIdx.x * ACT_WAVES + wv) * 16 * R + m;   // row block r: row0 + 16 r
  const int O = a.O;
  const float* w1f = a.Wpk;
  const float* w2f = w1f + 2 * NBP * 256;
  const float* whf = w2f + KG * 2 * NBP * 256;
  const float* b1 = whf + KG * 2 * 256;
  const float* b2 = b1 + NBP * 16;
  const float* bh = b2 + NBP * 16;
  const float* inv_w = bh + 16;
  auto row_max = [&](float mx) {
    mx = fmaxf(mx, __shfl_xor(mx, 16));
    return fmaxf(mx, __shfl_xor(mx, 32));
  };
  float xin[R][1][8], sc[R], inv[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t row = row0 + 16 * r;
    const bool ok = row < count;
    float mx = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = slot_feat(bf16_kperm(g, j), O);
      float v = 0.f;
      if (ok && k >= 0)
        v = a.obs_f64 ? (float)reinterpret_cast<const double*>(a.obs)[row * O + k]
                      : reinterpret_cast<const float*>(a.obs)[row * O + k];
      xin[r][0][j] = v;
      mx = fmaxf(mx, fabsf(v));
    }
    row_scale(row_max(mx), sc[r], inv[r]);
  }
  f32x4 acc[R][NBP];
  float hf[R][KG][8];
  auto to_input = [&](int r, const float* b, float f) {  // acc * f + bias, relu (mopo.py:277-278, 301), row scale
    float mx = 0.f;
#pragma unroll
    for (int c = 0; c < KG; ++c) {
      const f32x4 b0 = ld4(b + (2 * c) * 16 + 4 * g), bb1 = ld4(b + (2 * c + 1) * 16 + 4 * g);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        hf[r][c][t] = fmaxf(fmaf(acc[r][2 * c][t], f, b0[t]), 0.f);
        hf[r][c][4 + t] = fmaxf(fmaf(acc[r][2 * c + 1][t], f, bb1[t]), 0.f);
        mx = fmaxf(mx, fmaxf(hf[r][c][t], hf[r][c][4 + t]));
      }
    }
    row_scale(row_max(mx), sc[r], inv[r]);
  };
  // layer 1 (prefetching layer 2's first slice), layer 2 (prefetching the whole head); both have an
  // even slice count, so each prefetch lands in buffer 0
  layer_f16_rows<1, NBP, R, ACT_WAVES, SLOT, NBP, false, NBP>(w1f, xin, acc, lds, wv, lane, sc, nullptr, nullptr, w2f);
#pragma unroll
  for (int r = 0; r < R; ++r) to_input(r, b1, inv[r] * inv_w[0]);
  layer_f16_rows<KG, NBP, R, ACT_WAVES, SLOT, NBP, false, 2 * KG, true>(w2f, hf, acc, lds, wv, lane, sc, nullptr, nullptr,
                                                                      whf);
#pragma unroll
  for (int r = 0; r < R; ++r) to_input(r, b2, inv[r] * inv_w[1]);
  f32x4 hd[R];
  head_f16_rows<KG, R>(hf, hd, lds, lane, sc);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t row = row0 + 16 * r;
    const float f = inv[r] * inv_w[2];
    if (r > 0) __syncthreads();   // every wave is done with the previous row block's head rows
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int n = 4 * g + t;
      head[wv][m][n] = fmaf(hd[r][t], f, bh[n]);   // mu | log_std (mopo.py:302-303)
    }
    __syncthreads();
    actor_finish(a, head, wv, m, g, row, row < count);
  }
}
#endif

// f16x3 policy forward over a 3-slot LDS ring (ACT_F16_RING; bnn.hip bnn_fwd_f16q_kernel's pipeline):
// actor_f16_kernel's arithmetic, product for product, with the weight slices as ONE stream -- layer 1
// (2 slices: the fp16 parts), layer 2 (2 KG slices) and the whole head (its 2 KG fragments as one
// slice) -- slice j + 2 copied while slice j is consumed, behind counted vmcnt + raw barriers.  The
// hidden biases ride into LDS once, ahead of the first slices; the head's output rows reuse a ring slot.
// Same-box A/B (round 4): actor 0.062 -> 0.054 ms alone, but the split rollout 1.6 % slower (203 VGPRs
// beside the concurrent ensemble launch of the other row part), so it runs only where the actor runs
// alone (ActorArgs::alone: unsplit rollouts -- one-step C3, compacting walker / hopper rollouts)
#ifndef ACT_F16_RING
#define ACT_F16_RING 1
#endif
#if ACT_F16_RING
template <int NBP>
__global__ __launch_bounds__(ACT_WAVES * 64, 2) void actor_f16q_kernel(const ActorArgs a) {
  static_assert(NBP == 16, "ring actor: hidden 256");
  constexpr int KG = NBP / 2, NS = 2 + 2 * KG + 1;  // layer 1, layer 2, head
  constexpr int SLOT = Stage<NBP, ACT_WAVES>::SLOTS * 256, PER = Stage<NBP, ACT_WAVES>::PER;
  static_assert(2 * KG <= NBP, "the head's fragments fit one slice");
  static_assert(ACT_WAVES * 16 * 25 <= SLOT, "the head rows fit one ring slot");
  constexpr int BQ = (2 * NBP * 16 + 16) / 4;   // b1 | b2 | bh quads (contiguous in the packing)
  __shared__ __attribute__((aligned(16))) float lds[3 * SLOT + (BQ + 63) / 64 * 256];  // one array (see layer_lds)
  float* lds_bias = lds + 3 * SLOT;
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), m = lane & 15, g = lane >> 4;
  const int64_t count = a.d_count ? (int64_t)*a.d_count : a.B;
  if ((int64_t)blockIdx.x * ACT_WAVES * 16 >= count) return;  // whole workgroup past the live rows
  const int64_t row = ((int64_t)blockIdx.x * ACT_WAVES + wv) * 16 + m;
  const bool ok = row < count;
  const int O = a.O;
  const float* w1f = a.Wpk;
  const float* w2f = w1f + 2 * NBP * 256;
  const float* whf = w2f + KG * 2 * NBP * 256;
  const float* b1 = whf + KG * 2 * 256;
  const float* b2 = b1 + NBP * 16;
  const float* bh = b2 + NBP * 16;
  const float* inv_w = bh + 16;
  auto row_max = [&](float mx) {
    mx = fmaxf(mx, __shfl_xor(mx, 16));
    return fmaxf(mx, __shfl_xor(mx, 32));
  };
  float xv[8], mx = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = slot_feat(bf16_kperm(g, j), O);
    float v = 0.f;
    if (ok && k >= 0)
      v = a.obs_f64 ? (float)reinterpret_cast<const double*>(a.obs)[row * O + k]
                    : reinterpret_cast<const float*>(a.obs)[row * O + k];
    xv[j] = v;
    mx = fmaxf(mx, fabsf(v));
  }
  // per-matrix weight scales in SGPRs (a vector load of one later would be waited for with vmcnt(0),
  // draining the slices in flight)
  float sw[3];
#pragma unroll
  for (int l = 0; l < 3; ++l) sw[l] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(inv_w[l])));
  (void)bh;
  float s_in, inv_row;
  row_scale(row_max(mx), s_in, inv_row);
  // slice J: 0, 1 layer 1's parts, 2 .. 2 KG + 1 layer 2 (k-group (J - 2) / 2, part (J - 2) % 2), 2 KG + 2 the head
  auto issue = [&](auto jc) {
    constexpr int J = decltype(jc)::value;
    if constexpr (J < NS) {
      const float* src = J < 2 ? w1f + J * NBP * 256 : (J < NS - 1 ? w2f + (J - 2) * NBP * 256 : whf);
      stage_slice<NBP, ACT_WAVES>(src, lds + (J % 3) * SLOT, wv, lane);
    }
  };
  __builtin_amdgcn_sched_barrier(0);
  stage_bias<BQ, ACT_WAVES>(b1, lds_bias, wv, lane);
  issue(std::integral_constant<int, 0>{});
  issue(std::integral_constant<int, 1>{});
  auto bias4 = [&](int off) { return __builtin_bit_cast(f32x4, *reinterpret_cast<const bf16x8*>(lds_bias + off)); };
  f32x4 acc[NBP];
  float hf[KG][8];
  bf16x8 cur[2];
  auto to_input = [&](int boff, float f) {  // acc * f + bias, relu (mopo.py:277-278, 301), row scale
    float mx = 0.f;
#pragma unroll
    for (int c = 0; c < KG; ++c) {
      const f32x4 b0 = bias4(boff + (2 * c) * 16 + 4 * g), bb1 = bias4(boff + (2 * c + 1) * 16 + 4 * g);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        hf[c][t] = fmaxf(fmaf(acc[2 * c][t], f, b0[t]), 0.f);
        hf[c][4 + t] = fmaxf(fmaf(acc[2 * c + 1][t], f, bb1[t]), 0.f);
        mx = fmaxf(mx, fmaxf(hf[c][t], hf[c][4 + t]));
      }
    }
    row_scale(row_max(mx), s_in, inv_row);
  };
  auto split = [&](const float (&v)[8]) {
    u32x4v h4, l4;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const F16Pair pr = split_f16_pair(v[2 * q], v[2 * q + 1], s_in);
      h4[q] = pr.hi;
      l4[q] = pr.lo;
    }
    cur[0] = __builtin_bit_cast(bf16x8, h4);
    cur[1] = __builtin_bit_cast(bf16x8, l4);
  };
  auto top = [&](auto jc) {  // slice J landed for every wave; slice J + 2 goes out
    constexpr int J = decltype(jc)::value;
    wait_vm_lgkm0<(J + 1 < NS ? PER : 0)>();
    __builtin_amdgcn_s_barrier();
    issue(std::integral_constant<int, J + 2>{});
    __builtin_amdgcn_sched_barrier(0);
  };
  // layer 1 and layer 2: slice J (k-group kg, weight part p) feeds NBP blocks
  auto slices = [&](auto j0c, auto kgc, auto& in) {
    constexpr int J0 = decltype(j0c)::value, KGL = decltype(kgc)::value;
#pragma unroll
    for (int nb = 0; nb < NBP; ++nb) acc[nb] = zero4();
    RingRun<J0, J0 + 2 * KGL>::run([&](auto jc) {
      constexpr int J = decltype(jc)::value, s = J - J0, kg = s / 2, p = s % 2;
      if constexpr (p == 0) split(in[kg]);
      top(jc);
      const float* b = lds + (J % 3) * SLOT;
      bf16x8 fr_next = *reinterpret_cast<const bf16x8*>(b + lane * 4);
#pragma unroll
      for (int nb = 0; nb < NBP; ++nb) {
        const bf16x8 fr = fr_next;
        if (nb + 1 < NBP) fr_next = *reinterpret_cast<const bf16x8*>(b + ((nb + 1) * 64 + lane) * 4);
#pragma unroll
        for (int q = 1 - p; q >= 0; --q) acc[nb] = mfma_16x16x32<true>(fr, cur[q], acc[nb]);
      }
    });
  };
  {
    float x1[1][8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x1[0][j] = xv[j];
    slices(std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{}, x1);
  }
  to_input(0, inv_row * sw[0]);
  slices(std::integral_constant<int, 2>{}, std::integral_constant<int, KG>{}, hf);
  to_input(NBP * 16, inv_row * sw[1]);
  // the head: its 2 KG fragments (k-group kg: part 0 at 2 kg, part 1 at 2 kg + 1) in slice NS - 1
  split(hf[0]);
  top(std::integral_constant<int, NS - 1>{});
  f32x4 hd = zero4();
  {
    const float* b = lds + ((NS - 1) % 3) * SLOT;
#pragma unroll
    for (int kg = 0; kg < KG; ++kg) {
      if (kg > 0) split(hf[kg]);
      const bf16x8 f0 = *reinterpret_cast<const bf16x8*>(b + ((2 * kg) * 64 + lane) * 4);
      const bf16x8 f1 = *reinterpret_cast<const bf16x8*>(b + ((2 * kg + 1) * 64 + lane) * 4);
      hd = mfma_16x16x32<true>(f0, cur[1], hd);   // the product order of layer_lds_split_f32
      hd = mfma_16x16x32<true>(f0, cur[0], hd);
      hd = mfma_16x16x32<true>(f1, cur[0], hd);
    }
  }
  // mu | log_std (mopo.py:302-303) into a free ring slot (slot (NS - 1) % 3 holds the head's weights,
  // the slots of slices NS and NS + 1 were never filled)
  float (&head)[ACT_WAVES][16][25] = *reinterpret_cast<float (*)[ACT_WAVES][16][25]>(lds + (NS % 3) * SLOT);
  const float f = inv_row * sw[2];
  const f32x4 bn = bias4(2 * NBP * 16 + 4 * g);
#pragma unroll
  for (int t = 0; t < 4; ++t) head[wv][m][4 * g + t] = fmaf(hd[t], f, bn[t]);
  __syncthreads();
  actor_finish(a, head, wv, m, g, row, ok);
}
#endif

int launch_actor(const ActorArgs& a, hipStream_t s) {
  if (a.B == 0) return 0;
  MOPO_REQUIRE(!a.xs || (a.xs_mu && a.xs_sigma && a.xs_in == a.O + a.A && a.xs_in <= XS_STRIDE),
               "actor: scaled-input rows need the scaler and obs_dim + act_dim <= 32");
  MOPO_REQUIRE(a.A >= 1 && 2 * a.A <= 16, "actor: act_dim must be in [1, 8]");
  MOPO_REQUIRE(a.O >= 1 && a.O <= 32, "actor: obs_dim must be in [1, 32]");
  MOPO_REQUIRE(a.Wpk, "actor: packed weights required");
  dim3 grid(ceil_div((int)a.B, 16 * ACT_WAVES)), block(64 * ACT_WAVES);
#if ACT_F16_R > 0
  if (a.dtype == DT_F16X3) {
    constexpr int R = ACT_F16_R;
    const dim3 gr(ceil_div((int)a.B, 16 * ACT_WAVES * R));
    if (a.Hp == 256) hipLaunchKernelGGL((actor_f16r_kernel<16, R>), gr, block, 0, s, a);
    else if (a.Hp == 32) hipLaunchKernelGGL((actor_f16r_kernel<2, R>), gr, block, 0, s, a);
    else return fail("actor f16x3: unsupported hidden size (256 or 32)");
    MOPO_HIP(hipGetLastError());
    return 0;
  }
#endif
  if (a.dtype == DT_BF16X6) {
    if (a.Hp == 256) hipLaunchKernelGGL(actor_x6_kernel<16>, grid, block, 0, s, a);
    else if (a.Hp == 32) hipLaunchKernelGGL(actor_x6_kernel<2>, grid, block, 0, s, a);
    else return fail("actor bf16x6: unsupported hidden size (256 or 32)");
    MOPO_HIP(hipGetLastError());
    return 0;
  }
  if (a.dtype == DT_F16X3) {
#if ACT_F16_RING
    if (a.alone && a.Hp == 256) hipLaunchKernelGGL(actor_f16q_kernel<16>, grid, block, 0, s, a);
    else
#endif
    if (a.Hp == 256) hipLaunchKernelGGL(actor_f16_kernel<16>, grid, block, 0, s, a);
    else if (a.Hp == 32) hipLaunchKernelGGL(actor_f16_kernel<2>, grid, block, 0, s, a);
    else return fail("actor f16x3: unsupported hidden size (256 or 32)");
    MOPO_HIP(hipGetLastError());
    return 0;
  }
  const int KG0 = ceil_div(a.O, 16);
  if (a.Hp == 256 && KG0 == 2 && tail_steps(a.O) == 1)  // halfcheetah / walker2d: 17 = 16 + 1
    hipLaunchKernelGGL((actor_kernel<2, 16, 1>), grid, block, 0, s, a);
  else if (a.Hp == 256 && KG0 == 2)
    hipLaunchKernelGGL((actor_kernel<2, 16>), grid, block, 0, s, a);
  else if (a.Hp == 256 && KG0 == 1)
    hipLaunchKernelGGL((actor_kernel<1, 16>), grid, block, 0, s, a);
  else if (a.Hp == 32 && KG0 == 2)
    hipLaunchKernelGGL((actor_kernel<2, 2>), grid, block, 0, s, a);
  else if (a.Hp == 32 && KG0 == 1)
    hipLaunchKernelGGL((actor_kernel<1, 2>), grid, block, 0, s, a);
  else
    return fail("actor: unsupported hidden size (256 or 32)");
  MOPO_HIP(hipGetLastError());
  return 0;
}

}  // namespace mopo

using namespace mopo;

extern "C" int64_t mopo_sac_param_count(int O, int A, int H) {
  int64_t pi = (int64_t)O * H + H + (int64_t)H * H + H + 2 * ((int64_t)H * A + A);
  int64_t q = (int64_t)(O + A) * H + H + (int64_t)H * H + H + H + 1;
  return pi + 2 * q;
}

extern "C" int mopo_actor_forward_dtype(const float* P, int O, int A, int H, const void* obs, int obs_f64, int64_t B,
                                        const float* eps, uint64_t seed, uint32_t step, float* act, float* mu,
                                        int dtype, void* stream) {
  MOPO_REQUIRE(P && obs, "mopo_actor_forward: NULL pointer");
  MOPO_REQUIRE(dtype == DT_FP32 || dtype == DT_F16X3 || dtype == DT_BF16X6,
               "mopo_actor_forward: dtype must be 0 (fp32), 3 (bf16x6) or 4 (f16x3)");
  if (B == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int split = dtype == DT_F16X3 ? 1 : (dtype == DT_BF16X6 ? 2 : 0);
  float* wpk = nullptr;
  MOPO_HIP(hipMallocAsync((void**)&wpk, actor_packed_floats(O, H, split) * sizeof(float), s));
  int rc = pack_actor(P, O, A, H, wpk, s, split);
  if (rc == 0) {
    ActorArgs a{};
    a.P = P; a.Wpk = wpk; a.O = O; a.A = A; a.Hp = H; a.dtype = dtype;
    a.obs = obs; a.obs_f64 = obs_f64; a.B = B;
    a.eps = eps; a.seed = seed; a.step = step;
    a.act = act; a.mu = mu;
    a.stage_base = -1;
    rc = launch_actor(a, s);
  }
  (void)hipFreeAsync(wpk, s);
  return rc;
}

extern "C" int mopo_actor_forward(const float* P, int O, int A, int H, const void* obs, int obs_f64, int64_t B,
                                  const float* eps, uint64_t seed, uint32_t step, float* act, float* mu,
                                  void* stream) {
  return mopo_actor_forward_dtype(P, O, A, H, obs, obs_f64, B, eps, seed, step, act, mu, DT_FP32, stream);
}
