// Squashed-Gaussian policy forward (rollout actions).
//
// Replaces MOPO.get_action_meta -> mlp_gaussian_policy + apply_squashing_func
// (mopo/algorithms/mopo.py:468-485, 275-308, 286-296):
//   net = relu(relu(s W1 + b1) W2 + b2); mu = net Wmu + bmu; log_std = clip(net Wls + bls, -20, 2)
//   pi = tanh(mu + eps * exp(log_std)),  mu_out = tanh(mu)
// Same register-resident transposed-MFMA scheme as the BNN forward (bnn.hip), reading the
// weights straight from the SAC parameter buffer in TF [in, out] layout (the policy changes
// every SAC step, so no repacking).  One 64-thread wave per 16-row tile.
#include "actor.h"

namespace mopo {

// A-operand fragment from a TF-layout [K][N] matrix: lane (n = lane&15, g) gets
// W[kg*16 + 4g + t][nb*16 + n], t = 0..3
__device__ __forceinline__ f32x4 ld_tf(const float* __restrict__ W, int K, int N, int kg, int nb, int lane) {
  const int n = nb * 16 + (lane & 15), k0 = kg * 16 + 4 * (lane >> 4);
  f32x4 v;
#pragma unroll
  for (int t = 0; t < 4; ++t) v[t] = (n < N && k0 + t < K) ? W[(k0 + t) * N + n] : 0.f;
  return v;
}

template <int KG, int NB>
__device__ __forceinline__ void tf_layer(const float* __restrict__ W, int K, int N, const f32x4 (&in)[KG],
                                         f32x4 (&acc)[NB], int lane) {
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) acc[nb] = zero4();
#pragma unroll
  for (int kg = 0; kg < KG; ++kg) {
    f32x4 w[NB];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) w[nb] = ld_tf(W, K, N, kg, nb, lane);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) acc[nb] = mfma4(w[nb][t], in[kg][t], acc[nb]);
  }
}

template <int NB>
__device__ __forceinline__ void bias_relu(const float* __restrict__ b, int N, const f32x4 (&acc)[NB],
                                          f32x4 (&out)[NB], int g) {
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int n = nb * 16 + 4 * g + t;
      const float v = acc[nb][t] + (n < N ? b[n] : 0.f);
      out[nb][t] = fmaxf(v, 0.f);
    }
}

__device__ __forceinline__ void actor_noise(uint64_t seed, uint32_t step, int64_t uid, int A, float* z) {
  for (int blk = 0; blk * 4 < A; ++blk) {
    u32x4 c{(uint32_t)uid, (uint32_t)((uint64_t)uid >> 32) ^ ((uint32_t)blk << 20), step, RNG_ACT};
    u32x4 r = philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    float z0, z1, z2, z3;
    box_muller(r.x, r.y, z0, z1);
    box_muller(r.z, r.w, z2, z3);
    float zz[4] = {z0, z1, z2, z3};
    for (int i = 0; i < 4 && blk * 4 + i < A; ++i) z[blk * 4 + i] = zz[i];
  }
}

template <int KG0, int NBP>
__global__ __launch_bounds__(64) void actor_kernel(const ActorArgs a) {
  __shared__ float head[16][17];
  const int lane = threadIdx.x, m = lane & 15, g = lane >> 4;
  const int64_t count = a.d_count ? (int64_t)*a.d_count : a.B;
  const int64_t row0 = (int64_t)blockIdx.x * 16;
  if (row0 >= count) return;
  const int O = a.O, A = a.A, Hp = a.Hp;
  const float* W1 = a.P;
  const float* b1 = W1 + O * Hp;
  const float* W2 = b1 + Hp;
  const float* b2 = W2 + Hp * Hp;
  const float* Wm = b2 + Hp;
  const float* bm = Wm + Hp * A;
  const float* Wl = bm + A;
  const float* bl = Wl + Hp * A;
  const int64_t row = row0 + m;
  const bool ok = row < count;
  f32x4 x0[KG0];
#pragma unroll
  for (int kg = 0; kg < KG0; ++kg)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int k = kg * 16 + 4 * g + t;
      float v = 0.f;
      if (ok && k < O)
        v = a.obs_f64 ? (float)reinterpret_cast<const double*>(a.obs)[row * O + k]
                      : reinterpret_cast<const float*>(a.obs)[row * O + k];
      x0[kg][t] = v;
    }
  f32x4 acc[NBP], h[NBP];
  tf_layer<KG0, NBP>(W1, O, Hp, x0, acc, lane);
  bias_relu<NBP>(b1, Hp, acc, h, g);
  tf_layer<NBP, NBP>(W2, Hp, Hp, h, acc, lane);
  bias_relu<NBP>(b2, Hp, acc, h, g);
  // head: one 16-wide block, n < A -> mu, A <= n < 2A -> log_std
  f32x4 hd = zero4();
#pragma unroll
  for (int kg = 0; kg < NBP; ++kg) {
    const int n = lane & 15, k0 = kg * 16 + 4 * g;
    f32x4 w;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int k = k0 + t;
      w[t] = (k < Hp && n < 2 * A) ? (n < A ? Wm[k * A + n] : Wl[k * A + (n - A)]) : 0.f;
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) hd = mfma4(w[t], h[kg][t], hd);
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int n = 4 * g + t;
    float bias = n < A ? bm[n] : (n < 2 * A ? bl[n - A] : 0.f);
    head[m][n] = hd[t] + bias;
  }
  __syncthreads();
  if (g != 0 || !ok) return;
  float z[16];
  const int64_t uid = a.d_uid ? a.d_uid[row] : row + a.uid_offset;
  if (a.eps) {
    for (int j = 0; j < A; ++j) z[j] = a.eps[row * A + j];
  } else {
    actor_noise(a.seed, a.step, uid, A, z);
  }
  int64_t pos = -1;
  if (a.pool_act) {
    pos = a.stage_base >= 0 ? a.stage_base + row : (a.pool_state[0] + row) % a.pool_max;
  }
  for (int j = 0; j < A; ++j) {
    const float mu = head[m][j];
    const float ls = fminf(fmaxf(head[m][A + j], -20.f), 2.f);  // mopo.py:304
    const float sd = expf(ls);                                  // mopo.py:305
    const float u = mu + z[j] * sd;                             // mopo.py:306
    const float act = tanhf(u);                                 // mopo.py:295
    if (a.act) a.act[row * A + j] = act;
    if (a.mu) a.mu[row * A + j] = tanhf(mu);                    // mopo.py:294
    if (pos >= 0) a.pool_act[pos * A + j] = act;
  }
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
    } else {
      u32x4 c{(uint32_t)uid, (uint32_t)((uint64_t)uid >> 32), a.step, RNG_MODEL};
      u32x4 r = philox(c, (uint32_t)a.seed, (uint32_t)(a.seed >> 32));
      sel = a.elites[(int)(((uint64_t)r.x * (uint64_t)a.n_elites) >> 32)];
    }
    a.sel_out[row] = sel;
  }
}

int launch_actor(const ActorArgs& a, hipStream_t s) {
  if (a.B == 0) return 0;
  MOPO_REQUIRE(a.A >= 1 && 2 * a.A <= 16, "actor: act_dim must be in [1, 8]");
  MOPO_REQUIRE(a.O >= 1 && a.O <= 32, "actor: obs_dim must be in [1, 32]");
  dim3 grid(ceil_div((int)a.B, 16)), block(64);
  const int KG0 = ceil_div(a.O, 16);
  if (a.Hp == 256 && KG0 == 2)
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

extern "C" int mopo_actor_forward(const float* P, int O, int A, int H, const void* obs, int obs_f64, int64_t B,
                                  const float* eps, uint64_t seed, uint32_t step, float* act, float* mu,
                                  void* stream) {
  MOPO_REQUIRE(P && obs, "mopo_actor_forward: NULL pointer");
  ActorArgs a{};
  a.P = P; a.O = O; a.A = A; a.Hp = H;
  a.obs = obs; a.obs_f64 = obs_f64; a.B = B;
  a.eps = eps; a.seed = seed; a.step = step;
  a.act = act; a.mu = mu;
  a.stage_base = -1;
  return launch_actor(a, (hipStream_t)stream);
}
