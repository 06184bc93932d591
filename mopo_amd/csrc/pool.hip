// Device-resident SimpleReplayPool kernels.
//
// Replaces FlexibleReplayPool.add_samples / _advance / random_indices / batch_by_indices
// (softlearning/replay_pools/flexible_replay_pool.py:45-48, 57-92, 121-135) for the
// SimpleReplayPool field set (simple_replay_pool.py:48-70).  SoA layout, one array per field,
// ring index (pointer + i) % max_size, pointer/size live on the device (int64[2]) so a whole
// rollout or SAC epoch can run without host synchronisation.
#include "internal.h"

namespace mopo {

__global__ void pool_add_kernel(const mopo_pool_desc p, int O, int A, const float* obs, const float* act,
                                const float* rew, const uint8_t* term, const float* nobs, int64_t n) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t pos = (p.d_state[0] + i) % p.max_size;
  for (int k = 0; k < O; ++k) {
    p.d_obs[pos * O + k] = obs[i * O + k];
    p.d_next_obs[pos * O + k] = nobs[i * O + k];
  }
  for (int k = 0; k < A; ++k) p.d_act[pos * A + k] = act[i * A + k];
  p.d_rew[pos] = rew[i];
  p.d_term[pos] = term[i];
}

// _advance(count) (flexible_replay_pool.py:45-48)
__global__ void pool_advance_kernel(int64_t* state, int64_t max_size, int64_t n) {
  state[0] = (state[0] + n) % max_size;
  state[1] = min(state[1] + n, max_size);
}

__global__ void pool_gather_kernel(const mopo_pool_desc p, int O, int A, const int64_t* idx, int64_t n,
                                   float* dobs, float* dact, float* drew, float* dterm, float* dnobs,
                                   int64_t off) {
  // one thread per (row, column) over the widest field for coalesced stores
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int W = O;
  if (t >= n * W) return;
  const int64_t i = t / W;
  const int k = (int)(t % W);
  const int64_t src = idx[i];
  const int64_t dst = off + i;
  if (dobs) dobs[dst * O + k] = p.d_obs[src * O + k];
  if (dnobs) dnobs[dst * O + k] = p.d_next_obs[src * O + k];
  if (dact && k < A) dact[dst * A + k] = p.d_act[src * A + k];
  if (k == 0) {
    if (drew) drew[dst] = p.d_rew[src];
    if (dterm) dterm[dst] = (float)p.d_term[src];  // terminals placeholder is f32 (mopo.py:252-256)
  }
}

// random_indices perf mode: Philox uniform in [0, size)
__global__ void pool_rand_kernel(const int64_t* state, int64_t n, uint64_t seed, uint32_t step, int64_t* out) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t size = (uint64_t)state[1];
  u32x4 c{(uint32_t)i, (uint32_t)((uint64_t)i >> 32), step, RNG_SAC};
  u32x4 r = philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  const uint64_t u = ((uint64_t)r.x << 32) | r.y;
  out[i] = size ? (int64_t)(((unsigned __int128)u * size) >> 64) : 0;
}

int pool_advance(int64_t* state, int64_t max_size, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(pool_advance_kernel, dim3(1), dim3(1), 0, s, state, max_size, n);
  MOPO_HIP(hipGetLastError());
  return 0;
}

}  // namespace mopo

using namespace mopo;

static int check_pool(const mopo_pool_desc* p) {
  MOPO_REQUIRE(p != nullptr, "pool: NULL descriptor");
  MOPO_REQUIRE(p->d_obs && p->d_act && p->d_rew && p->d_term && p->d_next_obs && p->d_state,
               "pool: NULL field pointer");
  MOPO_REQUIRE(p->max_size > 0, "pool: max_size must be positive");
  return 0;
}

extern "C" int mopo_pool_add(const mopo_pool_desc* p, int O, int A, const float* obs, const float* act,
                             const float* rew, const uint8_t* term, const float* nobs, int64_t n,
                             void* stream) {
  if (check_pool(p)) return -1;
  if (n == 0) return 0;
  MOPO_REQUIRE(n <= p->max_size, "pool_add: more samples than the pool holds");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(pool_add_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, *p, O, A, obs, act,
                     rew, term, nobs, n);
  MOPO_HIP(hipGetLastError());
  return pool_advance(p->d_state, p->max_size, n, s);
}

// ---- append staged blocks in a given order (multi-GPU: the all-gathered per-step blocks, step-major
// then rank-major = the row order of one single-GPU rollout over the concatenated shards).
// Block b (at d_blocks + b * stride bytes) holds B rows as obs f32[B][O] | act f32[B][A] | rew f32[B] |
// next_obs f32[B][O] | term u8[B] (mopo_pool_staged_block_offsets); its first counts[b] rows are live.
__global__ void pool_add_blocks_kernel(const mopo_pool_desc p, int O, int A, const uint8_t* __restrict__ blocks,
                                       int64_t stride, int nb, int64_t B, const int64_t* __restrict__ counts) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (i >= B || i >= counts[b]) return;
  int64_t prefix = 0;
  for (int q = 0; q < b; ++q) prefix += counts[q];
  const uint8_t* base = blocks + b * stride;
  const float* obs = reinterpret_cast<const float*>(base);
  const float* act = obs + B * O;
  const float* rew = act + B * A;
  const float* nobs = rew + B;
  const uint8_t* term = reinterpret_cast<const uint8_t*>(nobs + B * O);
  const int64_t pos = (p.d_state[0] + prefix + i) % p.max_size;
  for (int k = 0; k < O; ++k) {
    p.d_obs[pos * O + k] = obs[i * O + k];
    p.d_next_obs[pos * O + k] = nobs[i * O + k];
  }
  for (int k = 0; k < A; ++k) p.d_act[pos * A + k] = act[i * A + k];
  p.d_rew[pos] = rew[i];
  p.d_term[pos] = term[i];
}

__global__ void pool_advance_counts_kernel(int64_t* state, int64_t max_size, const int64_t* counts, int nb) {
  int64_t n = 0;
  for (int q = 0; q < nb; ++q) n += counts[q];
  state[0] = (state[0] + n) % max_size;
  state[1] = min(state[1] + n, max_size);
}

extern "C" int64_t mopo_pool_staged_block_bytes(int O, int A, int64_t B) {
  return ((B * (2 * O + A + 1) * 4 + B) + 255) / 256 * 256;
}

extern "C" int mopo_pool_add_blocks(const mopo_pool_desc* p, int O, int A, const uint8_t* d_blocks, int64_t stride,
                                    int n_blocks, int64_t B, const int64_t* d_counts, void* stream) {
  if (check_pool(p)) return -1;
  MOPO_REQUIRE(d_blocks && d_counts && n_blocks >= 0 && B >= 0, "pool_add_blocks: bad argument");
  MOPO_REQUIRE(stride >= mopo_pool_staged_block_bytes(O, A, B), "pool_add_blocks: stride smaller than a block");
  if (n_blocks == 0 || B == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(pool_add_blocks_kernel, dim3((unsigned)((B + 255) / 256), n_blocks), dim3(256), 0, s, *p, O, A,
                     d_blocks, stride, n_blocks, B, d_counts);
  MOPO_HIP(hipGetLastError());
  hipLaunchKernelGGL(pool_advance_counts_kernel, dim3(1), dim3(1), 0, s, p->d_state, p->max_size, d_counts, n_blocks);
  MOPO_HIP(hipGetLastError());
  return 0;
}

extern "C" int mopo_pool_gather(const mopo_pool_desc* p, int O, int A, const int64_t* idx, int64_t n,
                                float* dobs, float* dact, float* drew, float* dterm, float* dnobs, int64_t off,
                                void* stream) {
  if (check_pool(p)) return -1;
  if (n == 0) return 0;
  MOPO_REQUIRE(A <= O, "pool_gather: act_dim must not exceed obs_dim");
  const int64_t tot = n * O;
  hipLaunchKernelGGL(pool_gather_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     *p, O, A, idx, n, dobs, dact, drew, dterm, dnobs, off);
  MOPO_HIP(hipGetLastError());
  return 0;
}

extern "C" int mopo_pool_random_indices(const mopo_pool_desc* p, int64_t n, uint64_t seed, uint32_t step,
                                        int64_t* idx, void* stream) {
  MOPO_REQUIRE(p && p->d_state && idx, "pool_random_indices: NULL argument");
  if (n == 0) return 0;
  hipLaunchKernelGGL(pool_rand_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     p->d_state, n, seed, step, idx);
  MOPO_HIP(hipGetLastError());
  return 0;
}
