// Shared device/host helpers for libmopo_hip (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace mopo {

// ------------------------------------------------------------------ errors
void set_error(const std::string& msg);
int fail(const std::string& msg);  // sets error, returns -1

#define MOPO_HIP(call)                                                                  \
  do {                                                                                  \
    hipError_t _e = (call);                                                             \
    if (_e != hipSuccess)                                                               \
      return ::mopo::fail(std::string(#call) + ": " + hipGetErrorString(_e));           \
  } while (0)

#define MOPO_REQUIRE(cond, msg)                                                         \
  do {                                                                                  \
    if (!(cond)) return ::mopo::fail(msg);                                              \
  } while (0)

// ------------------------------------------------------------------ MFMA (f32 in / f32 acc)
// v_mfma_f32_16x16x4_f32: lane l holds A[l&15][l>>4], B[l>>4][l&15];
// D: col = l&15, row = (l>>4)*4 + r.  We always compute the TRANSPOSED product
//   D[n][m] = sum_k W^T[n][k] * X^T[k][m]
// so that D (features on the register axis, rows m on the lane axis) is directly the
// B operand of the next layer (k-group of 16 = 4 steps t; lane group g feeds k = 4g+t).
__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

// Workgroup barrier that orders LDS only: __syncthreads() is a workgroup-scope fence on every address
// space, which makes each wave wait (s_waitcnt vmcnt(0)) for its own outstanding global loads and
// STORES before the s_barrier -- a write-back's full latency on the critical path wherever a barrier
// follows global stores.  Use this one where the barrier publishes LDS data only.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }

// ------------------------------------------------------------------ activations (TF1 f32 semantics)
__device__ __forceinline__ float swishf(float x) { return x * (1.0f / (1.0f + expf(-x))); }

// tf.nn.softplus (Eigen select form, thresholds as softplusf) on v_exp_f32 / v_log_f32
__device__ __forceinline__ float softplus_fast(float x) {
  const float thr = -13.942385f;
  const float ex = __builtin_amdgcn_exp2f(x * 1.4426950408889634f);
  if (x > -thr) return x;
  if (x < thr) return ex;
  return __builtin_amdgcn_logf(ex + 1.0f) * 0.6931471805599453f;
}

// swish on the hardware transcendentals: x * rcp(1 + 2^(-x log2 e)) -- v_exp_f32 / v_rcp_f32 (1 ulp
// each) instead of the range-reduced expf and the IEEE divide (~25 VALU instructions per element in
// the ensemble forward's epilogues).  For x -> -inf the exp overflows to inf and rcp gives 0.
__device__ __forceinline__ float swish_fast(float x) {
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-x * 1.4426950408889634f));
}

// swish in the log2 domain: for u = -log2(e) x returns -log2(e) swish(x) = u / (1 + 2^u)
__device__ __forceinline__ float swish_log2(float u) {
  return u * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(u));
}

// tf.nn.softplus (Eigen): threshold = log(eps_f32) + 2
__device__ __forceinline__ float softplusf(float x) {
  const float thr = -13.942385f;  // logf(1.1920929e-7f) + 2
  if (x > -thr) return x;
  float ex = expf(x);
  if (x < thr) return ex;
  return logf(ex + 1.0f);
}

// ------------------------------------------------------------------ Philox4x32-10 (perf-mode RNG)
struct u32x4 { uint32_t x, y, z, w; };

__host__ __device__ __forceinline__ u32x4 philox(u32x4 c, uint32_t k0, uint32_t k1) {
  for (int i = 0; i < 10; ++i) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// two standard normals from two u32 (Box-Muller, float precision)
__device__ __forceinline__ void box_muller(uint32_t a, uint32_t b, float& z0, float& z1) {
  float u1 = ((float)a + 1.0f) * 2.3283064e-10f;  // (0, 1]
  float u2 = (float)b * 2.3283064e-10f;
  float r = sqrtf(-2.0f * logf(u1));
  float s, c;
  sincosf(6.2831853f * u2, &s, &c);
  z0 = r * c;
  z1 = r * s;
}

// stream ids for the Philox counter (counter = {row_uid, step, stream, block})
enum : uint32_t { RNG_START = 1, RNG_ACT = 2, RNG_OBS_NOISE = 3, RNG_MODEL = 4, RNG_SAC = 5, RNG_ACT_UNIFORM = 6 };

__host__ __device__ inline int ceil_div(int a, int b) { return (a + b - 1) / b; }

}  // namespace mopo
