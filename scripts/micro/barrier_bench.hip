// Micro-benchmark: grid-barrier cost (agent-scope release/acquire counter) vs per-kernel launch
// floor inside a hipGraph -- decides the SAC step structure (persistent kernel vs launch chain).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ void grid_barrier(unsigned* ctr, unsigned target) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target && ++spins < (1u << 26))
      __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

__global__ void persistent(unsigned* ctr, int nbar, float* buf) {
  const unsigned G = gridDim.x;
  float acc = 0.f;
  for (int b = 0; b < nbar; ++b) {
    acc += buf[(blockIdx.x * 256 + threadIdx.x + b * 997) % (1 << 20)];
    buf[(blockIdx.x * 256 + threadIdx.x) % (1 << 20)] = acc;
    grid_barrier(ctr, G * (b + 1));
  }
}

__global__ void tiny(float* buf) {
  buf[blockIdx.x * blockDim.x + threadIdx.x] += 1.f;
}

int main() {
  unsigned* ctr;
  float* buf;
  hipMalloc(&ctr, 4);
  hipMalloc(&buf, (1 << 20) * 4);
  hipMemset(buf, 0, (1 << 20) * 4);
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int NB = 16, REP = 200;
  for (int G : {64, 128, 256}) {
    for (int w = 0; w < 2; ++w) {
      hipEventRecord(a, s);
      for (int r = 0; r < REP; ++r) {
        hipMemsetAsync(ctr, 0, 4, s);
        hipLaunchKernelGGL(persistent, dim3(G), dim3(256), 0, s, ctr, NB, buf);
      }
      hipEventRecord(b, s);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (w) printf("persistent G=%d: %.2f us per launch of %d barriers (%.2f us/barrier incl launch)\n", G,
                    ms * 1e3 / REP, NB, ms * 1e3 / REP / NB);
    }
  }
  // graph of 16 tiny kernels
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  for (int i = 0; i < NB; ++i) hipLaunchKernelGGL(tiny, dim3(256), dim3(256), 0, s, buf);
  hipStreamEndCapture(s, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  for (int w = 0; w < 2; ++w) {
    hipEventRecord(a, s);
    for (int r = 0; r < REP; ++r) hipGraphLaunch(ge, s);
    hipEventRecord(b, s);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (w) printf("graph of %d tiny kernels: %.2f us per graph (%.2f us/kernel)\n", NB, ms * 1e3 / REP, ms * 1e3 / REP / NB);
  }
  // plain stream launches
  for (int w = 0; w < 2; ++w) {
    hipEventRecord(a, s);
    for (int r = 0; r < REP; ++r)
      for (int i = 0; i < NB; ++i) hipLaunchKernelGGL(tiny, dim3(256), dim3(256), 0, s, buf);
    hipEventRecord(b, s);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (w) printf("stream launches: %.2f us/kernel\n", ms * 1e3 / REP / NB);
  }
  unsigned c;
  hipMemcpy(&c, ctr, 4, hipMemcpyDeviceToHost);
  printf("final counter %u\n", c);
  return 0;
}
