// Which XCD does each workgroup of consecutive launches run on?  Records HW_REG_XCC_ID per block for a
// sequence of launches (eager, then the same sequence replayed from a hipGraph) and prints, per launch,
// whether blocks b and b + 8 always share an XCD and which XCD block 0 got -- to test whether grids that are
// multiples of 8 keep b % 8 -> XCD fixed across launches (a speed-only placement question).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <algorithm>
#include <vector>

__global__ void rec(int* out) {
  if (threadIdx.x == 0) {
    int x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    out[blockIdx.x] = x;
  }
}

// L2 persistence across a kernel boundary: block b of `wr` writes region b (64 KB); block b of `rd` then
// reads region (b + shift) % grid and records its load time (s_memrealtime ticks, 100 MHz).  shift 0 (same
// block index: same XCD if placement is stable) against shift 1 (another XCD).
__global__ void wr(float* buf, int n) {
  float* r = buf + (size_t)blockIdx.x * n;
  for (int i = threadIdx.x; i < n; i += blockDim.x) r[i] = (float)i;
}
__global__ void rd(const float* buf, int n, int shift, long* t, float* sink) {
  const int b = (blockIdx.x + shift) % gridDim.x;
  const float* r = buf + (size_t)b * n;
  __syncthreads();
  const long t0 = __builtin_amdgcn_s_memrealtime();
  float acc = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) acc += r[i];
  __syncthreads();
  const long t1 = __builtin_amdgcn_s_memrealtime();
  if (acc == -1.f) sink[0] = acc;
  if (threadIdx.x == 0) t[blockIdx.x] = t1 - t0;
}

#define CK(e) do { hipError_t r = (e); if (r != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(r), __LINE__); return 1; } } while (0)

int main() {
  const std::vector<int> grids = {256, 256, 257, 100, 8, 13, 512, 249, 64, 64, 1025, 40, 16, 3, 256};
  int tot = 0;
  for (int g : grids) tot += g;
  int* d;
  CK(hipMalloc(&d, tot * 4 * 2));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  auto run = [&](int* base) {
    int off = 0;
    for (int g : grids) { hipLaunchKernelGGL(rec, dim3(g), dim3(64), 0, s, base + off); off += g; }
  };
  for (int rep = 0; rep < 3; ++rep) run(d);          // eager
  CK(hipStreamSynchronize(s));
  hipGraph_t gr; hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  run(d + tot);
  CK(hipStreamEndCapture(s, &gr));
  CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
  for (int rep = 0; rep < 3; ++rep) CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  std::vector<int> h(2 * tot);
  CK(hipMemcpy(h.data(), d, 2 * tot * 4, hipMemcpyDeviceToHost));
  for (int m = 0; m < 2; ++m) {
    printf("%s\n", m ? "graph replay (last of 3)" : "eager (last of 3)");
    int off = m * tot, prev0 = -1, prevg = 0;
    for (int g : grids) {
      bool cons = true;
      for (int b = 8; b < g; ++b) cons &= h[off + b] == h[off + b - 8];
      int distinct = 0, seen[16] = {};
      for (int b = 0; b < g; ++b) if (!seen[h[off + b] & 15]++) ++distinct;
      printf("  grid %5d: block0 xcc %d  b%%8 consistent %d  xccs used %d  (prev block0 + prev grid) %% 8 = %d  first 10:",
             g, h[off], (int)cons, distinct, prev0 < 0 ? -1 : (prev0 + prevg) % 8);
      for (int b = 0; b < 10 && b < g; ++b) printf(" %d", h[off + b]);
      printf("\n");
      prev0 = h[off]; prevg = g; off += g;
    }
  }
  {  // L2 persistence
    const int G = 256, n = 16384;
    float* buf; long* t; float* sink;
    CK(hipMalloc(&buf, (size_t)G * n * 4)); CK(hipMalloc(&t, G * 8)); CK(hipMalloc(&sink, 4));
    std::vector<long> ht(G);
    for (int rep = 0; rep < 4; ++rep)
      for (int shift : {0, 1, 8}) {
        hipLaunchKernelGGL(wr, dim3(G), dim3(256), 0, s, buf, n);
        hipLaunchKernelGGL(rd, dim3(G), dim3(256), 0, s, buf, n, shift, t, sink);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(ht.data(), t, G * 8, hipMemcpyDeviceToHost));
        std::vector<long> v = ht;
        std::sort(v.begin(), v.end());
        printf("rep %d shift %d: read 64 KB per block after the writer: p50 %.2f us  p90 %.2f us\n", rep, shift,
               v[G / 2] / 100.0, v[G * 9 / 10] / 100.0);
      }
  }
  return 0;
}
