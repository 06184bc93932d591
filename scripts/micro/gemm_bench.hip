// Micro-benchmark of the SAC grouped GEMM kernel (includes csrc/sac.hip to reach internals).
#include "../../mopo_amd/csrc/sac.hip"
#include <cstdio>

using namespace mopo;

__global__ void empty_kernel(const GemmGroup g) {
  if (threadIdx.x == 0 && g.n < 0) g.p[0].C[0] = 1.f;
}
__global__ void empty_small(float* p, int n) {
  if (threadIdx.x == 0 && n < 0) p[0] = 1.f;
}
// one dependent load + store per thread, big kernarg (the GemmGroup) read at a dynamic index
__global__ void ldst_kernel(const GemmGroup g) {
  int pi = 0;
  while (pi + 1 < g.n && (int)blockIdx.x >= g.prefix[pi + 1]) ++pi;
  const GemmProb& p = g.p[pi];
  p.C[blockIdx.x * 256 + threadIdx.x] = p.A[blockIdx.x * 256 + threadIdx.x] + 1.f;
}
__global__ void ldst_small(const float* a, float* c) {
  c[blockIdx.x * 256 + threadIdx.x] = a[blockIdx.x * 256 + threadIdx.x] + 1.f;
}

static float time_graph(std::vector<GemmProb> ps, int reps, hipStream_t s, int empty) {
  hipGraph_t gr; hipGraphExec_t ge;
  (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  for (int i = 0; i < 16; ++i) {
    if (!empty) launch_group(ps, s);
    else {
      GemmGroup g{}; g.n = 1; g.p[0] = ps[0]; g.prefix[1] = 1 << 20;
      if (empty == 1) hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(256), 0, s, g);
      if (empty == 2) hipLaunchKernelGGL(empty_small, dim3(256), dim3(256), 0, s, ps[0].C, 1);
      if (empty == 3) hipLaunchKernelGGL(ldst_kernel, dim3(256), dim3(256), 0, s, g);
      if (empty == 4) hipLaunchKernelGGL(ldst_small, dim3(256), dim3(256), 0, s, ps[0].A, ps[0].C);
    }
  }
  (void)hipStreamEndCapture(s, &gr);
  (void)hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0);
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  for (int w = 0; w < 3; ++w) (void)hipGraphLaunch(ge, s);
  (void)hipEventRecord(a, s);
  for (int r = 0; r < reps; ++r) (void)hipGraphLaunch(ge, s);
  (void)hipEventRecord(b, s);
  (void)hipEventSynchronize(b);
  float ms; (void)hipEventElapsedTime(&ms, a, b);
  return ms * 1e3f / reps / 16;
}

int main() {
  hipStream_t s; (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  const int n = 256, H = 256;
  float *X, *W, *Y, *M;
  (void)hipMalloc(&X, 8 * n * H * 4); (void)hipMalloc(&W, 8 * H * H * 4); (void)hipMalloc(&Y, 8 * n * H * 4);
  (void)hipMalloc(&M, n * H * 4);
  (void)hipMemset(X, 0, 8 * n * H * 4); (void)hipMemset(W, 0, 8 * H * H * 4); (void)hipMemset(M, 0, n * H * 4);
  auto fwd = [&](int i) { auto p = mk(n, H, H, X + i * n * H, H, 0, W + i * H * H, H, 0, Y + i * n * H, H); p.act = ACT_RELU; p.bias = W; return p; };
  auto bwd = [&](int i) { auto p = mk(n, H, H, X + i * n * H, H, 0, W + i * H * H, H, 1, Y + i * n * H, H); p.mask = M; p.ldm = H; return p; };
  auto wgt = [&](int i) { auto p = mk(H, H, n, X + i * n * H, H, 1, Y + i * n * H, H, 0, W + i * H * H, H); p.colsum = M; return p; };
  printf("empty kernel (GemmGroup kernarg): %.2f us\n", time_graph({fwd(0)}, 200, s, 1));
  printf("empty kernel (16 B kernarg):      %.2f us\n", time_graph({fwd(0)}, 200, s, 2));
  printf("load+store (GemmGroup kernarg):   %.2f us\n", time_graph({fwd(0)}, 200, s, 3));
  printf("load+store (16 B kernarg):        %.2f us\n", time_graph({fwd(0)}, 200, s, 4));
  auto w16 = [&](int i) { auto p = mk(16, 16, n, X + i * n * H, H, 1, Y + i * n * H, H, 0, W + i * H * H, H); return p; };
  printf("1 tile wgrad 16x16 K=256 (T):  %.2f us\n", time_graph({w16(0)}, 200, s, 0));
  printf("1 tile 16x16x16:              %.2f us\n", time_graph({mk(16, 16, 16, X, 16, 0, W, 16, 0, Y, 16)}, 200, s, 0));
  printf("1 tile 16x16x256:             %.2f us\n", time_graph({mk(16, 16, 256, X, 256, 0, W, 16, 0, Y, 16)}, 200, s, 0));
  printf("fwd 1 x 256x256x256:          %.2f us\n", time_graph({fwd(0)}, 200, s, 0));
  printf("fwd 4 x 256x256x256:          %.2f us\n", time_graph({fwd(0), fwd(1), fwd(2), fwd(3)}, 200, s, 0));
  printf("bwd-data 4 x (W^T, mask):     %.2f us\n", time_graph({bwd(0), bwd(1), bwd(2), bwd(3)}, 200, s, 0));
  printf("wgrad 2 x (X^T dY, colsum):   %.2f us\n", time_graph({wgt(0), wgt(1)}, 200, s, 0));
  {
    // the SAC forward launch: both hidden layers of 4 MLPs (layer 1 recomputed per tile, ta == 2)
    float *Xin, *W1, *B1, *H1;
    (void)hipMalloc(&Xin, n * 23 * 4); (void)hipMalloc(&W1, 4 * 23 * H * 4); (void)hipMalloc(&B1, 4 * H * 4);
    (void)hipMalloc(&H1, 4 * n * H * 4);
    (void)hipMemset(Xin, 0, n * 23 * 4); (void)hipMemset(W1, 0, 4 * 23 * H * 4); (void)hipMemset(B1, 0, 4 * H * 4);
    auto m12 = [&](int i, bool st) {
      auto a = mk(n, H, H, Xin, 23, 2, W + i * H * H, H, 0, Y + i * n * H, H);
      a.bias = W; a.act = ACT_RELU; a.a_u = W1 + i * 23 * H; a.a_v = B1 + i * H; a.a_ldm = 23; a.a_m = st ? H1 + i * n * H : nullptr;
      return a;
    };
    printf("mlp12 4 x (23->256->256), h1 stored x3: %.2f us\n", time_graph({m12(0, true), m12(1, false), m12(2, true), m12(3, true)}, 200, s, 0));
    printf("mlp12 4 x, no h1 store:        %.2f us\n", time_graph({m12(0, false), m12(1, false), m12(2, false), m12(3, false)}, 200, s, 0));
    printf("mlp12 1 x:                     %.2f us\n", time_graph({m12(0, false)}, 200, s, 0));
  }
  printf("fwd K=23 4 x 256x256:         %.2f us\n", time_graph({mk(n, H, 23, X, 23, 0, W, H, 0, Y, H), mk(n, H, 23, X, 23, 0, W, H, 0, Y + n * H, H), mk(n, H, 23, X, 23, 0, W, H, 0, Y + 2 * n * H, H), mk(n, H, 23, X, 23, 0, W, H, 0, Y + 3 * n * H, H)}, 200, s, 0));
  return 0;
}
