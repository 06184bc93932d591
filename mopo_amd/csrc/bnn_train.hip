// Probabilistic-ensemble training step (BNN.train) on CDNA4.
//
// Replaces the TF training graph of BNN.finalize (mopo/models/bnn.py:226-249: Gaussian NLL of
// _compile_losses :677-701 + weight decay fc.py:156-157 + 0.01 (sum maxlv - sum minlv), one
// tf.train.AdamOptimizer(1e-3) over all optvars, constructor.py:41) and the per-minibatch
// session.run of BNN.train (bnn.py:425-432); _compile_losses(inc_var_loss=False) for the holdout
// losses (bnn.py:463-475, 486-493); shuffle_rows (:385-387); _save_state / _set_state (:264-285).
// The loop control (holdout split, bootstrap indices, early stopping, elites) stays on the host
// (mopo_amd/bnn.py), drawing from numpy's global stream in the reference's order.
//
// One minibatch step = 2 launches (step_rows, train_rows.h): the row blocks (gather + scaler, 4 swish
// layers + heads, output gradient, loss partials, then the activation-gradient chain with the
// pre-activations held in LDS), and one launch whose block 0 runs the batch-level tail (max/min log-var
// gradients and their Adam) beside the weight-gradient tiles, which apply weight decay and the TF1
// Adam in their epilogue (gemm_group.h; parameters ping-pong between two buffers).  MOPO_TRAIN_FUSED=0
// keeps the 3-launch form (separate forward / backward row launches, the tail in the backward's).  The previous 12-launch form
// (gather, 5 forward GEMM launches, loss kernel, 5 backward GEMM launches: step_impl) remains for
// H > 256 and for the holdout evaluation's forward.  Full-batch steps are captured into hipGraphs
// (8 / 2 / 1+copy-back steps); the epoch's partial last batch runs eagerly.
//
// Parameter layout (training master copy, f32): per member, the reference's optvars with the two
// smv heads concatenated column-wise so one GEMM serves both:
//   W0 [E][IN][H] b0 [E][H]  W1..W3 [E][H][H] b1..b3 [E][H]  Whd [E][H][2D] bhd [E][2D]
//   maxlv [D] minlv [D]        (Whd[e][k][n]: n < D mean head, n >= D log-var head)
#include <algorithm>
#include <cstring>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "train_rows.h"

namespace mopo {

namespace {

constexpr int NHID = 4;
const float WDECAY[NHID + 1] = {0.000025f, 0.00005f, 0.000075f, 0.000075f, 0.0001f};  // constructor.py:30-36

struct Layout {
  int E, IN, H, D;
  int64_t W[NHID + 1], b[NHID + 1];  // offsets (layer NHID = concatenated heads)
  int64_t mx, mn, total;
};

Layout make_layout(int E, int IN, int H, int D) {
  Layout L{};
  L.E = E; L.IN = IN; L.H = H; L.D = D;
  int64_t c = 0;
  for (int l = 0; l <= NHID; ++l) {
    const int in = l == 0 ? IN : H, out = l == NHID ? 2 * D : H;
    L.W[l] = c; c += (int64_t)E * in * out;
    L.b[l] = c; c += (int64_t)E * out;
  }
  L.mx = c; c += D;
  L.mn = c; c += D;
  L.total = c;
  return L;
}

struct Train {
  Layout L{};
  int maxM = 0, max_batch = 0, max_eval = 0;
  float lr = 1e-3f;
  void* mem = nullptr;
  float *Pb[2] = {nullptr, nullptr}, *G = nullptr, *M = nullptr, *V = nullptr, *S = nullptr;  // S: snapshots
  float* beta_pow = nullptr;   // [3]: beta1^t, beta2^t, this step's lr_t
  int* bstep = nullptr;        // minibatch index within the epoch (device)
  unsigned* ticket = nullptr;
  float* part = nullptr;       // loss-kernel block partials
  float* lpart = nullptr;      // row-block path: per (member, row block) loss partials (train_rows.h)
  float* logs = nullptr;       // [4]: last train loss (data term), ...
  float *mu = nullptr, *sigma = nullptr;
  float *X = nullptr, *T = nullptr, *Z[NHID] = {}, *Hh[NHID] = {}, *OUT = nullptr, *dOUT = nullptr, *dZ[NHID] = {};
  float *X2 = nullptr, *T2 = nullptr;   // the staged gather's second row buffers (odd steps of a graph)
  std::vector<int> snap;       // members with a snapshot
  int32_t* wlist = nullptr;    // weight-gradient tiles per XCD (train_wgrad2_kernel): [8][wl_per_x], counts [8]
  int32_t* wcnt = nullptr;
  int wl_per_x = 0;
  // graphs (full-batch steps), keyed by the epoch's data pointers
  hipStream_t gs = nullptr;
  hipEvent_t ev_in = nullptr, ev_out = nullptr;
  hipEvent_t ev_order = nullptr, ev_applied = nullptr;   // shuffle: order ready / order consumed
  hipGraphExec_t gexec[3] = {nullptr, nullptr, nullptr};
  hipGraph_t graph[3] = {nullptr, nullptr, nullptr};
  const void* gkey[4] = {nullptr, nullptr, nullptr, nullptr};
  int64_t gkey_n = -1; int gkey_b = -1;
  // shuffle workspace
  void* sort_tmp = nullptr; size_t sort_tmp_bytes = 0;
  double* sort_keys = nullptr; int32_t* sort_vals_in = nullptr; int32_t* sort_vals = nullptr;
  int64_t sort_cap = 0;
};

constexpr int LOSS_TPB = 256;

// ---- minibatch gather: X[e][r] = scaler(inputs[row]), T[e][r] = targets[row] ----------------
// row = rows[e * stride + base + r] with base = (*bstep) * batch (training) or 0 (evaluation);
// rows == NULL: row = r for every member.
__global__ void train_gather_kernel(const float* __restrict__ inputs, const float* __restrict__ targets,
                                    const int32_t* __restrict__ rows, int64_t stride, const int* __restrict__ bstep,
                                    int batch, int M, int E, int IN, int D, const float* __restrict__ mu,
                                    const float* __restrict__ sigma, float* __restrict__ X, float* __restrict__ T) {
  const int W = IN + D;
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= (int64_t)E * M * W) return;
  const int c = i % W;
  const int64_t er = i / W;
  const int r = er % M, e = er / M;
  const int64_t base = bstep ? (int64_t)(*bstep) * batch : 0;
  const int64_t row = rows ? rows[e * stride + base + r] : r;
  if (c < IN) X[er * IN + c] = (inputs[row * IN + c] - mu[c]) / sigma[c];   // utils.py:96
  else T[er * D + (c - IN)] = targets[row * D + (c - IN)];
}

// ---- training loss gradient (bnn.py:241-249, 677-701): block = (dim d, 256 (member, row) pairs)
// mean = OUT[..., d], raw log-var = OUT[..., D + d];  lv1 = mx - softplus(mx - raw),
// lv = mn + softplus(lv1 - mn) (bnn.py:669-670).  d/dmean = 2 (mean - y) e^-lv / (M D),
// d/dlv = (1 - (mean - y)^2 e^-lv) / (M D); softplus' = sigmoid.
// The last block to finish reduces the per-dim partials (in block order), adds the 0.01 terms,
// applies Adam to max/min log-var, fixes this step's lr_t and advances beta powers and bstep.
struct LossArgs {
  int E, M, D;
  const float* OUT; const float* T; float* dOUT;
  float* part; unsigned* ticket; float* logs; float* beta_pow; int* bstep; float lr;
  int64_t off_mx, off_mn;
  float* G;                          // gradient buffer (max/min log-var slots written here)
  AdamCtx ad;
};

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

__global__ __launch_bounds__(LOSS_TPB) void train_loss_kernel(const LossArgs a) {
  __shared__ float sh[64];
  __shared__ int last;
  const int D = a.D, n = a.E * a.M;
  const int per_d = ceil_div(n, LOSS_TPB);
  const int d = blockIdx.x / per_d, chunk = blockIdx.x % per_d;
  const int i = chunk * LOSS_TPB + threadIdx.x;  // (member, row) pair
  const float mx = a.ad.Pc[a.off_mx + d], mn = a.ad.Pc[a.off_mn + d];
  float c_mx = 0.f, c_mn = 0.f, c_loss = 0.f;
  if (i < n) {
    const float* o = a.OUT + (int64_t)i * 2 * D;
    const float mean = o[d], raw = o[D + d], y = a.T[(int64_t)i * D + d];
    const float s = 1.f / ((float)a.M * (float)D);
    const float lv1 = mx - softplusf(mx - raw);
    const float lv = mn + softplusf(lv1 - mn);
    const float inv = expf(-lv);
    const float err = mean - y;
    const float dlv = (1.f - err * err * inv) * s;
    const float sb = sigm(lv1 - mn), sa = sigm(mx - raw);
    const float dlv1 = dlv * sb;
    float* g = a.dOUT + (int64_t)i * 2 * D;
    g[d] = 2.f * err * inv * s;
    g[D + d] = dlv1 * sa;
    c_mn = dlv * (1.f - sb);
    c_mx = dlv1 * (1.f - sa);
    c_loss = (err * err * inv + lv) * s;
  }
  float v[3] = {c_mx, c_mn, c_loss};
  {  // block sums (butterfly per wave, waves in order)
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) v[k] += __shfl_xor(v[k], off);
    if (lane == 0)
#pragma unroll
      for (int k = 0; k < 3; ++k) sh[w * 3 + k] = v[k];
    __syncthreads();
    if (threadIdx.x == 0) {
      float t[3] = {0.f, 0.f, 0.f};
      for (int q = 0; q < LOSS_TPB / 64; ++q)
#pragma unroll
        for (int k = 0; k < 3; ++k) t[k] += sh[q * 3 + k];
      float* pp = a.part + 4 * (int64_t)blockIdx.x;
      pp[0] = t[0]; pp[1] = t[1]; pp[2] = t[2];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      const unsigned tk = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = (tk == gridDim.x - 1);
      if (last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
  }
  __syncthreads();
  if (!last) return;
  // this step's TF1 Adam step size from the pre-update beta powers (every thread reads them
  // before thread 0 advances them below)
  const float b1p = a.beta_pow[0], b2p = a.beta_pow[1];
  const float lr_t = a.lr * sqrtf(1.f - b2p) / (1.f - b1p);
  __syncthreads();
  if ((int)threadIdx.x < D) {
    const int dd = threadIdx.x;
    float gmx = 0.f, gmn = 0.f, loss = 0.f;
    for (int c = 0; c < per_d; ++c) {
      const float* pp = a.part + 4 * (int64_t)(dd * per_d + c);
      gmx += pp[0]; gmn += pp[1]; loss += pp[2];
    }
    gmx += 0.01f;                                                   // 0.01 * sum(max_logvar)
    gmn -= 0.01f;                                                   // -0.01 * sum(min_logvar)
    a.G[a.off_mx + dd] = gmx;
    a.G[a.off_mn + dd] = gmn;
    adam_apply(a.ad, a.off_mx + dd, gmx, adam_load(a.ad, a.off_mx + dd), lr_t);
    adam_apply(a.ad, a.off_mn + dd, gmn, adam_load(a.ad, a.off_mn + dd), lr_t);
    sh[dd] = loss;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float loss = 0.f;
    for (int dd = 0; dd < D; ++dd) loss += sh[dd];
    a.logs[0] = loss;                                               // data term of the train loss
    a.beta_pow[2] = lr_t;
    a.beta_pow[0] = b1p * 0.9f;
    a.beta_pow[1] = b2p * 0.999f;
    if (a.bstep) *a.bstep += 1;
    *a.ticket = 0u;
  }
}

// ---- mse loss per member (inc_var_loss=False): mean over rows and dims of (mean - y)^2 --------
constexpr int MSE_TPB = 1024;
__global__ __launch_bounds__(MSE_TPB) void train_mse_kernel(const float* __restrict__ OUT, const float* __restrict__ T,
                                                            int M, int D, float* __restrict__ losses) {
  __shared__ float sh[MSE_TPB / 64];
  const int e = blockIdx.x;
  float acc = 0.f;
  for (int i = threadIdx.x; i < M * D; i += blockDim.x) {
    const int r = i / D, d = i % D;
    const float err = OUT[((int64_t)e * M + r) * 2 * D + d] - T[((int64_t)e * M + r) * D + d];
    acc += err * err;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < MSE_TPB / 64; ++w) t += sh[w];
    losses[e] = t / ((float)M * (float)D);
  }
}

// ---- scaler fit (utils.py:69-86): mean / std over rows, f64 accumulation, std < 1e-12 -> 1 ----
__global__ __launch_bounds__(256) void scaler_fit_kernel(const float* __restrict__ x, int64_t n, int IN,
                                                         float* __restrict__ mu, float* __restrict__ sigma) {
  __shared__ double sh[4];
  const int c = blockIdx.x;
  double s = 0.0;
  for (int64_t r = threadIdx.x; r < n; r += blockDim.x) s += x[r * IN + c];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  const double mean = (sh[0] + sh[1] + sh[2] + sh[3]) / (double)n;
  __syncthreads();
  double q = 0.0;
  for (int64_t r = threadIdx.x; r < n; r += blockDim.x) {
    const double dv = x[r * IN + c] - mean;
    q += dv * dv;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) q += __shfl_xor(q, off);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = q;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double sd = sqrt((sh[0] + sh[1] + sh[2] + sh[3]) / (double)n);
    mu[c] = (float)mean;
    sigma[c] = sd < 1e-12 ? 1.f : (float)sd;
  }
}

// ---- format_samples_for_training (constructor.py:46-57) over pool rows ---------------------
__global__ void format_kernel(const mopo_pool_desc p, int O, int A, const int64_t* __restrict__ rows, int64_t n,
                              float* __restrict__ inputs, float* __restrict__ targets) {
  const int IN = O + A, D = O + 1, W = IN + D;
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n * W) return;
  const int64_t r = i / W;
  const int c = i % W;
  const int64_t src = rows ? rows[r] : r;
  if (c < O) inputs[r * IN + c] = p.d_obs[src * O + c];
  else if (c < IN) inputs[r * IN + c] = p.d_act[src * A + (c - O)];
  else if (c == IN) targets[r * D] = p.d_rew[src];
  else targets[r * D + (c - IN)] = p.d_next_obs[src * O + (c - IN - 1)] - p.d_obs[src * O + (c - IN - 1)];
}

// ---- per-member variable copy (snapshots): dir 0: P -> S, 1: S -> P for member e ------------
constexpr int MAX_MEMBERS_SET = 64;
struct MemberSpan { int64_t off[2 * (NHID + 1)]; int64_t len[2 * (NHID + 1)]; };

__global__ void member_copy_kernel(float* __restrict__ P, float* __restrict__ S, const MemberSpan sp, int e,
                                   int dir) {
  const int k = blockIdx.y;
  const int64_t len = sp.len[k], off = sp.off[k] + (int64_t)e * len;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < len; i += (int64_t)gridDim.x * blockDim.x) {
    if (dir == 0) S[off + i] = P[off + i];
    else P[off + i] = S[off + i];
  }
}

// the same copy for a set of members in one launch (blockIdx.z = position in the set)
struct MemberSet { int n; int e[MAX_MEMBERS_SET]; };

__global__ void members_copy_kernel(float* __restrict__ P, float* __restrict__ S, const MemberSpan sp,
                                    const MemberSet ms, int dir) {
  const int k = blockIdx.y, e = ms.e[blockIdx.z];
  const int64_t len = sp.len[k], off = sp.off[k] + (int64_t)e * len;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < len; i += (int64_t)gridDim.x * blockDim.x) {
    if (dir == 0) S[off + i] = P[off + i];
    else P[off + i] = S[off + i];
  }
}

MemberSpan member_span(const Layout& L) {
  MemberSpan s{};
  for (int l = 0; l <= NHID; ++l) {
    const int in = l == 0 ? L.IN : L.H, out = l == NHID ? 2 * L.D : L.H;
    s.off[2 * l] = L.W[l]; s.len[2 * l] = (int64_t)in * out;
    s.off[2 * l + 1] = L.b[l]; s.len[2 * l + 1] = out;
  }
  return s;
}

// ---- shuffle_rows: idx[e] <- idx[e][order[e]] ---------------------------------------------
__global__ void apply_order_kernel(const int32_t* __restrict__ order, const int32_t* __restrict__ src, int64_t n,
                                   int E, int32_t* __restrict__ dst) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n * E) return;
  const int64_t e = i / n;
  dst[i] = src[e * n + order[i]];
}

// sort key of member e's k-th uniform: (e << 53) | u * 2^53.  numpy's random_sample is k / 2^53 with
// an integer k < 2^53 (two MT19937 draws, 27 + 26 bits), so the integer is exact and orders as the
// double does; value = the position within the member row.
__global__ void sort_keys_kernel(const double* __restrict__ u, int64_t n, int E, uint64_t* __restrict__ keys,
                                 int32_t* __restrict__ vals) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n * E) return;
  const uint64_t e = (uint64_t)(i / n);
  keys[i] = (e << 53) | (uint64_t)(u[i] * 9007199254740992.0);
  vals[i] = (int32_t)(i % n);
}

// ---------------------------------------------------------------------------------------------
int launch_gather(Train* h, const float* in, const float* tg, const int32_t* rows, int64_t stride, bool use_bstep,
                  int batch, int M, hipStream_t s) {
  const Layout& L = h->L;
  const int64_t tot = (int64_t)L.E * M * (L.IN + L.D);
  hipLaunchKernelGGL(train_gather_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, in, tg, rows, stride,
                     use_bstep ? h->bstep : nullptr, batch, M, L.E, L.IN, L.D, h->mu, h->sigma, h->X, h->T);
  MOPO_HIP(hipGetLastError());
  return 0;
}

// forward of the 4 swish layers + heads on X (M rows per member) with parameters P
int forward(Train* h, const float* P, int M, hipStream_t s, int tile = 0) {
  const Layout& L = h->L;
  const int E = L.E, H = L.H, IN = L.IN, D2 = 2 * L.D;
  for (int l = 0; l <= NHID; ++l) {
    const int K = l == 0 ? IN : H, N = l == NHID ? D2 : H;
    const float* A = l == 0 ? h->X : h->Hh[l - 1];
    std::vector<GemmProb> g;
    for (int e = 0; e < E; ++e) {
      auto p = mk(M, N, K, A + (int64_t)e * M * K, K, 0, P + L.W[l] + (int64_t)e * K * N, N, 0,
                  (l == NHID ? h->OUT : h->Hh[l]) + (int64_t)e * M * N, N);
      p.bias = P + L.b[l] + (int64_t)e * N;
      if (l < NHID) { p.act = ACT_SWISH; p.Z = h->Z[l] + (int64_t)e * M * N; }
      g.push_back(p);
    }
    if (launch_group(g, s, nullptr, nullptr, nullptr, tile)) return -1;
  }
  return 0;
}

// the holdout evaluation's GEMM tiles (MOPO_EVAL_TILE, default 32: ~1000 rows per member)
int eval_tile() {
  static const int v = [] {
    const char* e = std::getenv("MOPO_EVAL_TILE");
    return e ? std::atoi(e) : 32;
  }();
  return v;
}

// one minibatch Adam step on the gathered X/T (M rows per member): P = Pb[par] -> Pb[1 - par]
int step_impl(Train* h, int par, int M, bool use_bstep, hipStream_t s) {
  const Layout& L = h->L;
  const int E = L.E, H = L.H, IN = L.IN, D = L.D, D2 = 2 * D;
  const float* P = h->Pb[par];
  if (forward(h, P, M, s)) return -1;
  AdamCtx ad{};
  ad.G = h->G; ad.Pc = h->Pb[par]; ad.Pn = h->Pb[1 - par]; ad.M = h->M; ad.V = h->V; ad.T = nullptr;
  ad.lr_t = h->beta_pow + 2; ad.tau = 0.f; ad.total = L.total; ad.n_pi = 0; ad.n_q = 0; ad.norm_part = nullptr;
  {
    LossArgs a{};
    a.E = E; a.M = M; a.D = D; a.OUT = h->OUT; a.T = h->T; a.dOUT = h->dOUT; a.part = h->part; a.ticket = h->ticket;
    a.logs = h->logs; a.beta_pow = h->beta_pow; a.bstep = use_bstep ? h->bstep : nullptr; a.lr = h->lr;
    a.off_mx = L.mx; a.off_mn = L.mn; a.G = h->G; a.ad = ad;
    const int blocks = D * ceil_div(E * M, LOSS_TPB);
    hipLaunchKernelGGL(train_loss_kernel, dim3(blocks), dim3(LOSS_TPB), 0, s, a);
    MOPO_HIP(hipGetLastError());
  }
  // backward: launch l (l = NHID .. 0) forms dW_l (+ decay, Adam) and, for l >= 1, dZ_{l-1}
  for (int l = NHID; l >= 0; --l) {
    const int K = l == 0 ? IN : H, N = l == NHID ? D2 : H;  // layer l: [K -> N]
    const float* dY = l == NHID ? h->dOUT : h->dZ[l];        // gradient at layer l's output (pre-activation)
    const float* Xin = l == 0 ? h->X : h->Hh[l - 1];
    std::vector<GemmProb> g;
    for (int e = 0; e < E; ++e) {
      const float* dYe = dY + (int64_t)e * M * N;
      // dW_l = X_in^T dY  (+ db = colsum dY), fused decay + Adam
      auto w = mk(K, N, M, Xin + (int64_t)e * M * K, K, 1, dYe, N, 0, h->G + L.W[l] + (int64_t)e * K * N, N);
      w.colsum = h->G + L.b[l] + (int64_t)e * N;
      w.adam = 1;
      w.wd = WDECAY[l];
      g.push_back(w);
      if (l >= 1) {  // dZ_{l-1} = (dY W_l^T) * swish'(Z_{l-1})
        auto dz = mk(M, K, N, dYe, N, 0, P + L.W[l] + (int64_t)e * K * N, N, 1, h->dZ[l - 1] + (int64_t)e * M * K, K);
        dz.mask = h->Z[l - 1] + (int64_t)e * M * K; dz.ldm = K; dz.mask_kind = MASK_DSWISH;
        g.push_back(dz);
      }
    }
    if (launch_group(g, s, &ad, nullptr)) return -1;
  }
  return 0;
}

// The same step as three launches (train_rows.h): forward + output gradient, the activation-gradient
// chain + the batch-level tail, and every weight gradient (+ decay, Adam) as one batched gemm launch.
// Instantiated for the D4RL widths (inputs 14 / 23, hidden 32 / 200 / 256, 2D 24 / 36); H and 2D
// multiples of 4 (b128 weight rows).  MOPO_TRAIN_ROWS=0 selects step_impl (twelve launches) instead.
// the weight-gradient launch's tile width (MOPO_TRAIN_WGRAD_TILE: 16 or 32; default 32: 4,000 16x16
// tiles of K = 256 re-read each operand panel 16x over, 32x32 tiles half as often)
constexpr int TRAIN_WG_P = NHID + 1;   // weight-gradient problems of the fused step (one per layer)
int train_wgrad_tile() {
  static const int v = [] {
    const char* e = std::getenv("MOPO_TRAIN_WGRAD_TILE");
    return e ? std::atoi(e) : 32;
  }();
  return v == 16 ? 0 : 32;
}

bool use_rows(const Train* h) {
  static const int env = [] {
    const char* e = std::getenv("MOPO_TRAIN_ROWS");
    return e ? std::atoi(e) : 1;
  }();
  const Layout& L = h->L;
  const int g0 = ceil_div(L.IN, 16), gh = ceil_div(L.H, 16), gd = ceil_div(2 * L.D, 16);
  const bool inst = (gh == 13 || gh == 16 || gh == 2) && ((g0 == 2 && gd == 3) || (g0 == 1 && gd == 2));  // step_rows
  return env != 0 && inst && L.H % 4 == 0 && L.D % 2 == 0;
}

// the batch-level tail's inputs (train_rows.h train_loss_tail) -- the weight-gradient launch's block 0
struct TrainTail {
  int E, nrb, D;
  const float* lpart;
  int64_t mx, mn;
  float* logs; float* beta_pow; int* bstep_inc; float lr; float* G; AdamCtx ad;
};
// the weight-gradient launch of the fused step: block 0 the tail, then the problems' 32x32 tiles (gemm32_body)
struct TrainWgrad {
  int n;
  int prefix[TRAIN_WG_P + 1];
  AdamCtx ad;
  GemmProb p[TRAIN_WG_P];
  TrainTail t;
};
static __global__ __launch_bounds__(256, 2) void train_wgrad_kernel(const TrainWgrad g) {
  if (blockIdx.x == 0) {   // dispatched first: its serial chain runs beside the tiles
    __shared__ float sh[TR_TAIL_SH];   // small enough to keep 4 workgroups of the tiles per CU
    train_loss_tail(g.t, sh);
    return;
  }
  gemm32_body(g, (int)blockIdx.x - 1);
}

// ---- the weight-gradient launch, persistent XCD-local form -------------------------------------------
// Every weight gradient dW_l = X_in^T dY (+ db = colsum dY, decay, TF1 Adam) of every member as 32 x 32
// output tiles over the minibatch rows k < M (sac_wgrad.h's tile: 1024 threads, wave w the 16 x 16 quadrant
// w & 3 over the K quarter w >> 2, K in chunks of 256 staged [row][k]).  The tiles are dealt to XCDs on the
// host (build_wlist): member e's tiles go to XCD e mod 8 -- the XCD whose CUs ran its row blocks
// (train_rows.h tr_block), so its X_in / dY panels, parameters and Adam slots are that L2's -- up to an even
// share, the overflow to the least-loaded XCDs.  Each XCD's workgroups walk its list (workgroup j: entries
// j, j + nwx, ...) and load the next tile's panels and Adam inputs into registers while the current tile's
// MFMAs and epilogue run, so a workgroup has two tiles in flight instead of one memory latency per tile.
// The last block runs the batch-level tail (train_loss_tail).
#ifndef TRAIN_WG2_KC
// K rows staged per chunk (LDS: 2 x 32 x (KC + 4) floats per workgroup).  128 (33 KB, 76 VGPRs) lets three
// 512-thread workgroups share a CU instead of two at 256 (66.5 KB, 95 VGPRs): same box, 13.61-13.69k vs
// 13.41-13.45k grad-steps/s (profiles/r05_train_ab_wg2_chunk.txt; four per CU at a 64-VGPR cap spill: 13.4k)
#define TRAIN_WG2_KC 128
#endif
#ifndef TRAIN_WG2_MINW
#define TRAIN_WG2_MINW 0   // > 0: waves per SIMD the tile kernel's registers are capped for (0: NT / 128)
#endif
// LDS panels [row][k] of the weight-gradient tiles: k XOR-swizzled by row group ((row >> 2) & 7, in units of
// 4 floats: a b128 read of 4 consecutive k stays contiguous) at a 140-float row stride, so the transposing
// b32 stores (8 rows x 8 k per 32-lane group) hit 32 distinct banks instead of 8 and the b128 MFMA reads
// conflict less (modelled with MI355X_MICROARCH's LDS lane groups: 128 + 320 vs 512 + 256 LDS cycles per chunk)
#ifndef TW2_SWZ
#define TW2_SWZ 1
#endif
constexpr int TW2_T = 32, TW2_KC = TRAIN_WG2_KC, TW2_KP = TW2_KC + (TW2_SWZ ? 12 : 4);
static __device__ __forceinline__ int tw2_at(int row, int k) {
  return row * TW2_KP + (TW2_SWZ ? (k ^ (((row >> 2) & 7) << 2)) : k);
}
struct TrainWg2 {
  int M;                               // minibatch rows per member (the contraction length)
  int nwx, per_x;                      // tile workgroups per XCD; list stride per XCD
  const int32_t* list;                 // [8][per_x]: l | e << 3 | tm << 7 | tn << 12
  const int32_t* cnt;                  // [8] entries per XCD
  const float* A[NHID + 1];            // X_in of layer l, member 0 ([E][M][K_l])
  const float* B[NHID + 1];            // dY of layer l, member 0 ([E][M][N_l])
  int K[NHID + 1], N[NHID + 1];
  int64_t W[NHID + 1], b[NHID + 1];
  float wd[NHID + 1];
  AdamCtx ad;
  TrainTail t;
};

struct Wg2Tile {
  const float* A; const float* B;
  int K, N, i0, j0;
  int64_t w0, b0;                      // parameter index of W(0, 0) / b(0) of the tile's member and layer
  float wd;
  bool cs;                             // tile-row 0: also the bias column sums
  int e, l;                            // member, layer
};

static __device__ __forceinline__ Wg2Tile wg2_tile(const TrainWg2& g, int v) {
  Wg2Tile t;
  const int l = v & 7, e = (v >> 3) & 15, tm = (v >> 7) & 31, tn = (v >> 12) & 31;
  t.K = g.K[l]; t.N = g.N[l];
  t.A = g.A[l] + (int64_t)e * g.M * t.K;
  t.B = g.B[l] + (int64_t)e * g.M * t.N;
  t.i0 = TW2_T * tm; t.j0 = TW2_T * tn;
  t.w0 = g.W[l] + (int64_t)e * t.K * t.N;
  t.b0 = g.b[l] + (int64_t)e * t.N;
  t.wd = g.wd[l];
  t.cs = tm == 0;
  t.e = e; t.l = l;
  return t;
}

// Workgroups of NT threads (512 or 1024): wave w owns quadrant w & 3 of the tile over the K part w >> 2 of
// KW = 256 / (NT / 256) rows.  Thread t stages elements (row 4 (t % 8) + u, k (t / 8) + NT / 8 q), u < 4,
// q < NQ: one b128 load per (operand, q) where the operand's row length is a multiple of 4 floats (b32
// loads otherwise -- the 14 / 23-wide inputs of layer 0).  k >= M read 0 (buffer range); rows past the
// operand's width read the next minibatch row's values, which only reach outputs that are not stored.
template <int NT>
struct Wg2 {
  static constexpr int NQ = TW2_T * TW2_KC / (4 * NT);   // b128 loads per operand and chunk
  static constexpr int NKQ = NT / 256, KW = TW2_KC / NKQ;
  static constexpr int NE = TW2_T * TW2_T / NT;          // output elements per thread
  static constexpr int CT = NT / TW2_T, CK = TW2_KC / CT; // colsum: threads per column, k per thread
};

template <int NT>
static __device__ __forceinline__ void wg2_issue(const Wg2Tile& t, int M, int kc, int tid, f32x4 (&va)[Wg2<NT>::NQ],
                                                 f32x4 (&vb)[Wg2<NT>::NQ]) {
  const auto dA = rsrc(t.A, (int64_t)M * t.K), dB = rsrc(t.B, (int64_t)M * t.N);
  const int r0 = 4 * (tid & 7), k0 = kc + (tid >> 3);
  const bool a4 = (t.K & 3) == 0, b4 = (t.N & 3) == 0;   // wave-uniform
#pragma unroll
  for (int q = 0; q < Wg2<NT>::NQ; ++q) {
    const int k = k0 + (NT / 8) * q;
    const int ia = k * t.K + t.i0 + r0, ib = k * t.N + t.j0 + r0;
    if (a4) va[q] = bload4(dA, ia);
    else va[q] = f32x4{bload(dA, ia), bload(dA, ia + 1), bload(dA, ia + 2), bload(dA, ia + 3)};
    if (b4) vb[q] = bload4(dB, ib);
    else vb[q] = f32x4{bload(dB, ib), bload(dB, ib + 1), bload(dB, ib + 2), bload(dB, ib + 3)};
  }
}

template <int NT>
static __device__ __forceinline__ void wg2_adam_in(const AdamCtx& ad, const Wg2Tile& t, int tid,
                                                   AdamIn (&a)[Wg2<NT>::NE], AdamIn& c) {
#pragma unroll
  for (int h = 0; h < Wg2<NT>::NE; ++h) {
    const int e = tid + NT * h;
    const int gi = min(t.i0 + (e >> 5), t.K - 1), gj = min(t.j0 + (e & 31), t.N - 1);
    const int64_t ix = t.w0 + (int64_t)gi * t.N + gj;
    a[h] = AdamIn{ad.Pc[ix], ad.M[ix], ad.V[ix], 0.f};   // no target copy in training (ad.T == NULL)
  }
  c = AdamIn{0.f, 0.f, 0.f, 0.f};
  if (t.cs && tid % Wg2<NT>::CT == 0) {
    const int64_t ix = t.b0 + min(t.j0 + tid / Wg2<NT>::CT, t.N - 1);
    c = AdamIn{ad.Pc[ix], ad.M[ix], ad.V[ix], 0.f};
  }
}

template <int NT>
// 512 threads: registers capped for 6 waves per SIMD, i.e. three workgroups per CU (the swizzled indexing
// otherwise takes 82 VGPRs: two)
static __global__ __launch_bounds__(NT, TRAIN_WG2_MINW > 0 ? TRAIN_WG2_MINW : (NT == 512 ? 6 : NT / 128)) void train_wgrad2_kernel(const TrainWg2 g) {
  using C = Wg2<NT>;
  __shared__ __attribute__((aligned(16))) float As[TW2_T * TW2_KP];   // [i][k]; later the K-part partials
  __shared__ __attribute__((aligned(16))) float Bs[TW2_T * TW2_KP];   // [j][k]
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (blockIdx.x == gridDim.x - 1) {   // the batch-level tail
    train_loss_tail(g.t, As);
    return;
  }
  const int x = blockIdx.x & 7, j = blockIdx.x >> 3;   // workgroups are dealt round-robin over the XCDs
  const int cnt = g.cnt[x];
  if (j >= cnt) return;
  const int32_t* lst = g.list + (int64_t)x * g.per_x;
  const int M = g.M;
  const AdamCtx& ad = g.ad;
  const float lr_t = *ad.lr_t;
  const int qd = w & 3, qi = qd >> 1, qj = qd & 1, kq = w >> 2, li = lane & 15, lk = lane >> 4;
  int i = j;
  Wg2Tile cur = wg2_tile(g, __builtin_amdgcn_readfirstlane(lst[i]));
  f32x4 va[C::NQ], vb[C::NQ];
  wg2_issue<NT>(cur, M, 0, tid, va, vb);
  AdamIn a_in[C::NE], c_in;
  wg2_adam_in<NT>(ad, cur, tid, a_in, c_in);
  while (true) {
    const int inx = i + g.nwx;
    const bool has_nx = inx < cnt;
    const Wg2Tile nx = wg2_tile(g, has_nx ? __builtin_amdgcn_readfirstlane(lst[inx]) : 0);
    AdamIn a_nx[C::NE], c_nx{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int h = 0; h < C::NE; ++h) a_nx[h] = AdamIn{0.f, 0.f, 0.f, 0.f};
    f32x4 acc0 = zero4(), acc1 = zero4();
    float cs = 0.f;
    for (int kc = 0; kc < M; kc += TW2_KC) {
      // re-derive the thread index here: otherwise the per-thread LDS / buffer offsets are hoisted out of
      // the loops and held in registers across them
      int tt = tid;
      asm volatile("" : "+v"(tt));
      {
        const int r0 = 4 * (tt & 7), k0 = tt >> 3;
#pragma unroll
        for (int q = 0; q < C::NQ; ++q)
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            As[tw2_at(r0 + u, k0 + (NT / 8) * q)] = va[q][u];
            Bs[tw2_at(r0 + u, k0 + (NT / 8) * q)] = vb[q][u];
          }
      }
      lds_barrier();
      // the next chunk, or the next tile's first chunk and Adam inputs, in flight during this one
      if (kc + TW2_KC < M) {
        wg2_issue<NT>(cur, M, kc + TW2_KC, tt, va, vb);
      } else if (has_nx) {
        wg2_issue<NT>(nx, M, 0, tt, va, vb);
        wg2_adam_in<NT>(ad, nx, tt, a_nx, c_nx);
      }
#pragma unroll
      for (int s = 0; s < C::KW / 16; ++s) {         // k = KW kq + (KW / 4) lk + 4 s + u
        const int k = C::KW * kq + (C::KW / 4) * lk + 4 * s;
        const f32x4 a4 = ld4(As + tw2_at(16 * qi + li, k)), b4 = ld4(Bs + tw2_at(16 * qj + li, k));
        acc0 = mfma4(a4[0], b4[0], acc0);
        acc1 = mfma4(a4[1], b4[1], acc1);
        acc0 = mfma4(a4[2], b4[2], acc0);
        acc1 = mfma4(a4[3], b4[3], acc1);
      }
      if (cur.cs) {                                  // column tid / CT, k = CK (tid % CT) .. + CK - 1
        const int crow = tid / C::CT, ck0 = C::CK * (tid % C::CT);
#pragma unroll
        for (int v = 0; v < C::CK; v += 4) {
          const f32x4 x0 = ld4(Bs + tw2_at(crow, ck0 + v));
          cs += (x0[0] + x0[1]) + (x0[2] + x0[3]);
        }
      }
      lds_barrier();
    }
    // ---- K parts through LDS (As reused), then decay + Adam per element
    float* part = As;
#pragma unroll
    for (int r = 0; r < 4; ++r) part[kq * 1024 + (16 * qi + 4 * lk + r) * 32 + 16 * qj + li] = acc0[r] + acc1[r];
    if (cur.cs) {
#pragma unroll
      for (int off = C::CT / 2; off > 0; off >>= 1) cs += __shfl_xor(cs, off);
    }
    lds_barrier();
#pragma unroll
    for (int h = 0; h < C::NE; ++h) {
      const int e = tid + NT * h;
      float v = part[e];
#pragma unroll
      for (int q = 1; q < C::NKQ; ++q) v += part[1024 * q + e];
      const int gi = cur.i0 + (e >> 5), gj = cur.j0 + (e & 31);
      if (gi < cur.K && gj < cur.N)
        adam_apply(ad, cur.w0 + (int64_t)gi * cur.N + gj, v + cur.wd * a_in[h].p, a_in[h], lr_t);   // fc.py:156-157
    }
    {
      const int cj = cur.j0 + tid / C::CT;
      if (cur.cs && tid % C::CT == 0 && cj < cur.N) adam_apply(ad, cur.b0 + cj, cs, c_in, lr_t);
    }
    if (!has_nx) break;
    lds_barrier();                                   // the partials are read before the next panels land
    i = inx;
    cur = nx;
    for (int h = 0; h < C::NE; ++h) a_in[h] = a_nx[h];
    c_in = c_nx;
  }
}

// MOPO_TRAIN_WG2 (default 1): the persistent XCD-local weight-gradient launch; 0: train_wgrad_kernel
int train_wg2() {
  static const int v = [] {
    const char* e = std::getenv("MOPO_TRAIN_WG2");
    return e ? std::atoi(e) : 1;
  }();
  return v;
}

// tiles of member e to XCD e mod 8 up to ceil(total / 8) per XCD, the rest to the least-loaded XCDs; within
// an XCD in (member, layer NHID .. 0, tile row, tile column) order, so a round's workgroups share panels
// host image: [8][per] tile lists (-1 padded) then the 8 counts; *per = the list stride
std::vector<int32_t> make_wlist(int E, int IN, int H, int D, int order, int* per_out) {
  std::vector<std::vector<int32_t>> xl(8);
  std::vector<int32_t> over;
  int total = 0;
  for (int l = 0; l <= NHID; ++l) {
    const int K = l == 0 ? IN : H, N = l == NHID ? 2 * D : H;
    total += E * ceil_div(K, TW2_T) * ceil_div(N, TW2_T);
  }
  const int target = ceil_div(total, 8);
  int rr = 0;
  for (int e = 0; e < E; ++e) {
    auto& home = xl[e % 8];
    for (int l = NHID; l >= 0; --l) {
      const int K = l == 0 ? IN : H, N = l == NHID ? 2 * D : H;
      for (int tm = 0; tm < ceil_div(K, TW2_T); ++tm)
        for (int tn = 0; tn < ceil_div(N, TW2_T); ++tn) {
          const int32_t v = l | (e << 3) | (tm << 7) | (tn << 12);
          if (order == 1) xl[rr++ % 8].push_back(v);
          else if ((int)home.size() < target) home.push_back(v);
          else over.push_back(v);
        }
    }
  }
  for (int32_t v : over) {
    int best = 0;
    for (int x = 1; x < 8; ++x)
      if (xl[x].size() < xl[best].size()) best = x;
    xl[best].push_back(v);
  }
  int per = 1;
  for (auto& v : xl) per = std::max(per, (int)v.size());
  std::vector<int32_t> host((size_t)8 * per + 8, -1);
  for (int x = 0; x < 8; ++x) {
    std::copy(xl[x].begin(), xl[x].end(), host.begin() + (size_t)x * per);
    host[(size_t)8 * per + x] = (int32_t)xl[x].size();
  }
  *per_out = per;
  return host;
}

int build_wlist(Train* h) {
  const Layout& L = h->L;
  static const int order = [] {   // MOPO_TRAIN_WG2_ORDER=1: tiles dealt round-robin, no member -> XCD grouping (A/B)
    const char* e = std::getenv("MOPO_TRAIN_WG2_ORDER");
    return e ? std::atoi(e) : 0;
  }();
  int per = 0;
  const std::vector<int32_t> host = make_wlist(L.E, L.IN, L.H, L.D, order, &per);
  if (hipMalloc(&h->wlist, host.size() * 4) != hipSuccess) return fail("bnn train: out of device memory (tile list)");
  h->wcnt = h->wlist + (size_t)8 * per;
  h->wl_per_x = per;
  MOPO_HIP(hipMemcpy(h->wlist, host.data(), host.size() * 4, hipMemcpyHostToDevice));
  return 0;
}

// threads per tile workgroup (MOPO_TRAIN_WG2_NT: 512, two per CU; or 1024, one per CU) and tile
// workgroups per XCD (MOPO_TRAIN_WG2_NWX; default: the CUs' resident workgroups)
int train_wg2_nt() {
  static const int v = [] {
    const char* e = std::getenv("MOPO_TRAIN_WG2_NT");
    const int n = e ? std::atoi(e) : 512;
    return n == 1024 ? 1024 : n == 256 ? 256 : 512;
  }();
  return v;
}
int train_wg2_nwx() {
  static const int v = [] {
    const char* e = std::getenv("MOPO_TRAIN_WG2_NWX");
    // the resident workgroups: three 512-thread ones per CU (TRAIN_WG2_KC), one 1024-thread one
    return e ? std::max(1, std::atoi(e)) : (train_wg2_nt() == 1024 ? 32 : train_wg2_nt() == 256 ? 192 : 96);
  }();
  return v;
}

#ifndef MOPO_TRAIN_FUSED
#define MOPO_TRAIN_FUSED 1  // forward + backward rows in one launch, the loss tail in the weight-gradient launch
#endif

// MOPO_TRAIN_STAGE (default 1): graph-captured full minibatches read rows the previous step gathered
// (train_rows.h TrainRows::staged); needs 16 (IN + D) <= 1024 (two items per row-block thread)
bool train_stage(const Train* h) {
  static const int v = [] {
    const char* e = std::getenv("MOPO_TRAIN_STAGE");
    return e ? std::atoi(e) : 1;
  }();
  return v != 0 && MOPO_TRAIN_FUSED && 16 * (h->L.IN + h->L.D) <= 2 * TR_WAVES * 64;
}


int step_rows(Train* h, int par, const float* in, const float* tg, const int32_t* idx, int64_t stride, bool use_bstep,
              int batch, int M, hipStream_t s, bool staged = false) {
  const Layout& L = h->L;
  const int E = L.E, H = L.H, IN = L.IN, D = L.D, D2 = 2 * D;
  const float* P = h->Pb[par];
  AdamCtx ad{};
  ad.G = h->G; ad.Pc = h->Pb[par]; ad.Pn = h->Pb[1 - par]; ad.M = h->M; ad.V = h->V; ad.T = nullptr;
  ad.lr_t = h->beta_pow + 2; ad.tau = 0.f; ad.total = L.total; ad.n_pi = 0; ad.n_q = 0; ad.norm_part = nullptr;
  TrainRows a{};
  a.E = E; a.M = M; a.IN = IN; a.H = H; a.D = D; a.nrb = ceil_div(M, 16);
  a.inputs = in; a.targets = tg; a.rows = idx; a.stride = stride; a.bstep = use_bstep ? h->bstep : nullptr;
  a.batch = batch; a.mu = h->mu; a.sigma = h->sigma; a.P = P;
  for (int l = 0; l <= NHID; ++l) { a.W[l] = L.W[l]; a.b[l] = L.b[l]; }
  a.mx = L.mx; a.mn = L.mn;
  a.X = h->X; a.T = h->T; a.OUT = h->OUT; a.dOUT = h->dOUT;
  if (staged) {   // step parity par reads X / T[par], gathers the next step into the other pair
    a.staged = 1;
    a.X = par ? h->X2 : h->X; a.T = par ? h->T2 : h->T;
    a.Xn = par ? h->X : h->X2; a.Tn = par ? h->T : h->T2;
  }
  for (int l = 0; l < NHID; ++l) { a.Z[l] = h->Z[l]; a.Hh[l] = h->Hh[l]; a.dZ[l] = h->dZ[l]; }
  a.lpart = h->lpart; a.logs = h->logs; a.beta_pow = h->beta_pow; a.bstep_inc = use_bstep ? h->bstep : nullptr;
  a.lr = h->lr; a.G = h->G; a.ad = ad;
  const int grid = 8 * a.nrb * ceil_div(E, 8);   // train_rows.h tr_block: a member's row blocks on one XCD
  const int g0 = ceil_div(IN, 16), gh = ceil_div(H, 16), gd = ceil_div(D2, 16);
  if (MOPO_TRAIN_FUSED) {
#define MOPO_TRF(G0, GH, GD)                                                                                 \
    if (g0 == G0 && gh == GH && gd == GD) {                                                                  \
      hipLaunchKernelGGL((train_rows_kernel<G0, GH, GD>), dim3(grid), dim3(TR_WAVES * 64), 0, s, a);                  \
      MOPO_HIP(hipGetLastError());                                                                           \
    } else
    MOPO_TRF(2, 13, 3) MOPO_TRF(1, 13, 2) MOPO_TRF(1, 2, 2) MOPO_TRF(2, 2, 3) MOPO_TRF(2, 16, 3) MOPO_TRF(1, 16, 2)
    return fail("bnn train: no row-block instantiation for these widths (use_rows)");
#undef MOPO_TRF
    // on this path h->G holds only the max/min log-var gradients (train_rows.h loss tail); the W/b
    // gradients stay in the tile workgroups' registers and go straight into Adam, never through G
    // (ad.G is then only the base the Adam state offsets are taken against)
    if (train_wg2()) {
      TrainWg2 g{};
      g.M = M;
      g.nwx = train_wg2_nwx();
      g.per_x = h->wl_per_x;
      g.list = h->wlist;
      g.cnt = h->wcnt;
      for (int l = 0; l <= NHID; ++l) {
        g.K[l] = l == 0 ? IN : H;
        g.N[l] = l == NHID ? D2 : H;
        g.A[l] = l == 0 ? a.X : h->Hh[l - 1];
        g.B[l] = l == NHID ? h->dOUT : h->dZ[l];
        g.W[l] = L.W[l];
        g.b[l] = L.b[l];
        g.wd[l] = WDECAY[l];
      }
      g.ad = ad;
      TrainTail& t = g.t;
      t.E = E; t.nrb = a.nrb; t.D = D; t.lpart = h->lpart; t.mx = L.mx; t.mn = L.mn;
      t.logs = h->logs; t.beta_pow = h->beta_pow; t.bstep_inc = a.bstep_inc; t.lr = h->lr; t.G = h->G; t.ad = ad;
      if (train_wg2_nt() == 1024) hipLaunchKernelGGL(train_wgrad2_kernel<1024>, dim3(8 * g.nwx + 1), dim3(1024), 0, s, g);
      else if (train_wg2_nt() == 256) hipLaunchKernelGGL(train_wgrad2_kernel<256>, dim3(8 * g.nwx + 1), dim3(256), 0, s, g);
      else hipLaunchKernelGGL(train_wgrad2_kernel<512>, dim3(8 * g.nwx + 1), dim3(512), 0, s, g);
      MOPO_HIP(hipGetLastError());
      return 0;
    }
    TrainWgrad g{};
    g.n = NHID + 1;
    g.ad = ad;
    int tot = 0;
    for (int l = NHID, i = 0; l >= 0; --l, ++i) {   // dW_l = X_in^T dY (+ db = colsum dY), decay + Adam; batch = member
      const int K = l == 0 ? IN : H, N = l == NHID ? D2 : H;
      const float* dY = l == NHID ? h->dOUT : h->dZ[l];
      const float* Xin = l == 0 ? a.X : h->Hh[l - 1];   // a.X: the staged pair
      GemmProb w = mk(K, N, M, Xin, K, 1, dY, N, 0, h->G + L.W[l], N);
      w.colsum = h->G + L.b[l];
      w.adam = 1;
      w.wd = WDECAY[l];
      w.nb = E;
      g.p[i] = w;
      g.prefix[i] = tot;
      tot += E * ceil_div(K, 32) * ceil_div(N, 32);
    }
    g.prefix[g.n] = tot;
    TrainTail& t = g.t;
    t.E = E; t.nrb = a.nrb; t.D = D; t.lpart = h->lpart; t.mx = L.mx; t.mn = L.mn;
    t.logs = h->logs; t.beta_pow = h->beta_pow; t.bstep_inc = a.bstep_inc; t.lr = h->lr; t.G = h->G; t.ad = ad;
    hipLaunchKernelGGL(train_wgrad_kernel, dim3(tot + 1), dim3(256), 0, s, g);
    MOPO_HIP(hipGetLastError());
    return 0;
  }
#define MOPO_TRR(G0, GH, GD)                                                                                 \
  if (g0 == G0 && gh == GH && gd == GD) {                                                                    \
    hipLaunchKernelGGL((train_fwd_rows_kernel<G0, GH>), dim3(grid), dim3(TR_WAVES * 64), 0, s, a);                     \
    MOPO_HIP(hipGetLastError());                                                                             \
    hipLaunchKernelGGL((train_bwd_rows_kernel<GD, GH>), dim3(grid + 1), dim3(TR_WAVES * 64), 0, s, a);                 \
    MOPO_HIP(hipGetLastError());                                                                             \
  } else
  MOPO_TRR(2, 13, 3) MOPO_TRR(1, 13, 2) MOPO_TRR(1, 2, 2) MOPO_TRR(2, 2, 3) MOPO_TRR(2, 16, 3) MOPO_TRR(1, 16, 2)
  return fail("bnn train: no row-block instantiation for these widths (use_rows)");
#undef MOPO_TRR
  std::vector<GemmProb> g;
  for (int l = NHID; l >= 0; --l) {   // dW_l = X_in^T dY (+ db = colsum dY), fused decay + Adam; batch = member
    const int K = l == 0 ? IN : H, N = l == NHID ? D2 : H;
    const float* dY = l == NHID ? h->dOUT : h->dZ[l];
    const float* Xin = l == 0 ? h->X : h->Hh[l - 1];
    auto w = mk(K, N, M, Xin, K, 1, dY, N, 0, h->G + L.W[l], N);
    w.colsum = h->G + L.b[l];
    w.adam = 1;
    w.wd = WDECAY[l];
    w.nb = E;
    g.push_back(w);
  }
  return launch_group(g, s, &ad, nullptr, nullptr, train_wgrad_tile());
}

int copy_back(Train* h, hipStream_t s) {
  MOPO_HIP(hipMemcpyAsync(h->Pb[0], h->Pb[1], h->L.total * 4, hipMemcpyDeviceToDevice, s));
  return 0;
}

void drop_graphs(Train* h) {
  for (int i = 0; i < 3; ++i) {
    if (h->gexec[i]) (void)hipGraphExecDestroy(h->gexec[i]);
    if (h->graph[i]) (void)hipGraphDestroy(h->graph[i]);
    h->gexec[i] = nullptr;
    h->graph[i] = nullptr;
  }
}

constexpr int TRAIN_GRAPH_STEPS = 8;

int capture(Train* h, int which, const float* in, const float* tg, const int32_t* idx, int64_t n_idx, int batch) {
  hipStream_t gs = h->gs;
  MOPO_HIP(hipStreamBeginCapture(gs, hipStreamCaptureModeThreadLocal));
  const int steps = which == 0 ? TRAIN_GRAPH_STEPS : which == 1 ? 2 : 1;
  int rc = 0;
  for (int i = 0; i < steps && !rc; ++i) {
    if (use_rows(h)) {
      rc = step_rows(h, i & 1, in, tg, idx, n_idx, true, batch, batch, gs, train_stage(h));
    } else {
      rc = launch_gather(h, in, tg, idx, n_idx, true, batch, batch, gs);
      if (!rc) rc = step_impl(h, i & 1, batch, true, gs);
    }
  }
  if (!rc && which == 2) rc = copy_back(h, gs);
  hipGraph_t g = nullptr;
  const hipError_t e = hipStreamEndCapture(gs, &g);
  if (rc) { if (g) (void)hipGraphDestroy(g); return -1; }
  if (e != hipSuccess) return fail(std::string("bnn train: capture failed: ") + hipGetErrorString(e));
  h->graph[which] = g;
  MOPO_HIP(hipGraphInstantiate(&h->gexec[which], g, nullptr, nullptr, 0));
  return 0;
}

}  // namespace
}  // namespace mopo

using namespace mopo;

extern "C" int mopo_bnn_train_create(mopo_bnn_train_t* out, int E, int obs_dim, int act_dim, int hidden,
                                     int max_batch, int max_eval, float lr) {
  MOPO_REQUIRE(out, "mopo_bnn_train_create: out is NULL");
  MOPO_REQUIRE(E >= 1 && E <= 16, "mopo_bnn_train_create: num_networks must be in [1, 16]");
  MOPO_REQUIRE(obs_dim >= 1 && act_dim >= 1 && hidden >= 1, "mopo_bnn_train_create: bad dims");
  MOPO_REQUIRE(obs_dim + 1 <= 64, "mopo_bnn_train_create: obs_dim + 1 must be <= 64");
  MOPO_REQUIRE(max_batch >= 1 && max_eval >= 0, "mopo_bnn_train_create: bad batch sizes");
  Train* h = new Train();
  h->L = make_layout(E, obs_dim + act_dim, hidden, obs_dim + 1);
  h->lr = lr;
  h->max_batch = max_batch; h->max_eval = max_eval;
  h->maxM = std::max(max_batch, max_eval);
  const Layout& L = h->L;
  const int64_t tot = (L.total + 3) / 4 * 4, mM = h->maxM;
  const int loss_blocks = L.D * ceil_div(E * h->maxM, LOSS_TPB);
  std::vector<std::pair<void**, size_t>> reg;
  auto f = [&](float** p, int64_t cnt) { reg.push_back({(void**)p, (size_t)cnt * 4}); };
  f(&h->Pb[0], tot); f(&h->Pb[1], tot); f(&h->G, tot); f(&h->M, tot); f(&h->V, tot); f(&h->S, tot);
  f(&h->beta_pow, 3); f(&h->part, 4 * (int64_t)loss_blocks);
  f(&h->lpart, 4 * (int64_t)E * ceil_div(max_batch, 16) * L.D); f(&h->logs, 4); f(&h->mu, L.IN); f(&h->sigma, L.IN);
  reg.push_back({(void**)&h->bstep, 4});
  reg.push_back({(void**)&h->ticket, 4});
  f(&h->X, E * mM * L.IN); f(&h->T, E * mM * L.D); f(&h->X2, E * max_batch * L.IN); f(&h->T2, E * max_batch * L.D); f(&h->OUT, E * mM * 2 * L.D); f(&h->dOUT, E * mM * 2 * L.D);
  for (int l = 0; l < NHID; ++l) { f(&h->Z[l], E * mM * L.H); f(&h->Hh[l], E * mM * L.H); f(&h->dZ[l], E * mM * L.H); }
  size_t bytes = 0;
  for (auto& r : reg) bytes += (r.second + 255) & ~(size_t)255;
  if (hipMalloc(&h->mem, bytes) != hipSuccess) { delete h; return fail("mopo_bnn_train_create: out of device memory"); }
  if (hipMemset(h->mem, 0, bytes) != hipSuccess) { (void)hipFree(h->mem); delete h; return fail("memset failed"); }
  char* m = (char*)h->mem;
  for (auto& r : reg) { *r.first = m; m += (r.second + 255) & ~(size_t)255; }
  const float bp[3] = {0.9f, 0.999f, 0.f};
  MOPO_HIP(hipMemcpy(h->beta_pow, bp, sizeof(bp), hipMemcpyHostToDevice));
  if (build_wlist(h)) { (void)hipFree(h->mem); delete h; return -1; }
  std::vector<float> one(L.IN, 1.f);
  MOPO_HIP(hipMemcpy(h->sigma, one.data(), L.IN * 4, hipMemcpyHostToDevice));
  *out = reinterpret_cast<mopo_bnn_train_t>(h);
  return 0;
}

// host only (no device call): the weight-gradient launch's per-XCD tile lists, for tests and tools
static int tile_lists(int E, int obs_dim, int act_dim, int hidden, int order, int32_t* out, int64_t cap);
extern "C" int mopo_bnn_train_tile_lists(int E, int obs_dim, int act_dim, int hidden, int32_t* out, int64_t cap) {
  return tile_lists(E, obs_dim, act_dim, hidden, 0, out, cap);
}
static int tile_lists(int E, int obs_dim, int act_dim, int hidden, int order, int32_t* out, int64_t cap) {
  MOPO_REQUIRE(E >= 1 && E <= 16 && obs_dim >= 1 && act_dim >= 1 && hidden >= 1 && obs_dim + 1 <= 64,
               "mopo_bnn_train_tile_lists: bad dims");
  // a packed tile id holds the tile row and column in 5 bits each (make_wlist): K, N <= 32 tiles of 32
  MOPO_REQUIRE(ceil_div(obs_dim + act_dim, TW2_T) <= 32 && ceil_div(hidden, TW2_T) <= 32 &&
               ceil_div(2 * (obs_dim + 1), TW2_T) <= 32,
               "mopo_bnn_train_tile_lists: hidden and obs_dim + act_dim must be <= 1024 (5-bit tile ids)");
  int per = 0;
  const std::vector<int32_t> host = make_wlist(E, obs_dim + act_dim, hidden, obs_dim + 1, order, &per);
  if (out) {
    MOPO_REQUIRE(cap >= (int64_t)host.size(), "mopo_bnn_train_tile_lists: output too small (8 per + 8 ints)");
    std::copy(host.begin(), host.end(), out);
  }
  return per;
}

// Diagnostic builds only (MOPO_TRAIN_STAMPS=1; otherwise -1): the rows launch's per-workgroup phase stamps
// of the last step ([block][8]: 0 start, 1 gathered, 2 layer 0, 3 forward, 4 loss, 5 / 6 / 7 backward), 100 MHz clock
extern "C" int mopo_bnn_train_debug_stamps(uint64_t* h_out, int64_t n) {
#if MOPO_TRAIN_STAMPS
  MOPO_REQUIRE(h_out && n >= 0 && n <= 2048 * 8, "mopo_bnn_train_debug_stamps: bad output");
  MOPO_HIP(hipDeviceSynchronize());
  MOPO_HIP(hipMemcpyFromSymbol(h_out, HIP_SYMBOL(g_train_stamps), n * 8));
  return 0;
#else
  (void)h_out; (void)n;
  return fail("mopo_bnn_train_debug_stamps: library built without MOPO_TRAIN_STAMPS");
#endif
}

extern "C" int mopo_bnn_train_destroy(mopo_bnn_train_t hh) {
  Train* h = reinterpret_cast<Train*>(hh);
  if (!h) return 0;
  drop_graphs(h);
  if (h->ev_in) (void)hipEventDestroy(h->ev_in);
  if (h->ev_out) (void)hipEventDestroy(h->ev_out);
  if (h->ev_order) (void)hipEventDestroy(h->ev_order);
  if (h->ev_applied) (void)hipEventDestroy(h->ev_applied);
  if (h->gs) (void)hipStreamDestroy(h->gs);
  if (h->sort_keys) (void)hipFree(h->sort_keys);  // one allocation (keys | values | offsets | temp)
  if (h->wlist) (void)hipFree(h->wlist);
  if (h->mem) (void)hipFree(h->mem);
  delete h;
  return 0;
}

// .mat order (smv, 16 arrays): mu, sigma, (W, b) x 5 mean layers, (Wv, bv), maxlv, minlv
extern "C" int mopo_bnn_train_set_params(mopo_bnn_train_t hh, const float* const* a) {
  Train* h = reinterpret_cast<Train*>(hh);
  MOPO_REQUIRE(h && a, "mopo_bnn_train_set_params: NULL argument");
  const Layout& L = h->L;
  const int E = L.E, H = L.H, D = L.D;
  std::vector<float> P(L.total);
  for (int l = 0; l < NHID; ++l) {
    const int in = l == 0 ? L.IN : H;
    std::memcpy(P.data() + L.W[l], a[2 + 2 * l], (size_t)E * in * H * 4);
    std::memcpy(P.data() + L.b[l], a[3 + 2 * l], (size_t)E * H * 4);
  }
  for (int e = 0; e < E; ++e) {
    for (int k = 0; k < H; ++k)
      for (int j = 0; j < D; ++j) {
        P[L.W[NHID] + ((int64_t)e * H + k) * 2 * D + j] = a[10][((int64_t)e * H + k) * D + j];
        P[L.W[NHID] + ((int64_t)e * H + k) * 2 * D + D + j] = a[12][((int64_t)e * H + k) * D + j];
      }
    for (int j = 0; j < D; ++j) {
      P[L.b[NHID] + (int64_t)e * 2 * D + j] = a[11][e * D + j];
      P[L.b[NHID] + (int64_t)e * 2 * D + D + j] = a[13][e * D + j];
    }
  }
  std::memcpy(P.data() + L.mx, a[14], D * 4);
  std::memcpy(P.data() + L.mn, a[15], D * 4);
  MOPO_HIP(hipMemcpy(h->Pb[0], P.data(), L.total * 4, hipMemcpyHostToDevice));
  MOPO_HIP(hipMemcpy(h->Pb[1], P.data(), L.total * 4, hipMemcpyHostToDevice));
  MOPO_HIP(hipMemcpy(h->mu, a[0], L.IN * 4, hipMemcpyHostToDevice));
  MOPO_HIP(hipMemcpy(h->sigma, a[1], L.IN * 4, hipMemcpyHostToDevice));
  // a fresh optimizer (the reference initialises the Adam slots with the graph, bnn.py:252)
  MOPO_HIP(hipMemset(h->M, 0, L.total * 4));
  MOPO_HIP(hipMemset(h->V, 0, L.total * 4));
  const float bp[3] = {0.9f, 0.999f, 0.f};
  MOPO_HIP(hipMemcpy(h->beta_pow, bp, sizeof(bp), hipMemcpyHostToDevice));
  h->snap.clear();
  return 0;
}

extern "C" int mopo_bnn_train_get_params(mopo_bnn_train_t hh, float* const* a) {
  Train* h = reinterpret_cast<Train*>(hh);
  MOPO_REQUIRE(h && a, "mopo_bnn_train_get_params: NULL argument");
  const Layout& L = h->L;
  const int E = L.E, H = L.H, D = L.D;
  MOPO_HIP(hipDeviceSynchronize());
  std::vector<float> P(L.total);
  MOPO_HIP(hipMemcpy(P.data(), h->Pb[0], L.total * 4, hipMemcpyDeviceToHost));
  MOPO_HIP(hipMemcpy(a[0], h->mu, L.IN * 4, hipMemcpyDeviceToHost));
  MOPO_HIP(hipMemcpy(a[1], h->sigma, L.IN * 4, hipMemcpyDeviceToHost));
  for (int l = 0; l < NHID; ++l) {
    const int in = l == 0 ? L.IN : H;
    std::memcpy(a[2 + 2 * l], P.data() + L.W[l], (size_t)E * in * H * 4);
    std::memcpy(a[3 + 2 * l], P.data() + L.b[l], (size_t)E * H * 4);
  }
  for (int e = 0; e < E; ++e) {
    for (int k = 0; k < H; ++k)
      for (int j = 0; j < D; ++j) {
        a[10][((int64_t)e * H + k) * D + j] = P[L.W[NHID] + ((int64_t)e * H + k) * 2 * D + j];
        a[12][((int64_t)e * H + k) * D + j] = P[L.W[NHID] + ((int64_t)e * H + k) * 2 * D + D + j];
      }
    for (int j = 0; j < D; ++j) {
      a[11][e * D + j] = P[L.b[NHID] + (int64_t)e * 2 * D + j];
      a[13][e * D + j] = P[L.b[NHID] + (int64_t)e * 2 * D + D + j];
    }
  }
  std::memcpy(a[14], P.data() + L.mx, D * 4);
  std::memcpy(a[15], P.data() + L.mn, D * 4);
  return 0;
}

extern "C" int mopo_bnn_format_samples(const mopo_pool_desc* pool, int O, int A, const int64_t* d_rows, int64_t n,
                                       float* d_inputs, float* d_targets, void* stream) {
  MOPO_REQUIRE(pool && d_inputs && d_targets, "mopo_bnn_format_samples: NULL argument");
  MOPO_REQUIRE(n >= 0, "mopo_bnn_format_samples: n < 0");
  if (n == 0) return 0;
  const int64_t tot = n * (2 * O + A + 1);
  hipLaunchKernelGGL(format_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, (hipStream_t)stream, *pool, O, A,
                     d_rows, n, d_inputs, d_targets);
  MOPO_HIP(hipGetLastError());
  return 0;
}

extern "C" int mopo_bnn_train_fit_scaler(mopo_bnn_train_t hh, const float* d_inputs, int64_t n, void* stream) {
  Train* h = reinterpret_cast<Train*>(hh);
  MOPO_REQUIRE(h && d_inputs && n > 0, "mopo_bnn_train_fit_scaler: bad argument");
  hipLaunchKernelGGL(scaler_fit_kernel, dim3(h->L.IN), dim3(256), 0, (hipStream_t)stream, d_inputs, n, h->L.IN, h->mu,
                     h->sigma);
  MOPO_HIP(hipGetLastError());
  return 0;
}

extern "C" int mopo_bnn_train_epoch(mopo_bnn_train_t hh, const float* d_in, const float* d_tg, const int32_t* d_idxs,
                                    int64_t n_idx, int batch, void* stream) {
  Train* h = reinterpret_cast<Train*>(hh);
  MOPO_REQUIRE(h && d_in && d_tg && d_idxs, "mopo_bnn_train_epoch: NULL argument");
  MOPO_REQUIRE(batch >= 1 && batch <= h->max_batch, "mopo_bnn_train_epoch: batch exceeds max_batch");
  MOPO_REQUIRE(n_idx >= 1, "mopo_bnn_train_epoch: empty index set");
  hipStream_t s = (hipStream_t)stream;
  const int64_t nb = (n_idx + batch - 1) / batch;
  const int last = (int)(n_idx - (nb - 1) * batch);
  const int64_t nfull = last == batch ? nb : nb - 1;
  if (!h->gs) {
    MOPO_HIP(hipStreamCreateWithFlags(&h->gs, hipStreamNonBlocking));
    MOPO_HIP(hipEventCreateWithFlags(&h->ev_in, hipEventDisableTiming));
    MOPO_HIP(hipEventCreateWithFlags(&h->ev_out, hipEventDisableTiming));
  }
  hipStream_t gs = h->gs;
  MOPO_HIP(hipEventRecord(h->ev_in, s));
  MOPO_HIP(hipStreamWaitEvent(gs, h->ev_in, 0));
  MOPO_HIP(hipMemsetAsync(h->bstep, 0, 4, gs));
  if (nfull > 0) {
    if (!h->gexec[0] || h->gkey[0] != d_in || h->gkey[1] != d_tg || h->gkey[2] != d_idxs || h->gkey_n != n_idx ||
        h->gkey_b != batch) {
      drop_graphs(h);
      if (capture(h, 0, d_in, d_tg, d_idxs, n_idx, batch) || capture(h, 1, d_in, d_tg, d_idxs, n_idx, batch) ||
          capture(h, 2, d_in, d_tg, d_idxs, n_idx, batch))
        return -1;
      h->gkey[0] = d_in; h->gkey[1] = d_tg; h->gkey[2] = d_idxs; h->gkey_n = n_idx; h->gkey_b = batch;
    }
    // staged steps: the epoch's first minibatch is gathered here, every later one by the step before it
    if (use_rows(h) && train_stage(h) && launch_gather(h, d_in, d_tg, d_idxs, n_idx, true, batch, batch, gs))
      return -1;
    int64_t i = 0;
    for (; i + TRAIN_GRAPH_STEPS <= nfull; i += TRAIN_GRAPH_STEPS) MOPO_HIP(hipGraphLaunch(h->gexec[0], gs));
    for (; i + 2 <= nfull; i += 2) MOPO_HIP(hipGraphLaunch(h->gexec[1], gs));
    if (i < nfull) MOPO_HIP(hipGraphLaunch(h->gexec[2], gs));
  }
  if (nfull < nb) {  // the epoch's partial last minibatch (bnn.py:426: idxs[:, b*bs:(b+1)*bs])
    if (use_rows(h)) {
      if (step_rows(h, 0, d_in, d_tg, d_idxs, n_idx, true, batch, last, gs) || copy_back(h, gs)) return -1;
    } else if (launch_gather(h, d_in, d_tg, d_idxs, n_idx, true, batch, last, gs) || step_impl(h, 0, last, true, gs) ||
               copy_back(h, gs)) {
      return -1;
    }
  }
  MOPO_HIP(hipEventRecord(h->ev_out, gs));
  MOPO_HIP(hipStreamWaitEvent(s, h->ev_out, 0));
  return 0;
}

extern "C" int mopo_bnn_train_eval_mse(mopo_bnn_train_t hh, const float* d_in, const float* d_tg, const int32_t* d_rows,
                                       int n, float* d_losses, void* stream) {
  Train* h = reinterpret_cast<Train*>(hh);
  MOPO_REQUIRE(h && d_in && d_tg && d_losses, "mopo_bnn_train_eval_mse: NULL argument");
  MOPO_REQUIRE(n >= 1 && n <= h->maxM, "mopo_bnn_train_eval_mse: n must be in [1, max(max_batch, max_eval)]");
  hipStream_t s = (hipStream_t)stream;
  if (launch_gather(h, d_in, d_tg, d_rows, n, false, 0, n, s) ||
      forward(h, h->Pb[0], n, s, n >= 32 ? eval_tile() : 0))
    return -1;
  hipLaunchKernelGGL(train_mse_kernel, dim3(h->L.E), dim3(MSE_TPB), 0, s, h->OUT, h->T, n, h->L.D, d_losses);
  MOPO_HIP(hipGetLastError());
  return 0;
}

extern "C" int mopo_bnn_train_shuffle(mopo_bnn_train_t hh, int32_t* d_idxs, const double* d_keys, int64_t n,
                                      void* stream) {
  return mopo_bnn_train_shuffle_async(hh, d_idxs, d_keys, n, stream, stream);
}

extern "C" int mopo_bnn_train_shuffle_async(mopo_bnn_train_t hh, int32_t* d_idxs, const double* d_keys, int64_t n,
                                            void* order_stream, void* stream) {
  Train* h = reinterpret_cast<Train*>(hh);
  MOPO_REQUIRE(h && d_idxs && d_keys && n >= 1, "mopo_bnn_train_shuffle: bad argument");
  MOPO_REQUIRE(n * h->L.E < (1ll << 31), "mopo_bnn_train_shuffle: index set too large");
  hipStream_t s = (hipStream_t)stream, os = (hipStream_t)order_stream;
  const int E = h->L.E;
  const int64_t tot = n * E;
  int seg_bits = 0;
  while ((1 << seg_bits) < E) ++seg_bits;
  const int end_bit = 53 + seg_bits;
  if (!h->ev_order) {
    MOPO_HIP(hipEventCreateWithFlags(&h->ev_order, hipEventDisableTiming));
    MOPO_HIP(hipEventCreateWithFlags(&h->ev_applied, hipEventDisableTiming));
  }
  if (h->sort_cap < tot) {
    MOPO_HIP(hipStreamSynchronize(s));           // the buffers below may still be read by an earlier apply
    if (h->sort_keys) (void)hipFree(h->sort_keys);
    h->sort_tmp = nullptr; h->sort_keys = nullptr;
    size_t tb = 0;
    MOPO_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                                (const int32_t*)nullptr, (int32_t*)nullptr, (int)tot, 0, end_bit, os));
    // one allocation: keys in | keys out | values in | values out | temp storage
    const size_t kb = (size_t)tot * 8, vb = (size_t)tot * 4;
    char* m = nullptr;
    MOPO_HIP(hipMalloc((void**)&m, 2 * kb + 2 * vb + tb + 1024));
    h->sort_keys = (double*)m;
    h->sort_vals_in = (int32_t*)(m + 2 * kb);
    h->sort_vals = (int32_t*)(m + 2 * kb + vb);
    h->sort_tmp = (void*)(((uintptr_t)(m + 2 * kb + 2 * vb) + 255) & ~(uintptr_t)255);
    h->sort_tmp_bytes = tb;
    h->sort_cap = tot;
  } else if (os != s) {
    // the order is computed on the caller's order stream, which can run beside the epoch's steps; it
    // must not overwrite the order buffers before the previous shuffle's apply has read them
    MOPO_HIP(hipStreamWaitEvent(os, h->ev_applied, 0));
  }
  uint64_t* kin = reinterpret_cast<uint64_t*>(h->sort_keys);
  uint64_t* kout = kin + h->sort_cap;
  hipLaunchKernelGGL(sort_keys_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, os, d_keys, n, E, kin,
                     h->sort_vals_in);
  MOPO_HIP(hipGetLastError());
  size_t tb = h->sort_tmp_bytes;
  // one radix sort of (member, 53-bit integer of the uniform) == np.argsort within each member row
  MOPO_HIP(hipcub::DeviceRadixSort::SortPairs(h->sort_tmp, tb, kin, kout, h->sort_vals_in, h->sort_vals, (int)tot, 0,
                                              end_bit, os));
  if (os != s) {
    MOPO_HIP(hipEventRecord(h->ev_order, os));
    MOPO_HIP(hipStreamWaitEvent(s, h->ev_order, 0));
  }
  int32_t* tmp_idx = h->sort_vals_in;  // reuse: copy of the current indices
  MOPO_HIP(hipMemcpyAsync(tmp_idx, d_idxs, tot * 4, hipMemcpyDeviceToDevice, s));
  hipLaunchKernelGGL(apply_order_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, h->sort_vals, tmp_idx,
                     n, E, d_idxs);
  MOPO_HIP(hipGetLastError());
  MOPO_HIP(hipEventRecord(h->ev_applied, s));
  return 0;
}

extern "C" int mopo_bnn_train_snapshot(mopo_bnn_train_t hh, int member, void* stream) {
  Train* h = reinterpret_cast<Train*>(hh);
  MOPO_REQUIRE(h && member >= 0 && member < h->L.E, "mopo_bnn_train_snapshot: bad member");
  hipLaunchKernelGGL(member_copy_kernel, dim3(64, 2 * (NHID + 1)), dim3(256), 0, (hipStream_t)stream, h->Pb[0], h->S,
                     member_span(h->L), member, 0);
  MOPO_HIP(hipGetLastError());
  if (std::find(h->snap.begin(), h->snap.end(), member) == h->snap.end()) h->snap.push_back(member);
  return 0;
}

static int copy_members(Train* h, const std::vector<int>& members, int dir, hipStream_t s) {
  for (size_t i0 = 0; i0 < members.size(); i0 += MAX_MEMBERS_SET) {
    MemberSet ms{};
    ms.n = (int)std::min(members.size() - i0, (size_t)MAX_MEMBERS_SET);
    for (int i = 0; i < ms.n; ++i) ms.e[i] = members[i0 + i];
    hipLaunchKernelGGL(members_copy_kernel, dim3(64, 2 * (NHID + 1), ms.n), dim3(256), 0, s, h->Pb[0], h->S,
                       member_span(h->L), ms, dir);
    MOPO_HIP(hipGetLastError());
  }
  return 0;
}

extern "C" int mopo_bnn_train_snapshot_members(mopo_bnn_train_t hh, const int* h_members, int n, void* stream) {
  Train* h = reinterpret_cast<Train*>(hh);
  MOPO_REQUIRE(h && (h_members || n == 0) && n >= 0, "mopo_bnn_train_snapshot_members: bad argument");
  std::vector<int> ms;
  for (int i = 0; i < n; ++i) {
    const int e = h_members[i];
    MOPO_REQUIRE(e >= 0 && e < h->L.E, "mopo_bnn_train_snapshot_members: bad member");
    if (std::find(ms.begin(), ms.end(), e) == ms.end()) ms.push_back(e);
  }
  if (ms.empty()) return 0;
  if (copy_members(h, ms, 0, (hipStream_t)stream)) return -1;
  for (int e : ms)
    if (std::find(h->snap.begin(), h->snap.end(), e) == h->snap.end()) h->snap.push_back(e);
  return 0;
}

extern "C" int mopo_bnn_train_restore(mopo_bnn_train_t hh, void* stream) {
  Train* h = reinterpret_cast<Train*>(hh);
  MOPO_REQUIRE(h, "mopo_bnn_train_restore: NULL handle");
  if (!h->snap.empty() && copy_members(h, h->snap, 1, (hipStream_t)stream)) return -1;
  h->snap.clear();
  return 0;
}

extern "C" int mopo_bnn_train_logs(mopo_bnn_train_t hh, float* h_logs, int n) {
  Train* h = reinterpret_cast<Train*>(hh);
  MOPO_REQUIRE(h && h_logs && n >= 1 && n <= 4, "mopo_bnn_train_logs: bad argument");
  MOPO_HIP(hipDeviceSynchronize());
  MOPO_HIP(hipMemcpy(h_logs, h->logs, n * 4, hipMemcpyDeviceToHost));
  return 0;
}
