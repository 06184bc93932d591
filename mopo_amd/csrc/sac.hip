// MOPO's in-graph SAC update (K6/K7): forward, hand-derived backward, four TF1 Adams, Polyak.
//
// Replaces MOPO._build's training graph and MOPO._do_training / _update_target
// (mopo/algorithms/mopo.py:275-466, 834-853); batch assembly MOPO._training_batch (mopo.py:801-821).
// Semantics: every forward and gradient uses the pre-step parameters; then pi, q1, q2
// and alpha are updated by their own Adam (identical step counts -> one shared lr_t); then Polyak.
//
// Structure: 4 launches per step on one stream, captured into hipGraphs of 8 / 2 / 1 steps (no host
// work per step).  Everything up to the activation gradients is row-local, so it runs in three
// row-block launches (sac_rows.h) that hand each other per-column-block partial dot products instead
// of full rows: F1 the hidden layers of pi(s), pi(s'), Q1/Q2(s,a) + partial output layers; F2 the
// policy head (from F1's partials) feeding the hidden layers of Q1/Q2(s,pi) and the target critics +
// partial output layers, and the (s, pi) critics' action-gradient partials; B1 each row's TD target
// and dq (from the partials), the critics' dh1, the policy's row-local backward chain (head backward
// -> dh2p -> dh1p), the step control (lr_t) and the gather of the next step's batch.  Then ONE launch
// (sac_wgrad.h) computes every weight gradient with its TF1 Adam (+ Polyak for the critics) fused
// into the epilogue, reading parameters Pb[p] and writing Pb[1 - p] (every gradient of the step sees
// pre-step parameters), beside the batch loss tail (logs, the alpha update, the step counter).
#include <vector>
#include <cstring>
#include <cstdlib>

#define MOPO_GEMM_KERNELS 0   // the grouped-GEMM kernels are bnn_train.hip's; this file uses the helpers only
#include "sac_wgrad.h"

namespace mopo {

// ---------------------------------------------------------------------------------------------
struct SacDims { int O, A, H, n, n_env; int64_t P; };

// parameter offsets (flat, TF creation order; mopo.py:32-33)
struct Offs {
  int64_t pW1, pb1, pW2, pb2, pWm, pbm, pWl, pbl;
  int64_t q[2][6];  // W1 b1 W2 b2 W3 b3 for q1, q2
  int64_t n_pi, n_q, total;
};

static Offs make_offs(int O, int A, int H) {
  Offs o{};
  int64_t c = 0;
  auto take = [&](int64_t n) { int64_t r = c; c += n; return r; };
  o.pW1 = take((int64_t)O * H); o.pb1 = take(H); o.pW2 = take((int64_t)H * H); o.pb2 = take(H);
  o.pWm = take((int64_t)H * A); o.pbm = take(A); o.pWl = take((int64_t)H * A); o.pbl = take(A);
  o.n_pi = c;
  for (int qi = 0; qi < 2; ++qi) {
    o.q[qi][0] = take((int64_t)(O + A) * H); o.q[qi][1] = take(H); o.q[qi][2] = take((int64_t)H * H);
    o.q[qi][3] = take(H); o.q[qi][4] = take(H); o.q[qi][5] = take(1);
  }
  o.n_q = o.q[1][0] - o.q[0][0];
  o.total = c;
  return o;
}


struct Sac {
  SacDims d{};
  Offs o{};
  float lr, gamma, tau, rscale, tent;
  void* mem = nullptr;
  float *P, *G, *M, *V, *T;       // [total + 1]: last element = log_alpha
  float* Pb[2];                   // parameter ping-pong: Pb[0] == P is the canonical copy between calls
  float* norm_part = nullptr;     // [nslots][2]
  int nslots = 0, nslots_cap = 0;
  float* beta_pow;                // [4] f32 beta1_power, beta2_power (TF1 non-slot vars), this step's lr_t,
                                  //     this step's target-update flag
  int64_t* iter;                  // device step counter (Philox)
  int64_t* tctl;                  // [3] target schedule: base step, n_train_repeat, target_update_interval
  float* logs;                    // [LOG_N]
  // activations
  Batch bt[2];                    // double-buffered batch (step parity)
  float *h1[8], *h2[8], *out[8];  // 0 pi(s) 1 pi(s') 2 Q1(s,a) 3 Q2(s,a) 4 Q1(s,pi) 5 Q2(s,pi) 6 Qt1 7 Qt2
  float *logp_s, *logp_n, *eps_s, *eps_n;
  float *dq[4];                   // dq for instances 2,3,4,5
  float *dh1[4];
  float *opart[8];                // [ncq][n][OPW] output-layer partials of the 8 instances (sac_rows.h)
  float *dapart[2];               // [ncq][n][OPW] action-gradient partials of Q1 / Q2 at (s, pi(s))
  uint64_t* stamps = nullptr;     // MOPO_SAC_STAMPS builds: [slot][block][8]
  unsigned* sync = nullptr;       // fused F2 + B1 launch: [nrb][2] row-block counters, then the timeout word
                                  //   (each on its own 128-B line: sac_rows.h SYNC_STRIDE)
  int fuse = 2;                   // 0: F1, F2, B1 separate; 1: F2 + B1 one launch; 2: F1 + F2 + B1 one launch
  float *dhead, *dh2p, *dh1p;
  // graph
  bool use_graph = true;
  hipGraphExec_t gexec[3] = {nullptr, nullptr, nullptr};
  hipGraph_t graph[3] = {nullptr, nullptr, nullptr};
  int prior = 0;                  // action_prior 'normal' (mopo_sac_set_action_prior)
  mopo_pool_desc genv{}, gmod{};
  hipStream_t gstream = nullptr;
  hipEvent_t ev_in = nullptr, ev_out = nullptr;
  uint64_t gseed = 0;
};

// ---- batch gather (gemm_group.h gather_elem), as its own launch for a call's first step
constexpr int GATHER_TPB = 256;
__global__ __launch_bounds__(GATHER_TPB) void sac_gather_kernel(const GatherArgs g, int n) {
  const int C = 2 * g.O + g.A + 2;
  const int e = blockIdx.x * GATHER_TPB + threadIdx.x;
  if (e >= n * C) return;
  const int r = e / C;
  gather_elem(g, r, e - r * C);
}

__device__ __forceinline__ float softplus_f(float x) { return softplusf(x); }

// Deterministic block-wide sums of NV values at once: butterfly within each wave (__shfl_xor),
// then the per-wave partials added in wave order.  Two barriers for all NV sums.
// sh must hold 16 * NV floats; blockDim.x a multiple of 64 (<= 1024).
template <int NV>
__device__ __forceinline__ void block_sums(float (&v)[NV], float* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v[i] += __shfl_xor(v[i], off);
  if (lane == 0)
#pragma unroll
    for (int i = 0; i < NV; ++i) sh[w * NV + i] = v[i];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    float s = 0.f;
    for (int q = 0; q < nw; ++q) s += sh[q * NV + i];
    v[i] = s;
  }
  __syncthreads();
}

__device__ __forceinline__ float block_sum(float v, float* sh) {
  float a[1] = {v};
  block_sums<1>(a, sh);
  return a[0];
}

// grad-norm logs of the last step (once per mopo_sac_step call): the per-block partials of the
// fused optimizer epilogues, plus the alpha gradient (counted with neither network)
__global__ __launch_bounds__(256) void sac_logs_kernel(const float* norm_part, int nslots, float* logs) {
  __shared__ float sh[64];
  float a = 0.f, b = 0.f;
  for (int i = threadIdx.x; i < nslots; i += blockDim.x) {
    a += norm_part[2 * i];
    b += norm_part[2 * i + 1];
  }
  float ab[2] = {a, b};
  block_sums<2>(ab, sh);
  if (threadIdx.x == 0) {
    logs[LOG_PI_GNORM] = sqrtf(ab[0]);
    logs[LOG_Q_GNORM] = 0.5f * sqrtf(ab[1]);                        // grads of Q_loss = (l1+l2)/2 wrt q1
  }
}

static GatherArgs gather_args(Sac* h, int par, const mopo_pool_desc* env, const mopo_pool_desc* mod, uint64_t seed,
                              const int64_t* idx_in) {
  GatherArgs g{};
  g.env = *env; g.mod = *mod; g.n = h->d.n; g.n_env = h->d.n_env; g.O = h->d.O; g.A = h->d.A;
  g.idx_in = idx_in; g.seed = seed; g.iter = h->iter; g.out = h->bt[par];
  return g;
}

static int launch_gather(Sac* h, int par, const mopo_pool_desc* env, const mopo_pool_desc* mod, uint64_t seed,
                         const int64_t* idx_in, hipStream_t s) {
  const SacDims& d = h->d;
  hipLaunchKernelGGL(sac_gather_kernel, dim3(ceil_div(d.n * (2 * d.O + d.A + 2), GATHER_TPB)), dim3(GATHER_TPB), 0, s,
                     gather_args(h, par, env, mod, seed, idx_in), d.n);
  MOPO_HIP(hipGetLastError());
  return 0;
}

// One SAC step on batch bt[par], reading parameters Pb[par] and writing the updated ones to
// Pb[1 - par].  With `prefetch`, B1 also gathers the next step's batch into bt[1 - par] (a separate
// gather launch, or a forked graph branch, costs more than it hides).
#ifndef MOPO_SAC_FUSE
#define MOPO_SAC_FUSE 2   // 0: F1, F2, B1 as three launches; 1: F2 + B1 fused; 2: F1 + F2 + B1 fused (the
                          // environment variable MOPO_SAC_FUSE overrides it at mopo_sac_create: the separate
                          // launches are the fused form's bit-identical cross-check in tests/test_gpu_sac.py)
#endif
static int sac_fuse_default() {
  const char* e = std::getenv("MOPO_SAC_FUSE");
  const int v = e ? std::atoi(e) : MOPO_SAC_FUSE;
  return v < 0 ? 0 : v > 2 ? 2 : v;
}

static int sac_step_impl(Sac* h, int par, const mopo_pool_desc* env, const mopo_pool_desc* mod, uint64_t seed,
                         const float* eps_in_s, const float* eps_in_n, hipStream_t s, bool prefetch) {
  const SacDims& d = h->d;
  const Offs& o = h->o;
  const int n = d.n, O = d.O, A = d.A, H = d.H, W = O + A;
  const float* P = h->Pb[par];
  AdamCtx ad{};
  ad.G = h->G; ad.Pc = h->Pb[par]; ad.Pn = h->Pb[1 - par]; ad.M = h->M; ad.V = h->V; ad.T = h->T;
  ad.lr_t = h->beta_pow + 2; ad.tau = h->tau; ad.total = o.total; ad.n_pi = o.n_pi; ad.n_q = o.n_q;
  ad.norm_part = h->norm_part;
  ad.tgt_on = h->beta_pow + 3;
  const float* T = h->T;
  float* G = h->G;
  const Batch& bt = h->bt[par];
  auto Wq = [&](int qi, int k) { return P + o.q[qi][k]; };
  auto Tq = [&](int qi, int k) { return T + o.q[qi][k]; };
  const int ncq = ceil_div(H, RB_COLS), nrb = ceil_div(n, 16);
  LossRows L{};
  for (int i = 0; i < 6; ++i) {
    L.qpart[i] = h->opart[2 + i];
    L.b3[i] = i < 4 ? Wq(i & 1, 5) : Tq(i & 1, 5);
  }
  L.logp_s = h->logp_s; L.logp_n = h->logp_n; L.head_s = h->out[0]; L.rew = bt.rew; L.term = bt.term;
  L.log_alpha = P + o.total; L.gamma = h->gamma; L.rscale = h->rscale;
  // ---- F1: pi(s), pi(s'), Q1(s,a), Q2(s,a) hidden layers + partial output layers
  FwdArgsR f1{};
  {
    FwdArgsR& f = f1;
    f.ninst = 4; f.n = n; f.H = H; f.A = A; f.ncq = ncq; f.nrb = nrb;
    for (int i = 0; i < 2; ++i) {
      FwdInst& q = f.in[i];
      q.x = i == 0 ? bt.sa : bt.xn; q.ldx = W; q.kx = O; q.k1 = O;
      q.w1 = P + o.pW1; q.b1 = P + o.pb1; q.w2 = P + o.pW2; q.b2 = P + o.pb2;
      q.h1 = i == 0 ? h->h1[0] : nullptr; q.h2 = i == 0 ? h->h2[0] : nullptr;   // pi(s') needs no gradient
      q.wo = P + o.pWm; q.wo2 = P + o.pWl; q.nout = 2 * A; q.split = A; q.opart = h->opart[i];
    }
    for (int qi = 0; qi < 2; ++qi) {
      FwdInst& q = f.in[2 + qi];
      q.x = bt.sa; q.ldx = W; q.kx = W; q.k1 = W;
      q.w1 = Wq(qi, 0); q.b1 = Wq(qi, 1); q.w2 = Wq(qi, 2); q.b2 = Wq(qi, 3);
      q.h1 = h->h1[2 + qi]; q.h2 = h->h2[2 + qi];
      q.wo = Wq(qi, 4); q.wo2 = nullptr; q.nout = 1; q.split = 1; q.opart = h->opart[2 + qi];
    }
    f.hd.iter = h->iter; f.hd.seed = seed; f.hd.eps_out[0] = h->eps_s; f.hd.eps_out[1] = h->eps_n;
    f.hd.gen_eps = (eps_in_s ? 0 : 1) | (eps_in_n ? 0 : 2);   // the heads whose noise is not injected
    f.st = Stamps{h->stamps, 0};
    if (h->fuse == 1) { f.sync_reset = h->sync; f.n_sync = SYNC_N * nrb; }   // this step's F2 -> B1 counters
    f.sync = h->sync;
    if (h->fuse < 2) {
      hipLaunchKernelGGL(sac_fwd_kernel<false>, dim3(ncq, nrb, 4), dim3(256), 0, s, f);
      MOPO_HIP(hipGetLastError());
    }
  }
  // ---- F2: the policy head from F1's partials -> Q1/Q2(s, pi(s)) (main), Qt1/Qt2(s', pi(s')) (target);
  //      the main critics' blocks also emit their action-gradient partials (dq = 1)
  FwdArgsR f2{};
  {
    FwdArgsR& f = f2;
    f.ninst = 4; f.n = n; f.H = H; f.A = A; f.ncq = ncq; f.nrb = nrb;
    for (int i = 0; i < 4; ++i) {
      const int qi = i & 1;
      const bool tgt = i >= 2;
      auto Lw = [&](int k) { return tgt ? Tq(qi, k) : Wq(qi, k); };
      FwdInst& q = f.in[i];
      q.x = tgt ? bt.xn : bt.sa; q.ldx = W; q.kx = O; q.k1 = W;
      q.w1 = Lw(0); q.b1 = Lw(1); q.w2 = Lw(2); q.b2 = Lw(3);
      q.h1 = nullptr; q.h2 = nullptr;
      q.wo = Lw(4); q.wo2 = nullptr; q.nout = 1; q.split = 1; q.opart = h->opart[4 + i];
      q.head = tgt ? 1 : 0;
      q.w1a = tgt ? nullptr : Wq(qi, 0) + (int64_t)O * H;
      q.dapart = tgt ? nullptr : h->dapart[qi];
    }
    FwdHead& hd = f.hd;
    hd.opart[0] = h->opart[0]; hd.opart[1] = h->opart[1]; hd.bm = P + o.pbm; hd.bl = P + o.pbl;
    hd.eps_in[0] = eps_in_s; hd.eps_in[1] = eps_in_n; hd.eps_out[0] = h->eps_s; hd.eps_out[1] = h->eps_n;
    hd.head_out[0] = h->out[0]; hd.head_out[1] = h->out[1]; hd.logp[0] = h->logp_s; hd.logp[1] = h->logp_n;
    hd.seed = seed; hd.iter = h->iter;
    f.st = Stamps{h->stamps, 1};
    f.sync = h->sync;
    if (h->fuse == 0) {
      hipLaunchKernelGGL(sac_fwd_kernel<true>, dim3(ncq, nrb, 4), dim3(256), 0, s, f);
      MOPO_HIP(hipGetLastError());
    }
  }
  // ---- B1: per-row TD targets and dq -> Q1/Q2(s,a) dh1; the policy's row-local backward chain; the
  //      step control; the gather of the next step's batch (with `prefetch`)
  Dh1Args b1a{};
  {
    Dh1Args& d = b1a;
    const int ncq1 = ceil_div(H, B1_COLS);
    d.n = n; d.H = H; d.A = A; d.ncq = ncq; d.ncq1 = ncq1; d.nrb = nrb;
    for (int i = 0; i < 2; ++i) {
      Dh1Inst& q = d.in[i];
      q.h1 = h->h1[2 + i]; q.h2 = h->h2[2 + i]; q.w2 = Wq(i, 2); q.w3 = Wq(i, 4); q.kind = i;
      q.dh1 = h->dh1[i]; q.dq = h->dq[i];
    }
    d.L = L;
    d.lr = h->lr; d.beta_pow = h->beta_pow; d.iter = h->iter; d.tctl = h->tctl;
    PolicyRows& pr = d.pr;
    pr.n = n; pr.O = O; pr.A = A; pr.H = H; pr.ncq = ncq;
    pr.dapart[0] = h->dapart[0]; pr.dapart[1] = h->dapart[1];
    pr.qpart[0] = h->opart[4]; pr.qpart[1] = h->opart[5];
    pr.b3[0] = Wq(0, 5); pr.b3[1] = Wq(1, 5);
    // the policy noise of pi(s): F1's draws, or the injected array itself (F2's copy of it is not handed over)
    pr.head_s = h->out[0]; pr.eps_s = eps_in_s ? eps_in_s : h->eps_s; pr.lde = eps_in_s ? A : EPW;
    pr.log_alpha = P + o.total; pr.Wm = P + o.pWm; pr.Wl = P + o.pWl;
    pr.h2p = h->h2[0]; pr.h1p = h->h1[0]; pr.W2p = P + o.pW2;
    pr.dhead = h->dhead; pr.dh2p = h->dh2p; pr.dh1p = h->dh1p; pr.prior = h->prior;
    d.gather = prefetch ? 1 : 0;
    if (prefetch) {
      d.ga = gather_args(h, 1 - par, env, mod, seed, nullptr);
      d.ga.iter_add = 1;                       // the next step's batch (the counter advances in B2)
    }
    d.st = Stamps{h->stamps, h->fuse >= 2 ? 0 : h->fuse ? 1 : 2};
    d.sync = h->sync;
    if (ncq1 * nrb < 2 && prefetch) return fail("sac: B1 needs at least one gather block");
    static_assert(B1_COLS == RB_COLS && B1_WAVES == 4, "the fused launches share the F1 / F2 grid");
    f2.st = Stamps{h->stamps, h->fuse >= 2 ? 0 : 1};
    if (h->fuse == 2) {
      hipLaunchKernelGGL(sac_f12b1_kernel, dim3(ncq, nrb, 12), dim3(256), 0, s, f1, f2, d);
    } else if (h->fuse == 1) {
      hipLaunchKernelGGL(sac_f2b1_kernel, dim3(ncq, nrb, 8), dim3(256), 0, s, f2, d);
    } else {
      hipLaunchKernelGGL(sac_dh1_kernel, dim3(ncq1, nrb, 4), dim3(B1_WAVES * 64), 0, s, d);
    }
    MOPO_HIP(hipGetLastError());
  }
  // ---- B2: every weight gradient with its fused TF1 Adam (+ Polyak for the critics), beside the batch
  //      loss tail (block 0)
  {
    WgradArgs g{};
    std::vector<WgProb> ps;
    for (int qi = 0; qi < 2; ++qi) {  // critics: dW2 = h1^T dh2 (+db2), dh2 = dq (x) W3 * (h2 > 0); dW3 = h2^T dq (+db3)
      WgProb w2 = wprob(H, H, h->h1[2 + qi], H, nullptr, H, G + o.q[qi][2], H, G + o.q[qi][3]);
      w2.bu = h->dq[qi]; w2.bv = Wq(qi, 4); w2.bm = h->h2[2 + qi]; w2.bldm = H;
      ps.push_back(w2);
      ps.push_back(wprob(H, 1, h->h2[2 + qi], H, h->dq[qi], 1, G + o.q[qi][4], 1, G + o.q[qi][5]));
    }
    for (int qi = 0; qi < 2; ++qi)    // critics: dW1 = [s,a]^T dh1 (+db1)
      ps.push_back(wprob(W, H, bt.sa, W, h->dh1[qi], H, G + o.q[qi][0], H, G + o.q[qi][1]));
    // the policy (dh2p, dh1p, dhead from the policy-row blocks of B1)
    ps.push_back(wprob(H, H, h->h1[0], H, h->dh2p, H, G + o.pW2, H, G + o.pb2));
    ps.push_back(wprob(H, A, h->h2[0], H, h->dhead, 2 * A, G + o.pWm, A, G + o.pbm));
    ps.push_back(wprob(H, A, h->h2[0], H, h->dhead + A, 2 * A, G + o.pWl, A, G + o.pbl));
    ps.push_back(wprob(O, H, bt.sa, W, h->dh1p, H, G + o.pW1, H, G + o.pb1));
    if ((int)ps.size() > WG_MAXP) return fail("sac: too many weight-gradient problems");
    for (size_t i = 0; i < ps.size(); ++i) ps[i].cls = i < 6 ? 0 : 1;   // critics' (B1 critic blocks) / the policy's
    int tot = 0;
    for (size_t i = 0; i < ps.size(); ++i) {
      g.p[i] = ps[i];
      g.prefix[i] = tot;
      tot += wgrad_tiles(ps[i].M, ps[i].N);
    }
    g.np = (int)ps.size();
    g.prefix[g.np] = tot;
    g.n = n;
    g.ad = ad;
    g.ad.slot0 = 0;
    g.L = L; g.A = A; g.ncq = ncq; g.tent = h->tent; g.logs = h->logs; g.iter = h->iter;
    g.prior = h->prior; g.eps_s = h->eps_s;
    g.sync_tmo = h->fuse ? h->sync + (SYNC_N * nrb + SYNC_TMO) * SYNC_STRIDE : nullptr;
    if (h->fuse == 2) { g.sync_reset = h->sync; g.n_sync = SYNC_N * nrb; }
    g.st = Stamps{h->stamps, 3};
    if (tot > h->nslots_cap) return fail("sac: grad-norm slots exceed the allocation");
    h->nslots = tot;
    hipLaunchKernelGGL(sac_wgrad_kernel, dim3(1 + tot), dim3(1024), 0, s, g);
    MOPO_HIP(hipGetLastError());
  }
  return 0;
}

// the tiles of the weight-gradient launch (32 x 32; one grad-norm slot each)
static int count_slots(const SacDims& d) {
  const int H = d.H, O = d.O, A = d.A, W = O + A;
  return 2 * wgrad_tiles(H, H) + 2 * wgrad_tiles(H, 1) + 2 * wgrad_tiles(W, H) + wgrad_tiles(H, H) +
         2 * wgrad_tiles(H, A) + wgrad_tiles(O, H);
}

}  // namespace mopo

using namespace mopo;

extern "C" int mopo_sac_create(mopo_sac_t* out, int O, int A, int H, int batch, int n_env, const float* h_params,
                               float log_alpha, float lr, float gamma, float tau, float reward_scale,
                               float target_entropy) {
  MOPO_REQUIRE(out && h_params, "mopo_sac_create: NULL argument");
  MOPO_REQUIRE(O >= 1 && A >= 1 && A <= 8 && H >= 1, "mopo_sac_create: bad dims (act_dim <= 8)");
  MOPO_REQUIRE(batch >= 1 && batch <= 1024, "mopo_sac_create: batch must be in [1, 1024]");
  MOPO_REQUIRE(O + A <= 31, "mopo_sac_create: obs_dim + act_dim must be <= 31 (layer-1 inputs + the bias in one 32-wide group)");
  MOPO_REQUIRE(H % 16 == 0 && H <= 256, "mopo_sac_create: hidden width must be a multiple of 16, <= 256");
  MOPO_REQUIRE(n_env >= 0 && n_env <= batch, "mopo_sac_create: n_env must be in [0, batch]");
  Sac* h = new Sac();
  h->d = SacDims{O, A, H, batch, n_env, 0};
  h->o = make_offs(O, A, H);
  h->d.P = h->o.total;
  h->lr = lr; h->gamma = gamma; h->tau = tau; h->rscale = reward_scale; h->tent = target_entropy;
  const int64_t tot = h->o.total + 1, n = batch, W = O + A;
  h->nslots_cap = h->nslots = count_slots(h->d);
  std::vector<std::pair<void**, size_t>> reg;
  auto f = [&](float** p, size_t cnt) { reg.push_back({(void**)p, cnt * 4}); };
  f(&h->Pb[1], tot); f(&h->norm_part, 2 * (size_t)h->nslots_cap);
  const int64_t ns = (n + 15) / 16 * 16;   // per-row records padded to whole row blocks (sac_rows.h rows_ns)
  const size_t npart = (size_t)ceil_div(H, RB_COLS) * ns * OPW;
  for (int i = 0; i < 8; ++i) f(&h->opart[i], npart);
  for (int i = 0; i < 2; ++i) f(&h->dapart[i], npart);
#if MOPO_SAC_STAMPS
  reg.push_back({(void**)&h->stamps, (size_t)4 * 1024 * 8 * 8});
#endif
  f(&h->P, tot); f(&h->G, tot); f(&h->M, tot); f(&h->V, tot); f(&h->T, tot);
  f(&h->beta_pow, 4); f(&h->logs, LOG_N);
  reg.push_back({(void**)&h->iter, 8});
  reg.push_back({(void**)&h->tctl, 3 * 8});
  for (int b = 0; b < 2; ++b) {
    Batch& t = h->bt[b];
    f(&t.sa, n * W); f(&t.xpi, n * W); f(&t.xn, n * W); f(&t.rew, n); f(&t.term, n);
    reg.push_back({(void**)&t.idx, (size_t)n * 8});
  }
  for (int i = 0; i < 8; ++i) { f(&h->h1[i], n * H); f(&h->h2[i], n * H); f(&h->out[i], n * 2 * A); }
  f(&h->logp_s, 2 * ns); f(&h->logp_n, 2 * ns); f(&h->eps_s, ns * EPW); f(&h->eps_n, ns * EPW);
  reg.push_back({(void**)&h->sync, (size_t)(SYNC_N * (ns / 16) + SYNC_GLOBAL) * SYNC_STRIDE * 4});
  h->fuse = sac_fuse_default();
  for (int i = 0; i < 4; ++i) { f(&h->dq[i], n); f(&h->dh1[i], n * H); }
  f(&h->dhead, n * 2 * A); f(&h->dh2p, n * H); f(&h->dh1p, n * H);
  size_t total = 0;
  for (auto& r : reg) total += (r.second + 255) & ~(size_t)255;
  if (hipMalloc(&h->mem, total) != hipSuccess) { delete h; return fail("mopo_sac_create: out of device memory"); }
  if (hipMemset(h->mem, 0, total) != hipSuccess) { (void)hipFree(h->mem); delete h; return fail("mopo_sac_create: memset"); }
  char* m = (char*)h->mem;
  for (auto& r : reg) { *r.first = m; m += (r.second + 255) & ~(size_t)255; }
  // parameters, target = main (target_init, mopo.py:449-450), log_alpha, beta powers
  std::vector<float> pv(h_params, h_params + h->o.total);
  pv.push_back(log_alpha);
  h->Pb[0] = h->P;
  MOPO_HIP(hipMemcpy(h->P, pv.data(), tot * 4, hipMemcpyHostToDevice));
  MOPO_HIP(hipMemcpy(h->Pb[1], pv.data(), tot * 4, hipMemcpyHostToDevice));
  MOPO_HIP(hipMemcpy(h->T, pv.data(), tot * 4, hipMemcpyHostToDevice));
  float bp[2] = {0.9f, 0.999f};
  MOPO_HIP(hipMemcpy(h->beta_pow, bp, 8, hipMemcpyHostToDevice));
  const int64_t tc[3] = {0, 1, 1};   // target_update_interval = 1: every step
  MOPO_HIP(hipMemcpy(h->tctl, tc, sizeof(tc), hipMemcpyHostToDevice));
  *out = reinterpret_cast<mopo_sac_t>(h);
  return 0;
}

static void drop_graphs(Sac* h) {
  for (int i = 0; i < 3; ++i) {
    if (h->gexec[i]) (void)hipGraphExecDestroy(h->gexec[i]);
    if (h->graph[i]) (void)hipGraphDestroy(h->graph[i]);
    h->gexec[i] = nullptr;
    h->graph[i] = nullptr;
  }
}

extern "C" int mopo_sac_destroy(mopo_sac_t hh) {
  Sac* h = reinterpret_cast<Sac*>(hh);
  if (!h) return 0;
  drop_graphs(h);
  if (h->ev_in) (void)hipEventDestroy(h->ev_in);
  if (h->ev_out) (void)hipEventDestroy(h->ev_out);
  if (h->gstream) (void)hipStreamDestroy(h->gstream);
  if (h->mem) (void)hipFree(h->mem);
  delete h;
  return 0;
}

extern "C" int mopo_sac_buffers(mopo_sac_t hh, float** params, float** target, float** adam_m, float** adam_v,
                                float** grads, float** logs, int64_t* n_params) {
  Sac* h = reinterpret_cast<Sac*>(hh);
  MOPO_REQUIRE(h, "mopo_sac_buffers: NULL handle");
  if (params) *params = h->P;
  if (target) *target = h->T;
  if (adam_m) *adam_m = h->M;
  if (adam_v) *adam_v = h->V;
  if (grads) *grads = h->G;
  if (logs) *logs = h->logs;
  if (n_params) *n_params = h->o.total;
  return 0;
}

extern "C" int mopo_sac_copy(mopo_sac_t hh, int which, int to_handle, void* d_buf, int64_t count, void* stream) {
  Sac* h = reinterpret_cast<Sac*>(hh);
  MOPO_REQUIRE(h && d_buf, "mopo_sac_copy: NULL argument");
  float* bufs[6] = {h->P, h->T, h->M, h->V, h->G, h->logs};
  MOPO_REQUIRE(which >= 0 && which < 6, "mopo_sac_copy: which must be in [0, 6)");
  const int64_t cap = which == 5 ? LOG_N : h->o.total + 1;
  MOPO_REQUIRE(count >= 0 && count <= cap, "mopo_sac_copy: count exceeds the buffer");
  if (to_handle)
    MOPO_HIP(hipMemcpyAsync(bufs[which], d_buf, count * 4, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  else
    MOPO_HIP(hipMemcpyAsync(d_buf, bufs[which], count * 4, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return 0;
}

extern "C" int mopo_sac_set_graph(mopo_sac_t hh, int enable) {
  Sac* h = reinterpret_cast<Sac*>(hh);
  MOPO_REQUIRE(h, "mopo_sac_set_graph: NULL handle");
  h->use_graph = enable != 0;
  return 0;
}

extern "C" int mopo_sac_check(mopo_sac_t hh, int* timed_out) {
  Sac* h = reinterpret_cast<Sac*>(hh);
  MOPO_REQUIRE(h && timed_out, "mopo_sac_check: NULL argument");
  MOPO_HIP(hipDeviceSynchronize());
  unsigned* w = h->sync + (SYNC_N * ceil_div(h->d.n, 16) + SYNC_TMO) * SYNC_STRIDE;
  unsigned v = 0;
  MOPO_HIP(hipMemcpy(&v, w, 4, hipMemcpyDeviceToHost));
  *timed_out = v != 0;
  if (v) {
    MOPO_HIP(hipMemset(w, 0, 4));
    MOPO_HIP(hipDeviceSynchronize());
    return fail("sac: an in-launch hand-off wait of the fused step timed out; the parameter, Adam and target "
                "updates of the steps since then were held (not applied) and their logs are NaN");
  }
  return 0;
}

extern "C" int mopo_sac_inject_timeout(mopo_sac_t hh) {
  Sac* h = reinterpret_cast<Sac*>(hh);
  MOPO_REQUIRE(h, "mopo_sac_inject_timeout: NULL handle");
  MOPO_HIP(hipDeviceSynchronize());
  const unsigned one = 1;
  MOPO_HIP(hipMemcpy(h->sync + (SYNC_N * ceil_div(h->d.n, 16) + SYNC_TMO) * SYNC_STRIDE, &one, 4, hipMemcpyHostToDevice));
  return 0;
}

static int launch_logs(Sac* h, hipStream_t s) {
  hipLaunchKernelGGL(sac_logs_kernel, dim3(1), dim3(256), 0, s, h->norm_part, h->nslots, h->logs);
  MOPO_HIP(hipGetLastError());
  return 0;
}

static bool same_desc(const mopo_pool_desc& a, const mopo_pool_desc& b) { return std::memcmp(&a, &b, sizeof(a)) == 0; }

// Steps alternate parameter buffers (parity 0 reads Pb[0] and writes Pb[1], parity 1 the
// reverse); a call ends with the parameters back in Pb[0] (one copy after an odd step count).
static int copy_back(Sac* h, hipStream_t s) {
  MOPO_HIP(hipMemcpyAsync(h->Pb[0], h->Pb[1], (h->o.total + 1) * 4, hipMemcpyDeviceToDevice, s));
  return 0;
}

#ifndef MOPO_SAC_GRAPH_STEPS
#define MOPO_SAC_GRAPH_STEPS 8
#endif
// steps per replay of the long graph (amortises the launch gap); 32 measured the same as 8 (same-box
// A/B 69.7 us/step both): the graph replay is not on the step's critical path
constexpr int GRAPH_STEPS = MOPO_SAC_GRAPH_STEPS;
// every captured graph starts at parity 0 and must end having written Pb[0] and prefetched bt[0]
static_assert(GRAPH_STEPS >= 2 && GRAPH_STEPS % 2 == 0, "MOPO_SAC_GRAPH_STEPS must be even and >= 2");

// which = 0: GRAPH_STEPS steps, 1: two steps (parity 0, 1), 2: one step + copy back.  Every step
// prefetches the other parity's batch, so a graph's last step prepares the next graph's first.
static int capture(Sac* h, int which, const mopo_pool_desc* env, const mopo_pool_desc* mod, uint64_t seed) {
  hipStream_t gs = h->gstream;
  MOPO_HIP(hipStreamBeginCapture(gs, hipStreamCaptureModeThreadLocal));
  const int steps = which == 0 ? GRAPH_STEPS : which == 1 ? 2 : 1;
  int rc = 0;
  for (int i = 0; i < steps && !rc; ++i) rc = sac_step_impl(h, i & 1, env, mod, seed, nullptr, nullptr, gs, true);
  if (!rc && which == 2) rc = copy_back(h, gs);
  hipGraph_t g = nullptr;
  const hipError_t e = hipStreamEndCapture(gs, &g);
  if (rc) { if (g) (void)hipGraphDestroy(g); return -1; }
  if (e != hipSuccess) return fail(std::string("mopo_sac_step: capture failed: ") + hipGetErrorString(e));
  h->graph[which] = g;
  MOPO_HIP(hipGraphInstantiate(&h->gexec[which], g, nullptr, nullptr, 0));
  return 0;
}

extern "C" int mopo_sac_step(mopo_sac_t hh, const mopo_pool_desc* env, const mopo_pool_desc* mod, int n_steps,
                             uint64_t seed, const int64_t* d_idx, const float* d_eps_s, const float* d_eps_n,
                             void* stream) {
  Sac* h = reinterpret_cast<Sac*>(hh);
  MOPO_REQUIRE(h && env && mod, "mopo_sac_step: NULL argument");
  MOPO_REQUIRE(env->d_state && mod->d_state, "mopo_sac_step: pool state required");
  MOPO_REQUIRE(n_steps >= 0, "mopo_sac_step: n_steps must be >= 0");
  if (n_steps == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const bool injected = d_idx || d_eps_s || d_eps_n;
  if (injected) {
    MOPO_REQUIRE(n_steps == 1, "mopo_sac_step: injected streams drive exactly one step");
    if (launch_gather(h, 0, env, mod, seed, d_idx, s) ||
        sac_step_impl(h, 0, env, mod, seed, d_eps_s, d_eps_n, s, false) || copy_back(h, s))
      return -1;
    return launch_logs(h, s);
  }
  if (!h->use_graph) {
    if (launch_gather(h, 0, env, mod, seed, nullptr, s)) return -1;
    for (int i = 0; i < n_steps; ++i)
      if (sac_step_impl(h, i & 1, env, mod, seed, nullptr, nullptr, s, true)) return -1;
    if ((n_steps & 1) && copy_back(h, s)) return -1;
    return launch_logs(h, s);
  }
  // graphs are captured and replayed on the handle's own stream (the caller's may be the legacy
  // NULL stream, which cannot capture); event edges order it after / before the caller's work.
  // gexec[0] = GRAPH_STEPS steps, gexec[1] = two, gexec[2] = one step + copy back.
  if (!h->gstream) {
    MOPO_HIP(hipStreamCreateWithFlags(&h->gstream, hipStreamNonBlocking));
    MOPO_HIP(hipEventCreateWithFlags(&h->ev_in, hipEventDisableTiming));
    MOPO_HIP(hipEventCreateWithFlags(&h->ev_out, hipEventDisableTiming));
  }
  hipStream_t gs = h->gstream;
  if (!h->gexec[0] || !same_desc(h->genv, *env) || !same_desc(h->gmod, *mod) || h->gseed != seed) {
    drop_graphs(h);
    if (capture(h, 0, env, mod, seed) || capture(h, 1, env, mod, seed) || capture(h, 2, env, mod, seed)) return -1;
    h->genv = *env; h->gmod = *mod; h->gseed = seed;
  }
  MOPO_HIP(hipEventRecord(h->ev_in, s));
  MOPO_HIP(hipStreamWaitEvent(gs, h->ev_in, 0));
  if (launch_gather(h, 0, env, mod, seed, nullptr, gs)) return -1;  // first step's batch
  int i = 0;
  for (; i + GRAPH_STEPS <= n_steps; i += GRAPH_STEPS) MOPO_HIP(hipGraphLaunch(h->gexec[0], gs));
  for (; i + 2 <= n_steps; i += 2) MOPO_HIP(hipGraphLaunch(h->gexec[1], gs));
  if (i < n_steps) MOPO_HIP(hipGraphLaunch(h->gexec[2], gs));
  if (launch_logs(h, gs)) return -1;
  MOPO_HIP(hipEventRecord(h->ev_out, gs));
  MOPO_HIP(hipStreamWaitEvent(s, h->ev_out, 0));
  return 0;
}

namespace mopo {
__global__ void sac_set_tctl_kernel(int64_t* tctl, int64_t base, int64_t repeat, int64_t interval) {
  tctl[0] = base; tctl[1] = repeat; tctl[2] = interval;
}
}  // namespace mopo

extern "C" int mopo_sac_set_target_schedule(mopo_sac_t hh, int64_t base, int64_t n_train_repeat, int64_t interval,
                                            void* stream) {
  Sac* h = reinterpret_cast<Sac*>(hh);
  MOPO_REQUIRE(h, "mopo_sac_set_target_schedule: NULL handle");
  MOPO_REQUIRE(n_train_repeat >= 1 && interval >= 1, "mopo_sac_set_target_schedule: repeat and interval must be >= 1");
  // a launch (not a copy from host memory) so it orders with the caller's stream and with graph replays
  hipLaunchKernelGGL(sac_set_tctl_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, h->tctl, base, n_train_repeat,
                     interval);
  MOPO_HIP(hipGetLastError());
  return 0;
}

extern "C" int mopo_sac_set_action_prior(mopo_sac_t hh, int normal) {
  Sac* h = reinterpret_cast<Sac*>(hh);
  MOPO_REQUIRE(h, "mopo_sac_set_action_prior: NULL handle");
  MOPO_REQUIRE(normal == 0 || normal == 1, "mopo_sac_set_action_prior: 0 (uniform) or 1 (normal)");
  if (h->prior != normal) drop_graphs(h);   // the flag is a kernel argument of the captured steps
  h->prior = normal;
  return 0;
}

extern "C" int mopo_sac_debug_stamps(mopo_sac_t hh, uint64_t* h_out, int64_t n) {
  Sac* h = reinterpret_cast<Sac*>(hh);
  MOPO_REQUIRE(h && h_out, "mopo_sac_debug_stamps: NULL argument");
  if (!h->stamps) return fail("mopo_sac_debug_stamps: library built without MOPO_SAC_STAMPS");
  MOPO_REQUIRE(n >= 0 && n <= 4 * 1024 * 8, "mopo_sac_debug_stamps: n exceeds the stamp buffer");
  MOPO_HIP(hipDeviceSynchronize());
  MOPO_HIP(hipMemcpy(h_out, h->stamps, n * 8, hipMemcpyDeviceToHost));
  return 0;
}
