// Internal declarations shared by the libmopo_hip translation units.
#pragma once
#include "common.h"
#include "../../include/mopo_hip.h"

namespace mopo {

constexpr int MAX_IN_KG = 4;  // layer-0 input features <= 64

// Device view of a packed ensemble.  Weight matrices are stored "fragment-major": for
// layer input K (KG = ceil(K/16) k-groups) and output N (NB = ceil(N/16) blocks), member e,
// fragment (kg, nb) is 64 lanes x 4 floats contiguous (1 KiB):
//   frag[((e*KG + kg)*NB + nb)*256 + lane*4 + t] = W[e][kg*16 + 4*(lane>>4) + t][nb*16 + (lane&15)]
// i.e. exactly the per-lane A operand of 4 consecutive v_mfma_f32_16x16x4_f32 steps.
struct BnnDev {
  int E, O, A, IN, H, D;
  int KG0, NBH, NBO;  // layer-0 k-groups, hidden blocks (= hidden k-groups), head blocks
  const float* w0;    // [E][KG0][NBH] frags
  const float* wh;    // [3][E][NBH][NBH] frags
  const float* whd;   // [E][NBH][NBO] frags (head: n < D mean, D <= n < 2D log-var)
  const float* b0;    // [E][NBH*16]
  const float* bh;    // [3][E][NBH*16]
  const float* bhd;   // [E][NBO*16]
  const float* mu;    // [IN]
  const float* sigma; // [IN]
  const float* maxlv; // [D]
  const float* minlv; // [D]
  int BS;             // per-member bias stride (floats): even(NBH) * 16
  // bf16 fragments (dtype 1..3): 1 KiB = 64 lanes x 8 bf16 per (32-deep k-group, 16-wide block),
  // addressed in float units like the f32 fragments; hidden width padded to NB2 = even(NBH)
  int NB2;
  const float* w0b;   // [E][1][NB2]
  const float* whb;   // [3][E][NB2/2][NB2]
  const float* whdb;  // [E][NB2/2][NBO]
  const float* wscale;  // f16x3: [5][E] inverse power-of-two weight scales (layer 0, hidden 1..3, head)
};

enum { DT_FP32 = 0, DT_BF16 = 1, DT_BF16X3 = 2, DT_BF16X6 = 3, DT_F16X3 = 4 };
// 16-bit parts per operand of a dtype (1 bf16, 2 bf16x3, 3 bf16x6, 2 f16x3; mlp_tile.h split_*)
__host__ __device__ constexpr int bf16_parts(int dtype) { return dtype < 1 ? 1 : (dtype == DT_F16X3 ? 2 : dtype); }

struct Bnn {
  int E, O, A, H, smv, dtype;
  bool has_params = false;
  float* buf = nullptr;      // one device allocation for all packed params
  uint16_t* bbuf = nullptr;  // bf16 packed weights
  int64_t buf_bytes = 0, bbuf_bytes = 0;  // sizes of buf / bbuf (mopo_bnn_packed_copy)
  BnnDev dev{};
};

// Input view: features [0, O) from xa (row stride sa), [O, IN) from xb (row stride sb).
struct FwdIn {
  const void* xa; int xa_f64; int64_t sa;
  const void* xb; int xb_f64; int64_t sb;
};

enum { FWD_PREDICT = 0, FWD_ROLLOUT = 1 };
constexpr int XS_STRIDE = 32;  // floats per pre-scaled input row (FwdArgs::xs): 2 k-groups of slots

struct FwdArgs {
  FwdIn in;
  int64_t B;              // launch rows (grid sized for this)
  const int* d_count;     // optional device row count (<= B)
  // optional pre-scaled input rows [B][32] f32 in slot_feat order (written once per row by the
  // rollout's actor): replaces the per-member f64 obs / act loads and scaler transform
  const float* xs;
  int ntiles;             // tiles per member in the grid
  int xcd_members;        // H = 400 f16x3 kernel: 1 = every XCD owns E / 8 members (set by launch_f16s)
  // predict outputs
  float* mean;            // [E][B][D]
  float* var;
  // rollout outputs
  uint32_t* pen_bits;     // [B] max_e ||std_e|| (as ordered uint bits)
  const int32_t* sel;     // [B] selected member per row
  float* mean_sel;        // [B][D]
  float* std_sel;         // [B][D]
  // rollout, optional: every member's mean / std (mean-distance penalty and deterministic mode,
  // fake_env.py:84-86, 98-108): [E][all_stride][D], row r of this launch at all_stride rows apart
  float* mean_all;
  float* std_all;
  int64_t all_stride;
};

int launch_bnn_fwd(const Bnn* h, int mode, const FwdArgs& a, hipStream_t s);
// W[E][K][N] (TF layout) -> fragment-major (see BnnDev) on stream s
// perm_k: the K side is an input width in slot_feat order (mlp_tile.h)
int pack_frags(const float* src, float* dst, int E, int K, int N, int KG, int NB, hipStream_t s, int perm_k = 0);

// termination kinds (mopo/static)
// nobs: next_obs[d] for d < O -- an array or any accessor callable with d
template <class F>
__device__ __forceinline__ bool term_fn_at(int kind, const F& nobs, int O) {
  if (kind == MOPO_TERM_WALKER2D) {  // walker2d.py:10-16
    double hh = nobs(0), an = nobs(1);
    bool not_done = (hh > 0.8) && (hh < 2.0) && (an > -1.0) && (an < 1.0);
    return !not_done;
  }
  if (kind == MOPO_TERM_HOPPER) {  // hopper.py:10-17 (np.abs(bool) == bool)
    bool fin = true, small = true;
    for (int d = 0; d < O; ++d) {
      double v = nobs(d);
      fin = fin && isfinite(v);
      if (d >= 1) small = small && (v < 100.0);
    }
    double hh = nobs(0), an = nobs(1);
    bool not_done = fin && small && (hh > 0.7) && (fabs(an) < 0.2);
    return !not_done;
  }
  if (kind == MOPO_TERM_ANT) {  // ant.py:9-15, antangle.py:9-15
    bool fin = true;
    for (int d = 0; d < O; ++d) fin = fin && isfinite(nobs(d));
    double x = nobs(0);
    bool not_done = fin && (x >= 0.2) && (x <= 1.0);
    return !not_done;
  }
  if (kind == MOPO_TERM_HUMANOID) {  // humanoid.py:10-11 (NaN compares false: not done)
    double z = nobs(0);
    return (z < 1.0) || (z > 2.0);
  }
  return false;  // halfcheetah.py:9-10 and the other never-done domains
}

__device__ __forceinline__ bool term_fn(int kind, const double* nobs, int O) {
  return term_fn_at(kind, [&](int d) { return nobs[d]; }, O);
}

}  // namespace mopo
