// Cost attribution for the ensemble forward (rollout mode, halfcheetah shape E=7 H=200, B=50000):
// the same kernel built with one part disabled (-DBNN_KNOB_* in bnn.hip/mlp_tile.h; timing only,
// results are garbage).  Build: scripts/micro/build_bnn_knobs.sh
#include "../../mopo_amd/csrc/bnn.hip"
#include <cstdio>
#include <random>

using namespace mopo;

int main(int argc, char** argv) {
#ifndef KNOB_E
#define KNOB_E 7
#endif
#ifndef KNOB_H
#define KNOB_H 200
#endif
  const int E = KNOB_E, O = 17, A = 6, H = KNOB_H, D = O + 1, IN = O + A;
  const int64_t B = argc > 1 ? atoll(argv[1]) : 50000;
  mopo_bnn_t hb;
#ifndef KNOB_DTYPE
#define KNOB_DTYPE 0
#endif
  if (mopo_bnn_create(&hb, E, O, A, H, 0, KNOB_DTYPE)) { printf("create: %s\n", mopo_last_error()); return 1; }
  std::mt19937 rng(1);
  std::normal_distribution<float> nd(0.f, 1.f);
  auto arr = [&](size_t n, float sc) { std::vector<float> v(n); for (auto& x : v) x = nd(rng) * sc; return v; };
  std::vector<std::vector<float>> a;
  a.push_back(arr(IN, 0.1f)); a.push_back(std::vector<float>(IN, 1.f));
  int dims[6] = {IN, H, H, H, H, 2 * D};
  for (int l = 0; l < 5; ++l) { a.push_back(arr((size_t)E * dims[l] * dims[l + 1], 1.f / sqrtf(dims[l]))); a.push_back(arr((size_t)E * dims[l + 1], 0.1f)); }
  a.push_back(std::vector<float>(D, 0.5f)); a.push_back(std::vector<float>(D, -10.f));
  std::vector<const float*> ptrs; for (auto& v : a) ptrs.push_back(v.data());
  if (mopo_bnn_set_params(hb, ptrs.data(), (int)ptrs.size())) { printf("set: %s\n", mopo_last_error()); return 1; }
  Bnn* h = reinterpret_cast<Bnn*>(hb);
  double* obs; float* act; uint32_t* pen; int32_t* sel; float *ms, *ss;
  (void)hipMalloc(&obs, B * O * 8); (void)hipMalloc(&act, B * A * 4); (void)hipMalloc(&pen, B * 4);
  (void)hipMalloc(&sel, B * 4); (void)hipMalloc(&ms, B * D * 4); (void)hipMalloc(&ss, B * D * 4);
  (void)hipMemset(obs, 0, B * O * 8); (void)hipMemset(act, 0, B * A * 4); (void)hipMemset(sel, 0, B * 4);
  FwdArgs f{};
  f.in = FwdIn{obs, 1, O, act, 0, A};
  f.B = B; f.pen_bits = pen; f.sel = sel; f.mean_sel = ms; f.std_sel = ss;
  hipStream_t s; (void)hipStreamCreate(&s);
  for (int i = 0; i < 5; ++i) launch_bnn_fwd(h, FWD_ROLLOUT, f, s);
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, s);
  const int reps = 30;
  for (int i = 0; i < reps; ++i) launch_bnn_fwd(h, FWD_ROLLOUT, f, s);
  (void)hipEventRecord(e1, s);
  (void)hipEventSynchronize(e1);
  float ms_; (void)hipEventElapsedTime(&ms_, e0, e1);
  const double t = ms_ / reps;
  const double flop = (double)B * 2 * E * ((double)IN * H + 3.0 * H * H + 2.0 * H * D);
  printf("%-12s B=%lld %.4f ms  %.1f TF/s\n", KNOB_NAME, (long long)B, t, flop / (t * 1e-3) / 1e12);
  return 0;
}
