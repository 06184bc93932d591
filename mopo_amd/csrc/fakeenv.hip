// FakeEnv.step post-processing on the device (general / API path).
//
// Replaces the numpy half of FakeEnv.step (mopo/models/fake_env.py:37-131) and
// _get_logprob (fake_env.py:20-35), with the termination functions of mopo/static.
// One thread per row; reads the ensemble mean/var [E,B,D] written by the BNN forward.
// dtype rules follow the reference: means stay f32 after the in-place residual add
// (fake_env.py:66), the noisy sample is f64 (fake_env.py:72), penalty is an f32 norm.
#include "internal.h"

namespace mopo {

constexpr int MAXD = 32;

// Every per-row quantity is re-read from the (L1/L2-resident) inputs where it is used instead of being
// held in per-thread arrays indexed by the runtime D: such arrays live in scratch (528 B per lane).
__global__ __launch_bounds__(256) void fakeenv_post_kernel(const mopo_fakeenv_args a, int E, int O, int A) {
  const int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (b >= a.B) return;
  const int D = O + 1;
  const int64_t B = a.B;
  auto obs_at = [&](int d) -> double {
    return a.obs_f64 ? reinterpret_cast<const double*>(a.d_obs)[b * O + d]
                     : (double)reinterpret_cast<const float*>(a.d_obs)[b * O + d];
  };
  auto mean_at = [&](int e, int d) -> float {  // fake_env.py:66 (f64 add, stored back to f32)
    float m = a.d_ens_mean[((int64_t)e * B + b) * D + d];
    return d >= 1 ? (float)((double)m + obs_at(d - 1)) : m;
  };
  auto var_at = [&](int e, int d) -> float { return a.d_ens_var[((int64_t)e * B + b) * D + d]; };
  const int sel = a.deterministic ? 0 : (int)a.d_model_inds[b];  // bnn.py:343 / fake_env.py:77-81
  // the selected mean / std (fake_env.py:77-81) or, deterministic, the plain f32 member means (:69-70, 84-86)
  auto mmean_at = [&](int d) -> float {
    if (!a.deterministic) return mean_at(sel, d);
    float sm = 0.f;
    for (int e = 0; e < E; ++e) sm += mean_at(e, d);
    return sm / (float)E;
  };
  auto mstd_at = [&](int d) -> float {
    if (!a.deterministic) return sqrtf(var_at(sel, d));
    float ss = 0.f;
    for (int e = 0; e < E; ++e) ss += sqrtf(var_at(e, d));
    return ss / (float)E;
  };
  auto sample_at = [&](int d) -> double {  // fake_env.py:72 (f64); deterministic: the mean
    if (a.deterministic) return (double)mmean_at(d);
    return (double)mean_at(sel, d) + a.d_noise_sel[b * D + d] * (double)sqrtf(var_at(sel, d));
  };
  // _get_logprob (fake_env.py:20-35): log-sum-exp over ALL members, naive exp then log
  if (a.d_log_prob || a.d_dev) {
    double prob = 0.0;
    const double k_log2pi = (double)D * log(2.0 * M_PI);
    for (int e = 0; e < E; ++e) {
      double slv = 0.0, sq = 0.0;
      for (int d = 0; d < D; ++d) {
        float v = var_at(e, d);
        slv += (double)logf(v);
        double df = sample_at(d) - (double)mean_at(e, d);
        sq += df * df / (double)v;
      }
      prob += exp(-0.5 * (k_log2pi + slv + sq));
    }
    if (a.d_log_prob) a.d_log_prob[b] = log(prob);
    if (a.d_dev) {  // np.std(means, 0).mean(-1) in f32
      float acc = 0.f;
      for (int d = 0; d < D; ++d) {
        float mu = 0.f;
        for (int e = 0; e < E; ++e) mu += mean_at(e, d);
        mu /= (float)E;
        float v = 0.f;
        for (int e = 0; e < E; ++e) {
          float df = mean_at(e, d) - mu;
          v += df * df;
        }
        acc += sqrtf(v / (float)E);
      }
      a.d_dev[b] = acc / (float)D;
    }
  }
  // termination on the f64 next_obs (fake_env.py:90-91)
  const bool term = term_fn_at(a.term_kind, [&](int d) { return sample_at(d + 1); }, O);
  // penalty (fake_env.py:97-115)
  float pen = 0.f;
  if (a.penalty_coeff != 0.f) {
    if (a.penalty_learned_var) {
      for (int e = 0; e < E; ++e) {
        float s2 = 0.f;
        for (int d = 0; d < D; ++d) {
          float s = sqrtf(var_at(e, d));
          s2 += s * s;
        }
        pen = fmaxf(pen, sqrtf(s2));
      }
    } else {  // max over members of || mean_e - mean over members || over the obs dims
      for (int e = 0; e < E; ++e) {
        float s2 = 0.f;
        for (int d = 1; d < D; ++d) {
          float sm = 0.f;
          for (int f = 0; f < E; ++f) sm += mean_at(f, d);
          const float df = mean_at(e, d) - sm / (float)E;
          s2 += df * df;
        }
        pen = fmaxf(pen, sqrtf(s2));
      }
    }
  }
  const double rew = sample_at(0);
  const double pen_rew = a.penalty_coeff != 0.f ? rew - (double)a.penalty_coeff * (double)pen : rew;
  for (int d = 0; d < O; ++d) a.d_next_obs[b * O + d] = sample_at(d + 1);
  a.d_rewards[b] = pen_rew;
  a.d_terminals[b] = term ? 1 : 0;
  if (a.d_penalty) a.d_penalty[b] = pen;
  if (a.d_unpenalized) a.d_unpenalized[b] = rew;
  if (a.d_info_mean) {  // fake_env.py:94-95
    float* im = a.d_info_mean + b * (D + 1);
    float* is = a.d_info_std + b * (D + 1);
    im[0] = mmean_at(0); im[1] = term ? 1.f : 0.f;
    is[0] = mstd_at(0); is[1] = 0.f;
    for (int d = 1; d < D; ++d) { im[d + 1] = mmean_at(d); is[d + 1] = mstd_at(d); }
  }
  (void)A;
}

}  // namespace mopo

using namespace mopo;

extern "C" int mopo_fakeenv_step(mopo_bnn_t hh, const mopo_fakeenv_args* a, void* stream) {
  Bnn* h = reinterpret_cast<Bnn*>(hh);
  MOPO_REQUIRE(h && a, "mopo_fakeenv_step: NULL argument");
  MOPO_REQUIRE(h->O + 1 <= MAXD, "mopo_fakeenv_step: obs_dim too large");
  MOPO_REQUIRE(a->B >= 0, "mopo_fakeenv_step: negative batch");
  MOPO_REQUIRE(a->term_kind >= 0 && a->term_kind < MOPO_TERM_KINDS, "mopo_fakeenv_step: unknown term_kind");
  if (a->B == 0) return 0;  // empty batch: nothing to read or write (empty buffers may be NULL)
  MOPO_REQUIRE(a->d_ens_mean && a->d_ens_var, "mopo_fakeenv_step: ensemble workspaces required");
  MOPO_REQUIRE(a->deterministic || (a->d_noise_sel && a->d_model_inds),
               "mopo_fakeenv_step: noise and model_inds required unless deterministic");
  MOPO_REQUIRE(a->d_next_obs && a->d_rewards && a->d_terminals, "mopo_fakeenv_step: NULL output");
  // the post kernel re-reads a row's obs (info_mean / info_std) after storing its next_obs
  MOPO_REQUIRE((const void*)a->d_next_obs != a->d_obs, "mopo_fakeenv_step: d_next_obs must not alias d_obs");
  MOPO_REQUIRE(!a->d_info_mean == !a->d_info_std, "mopo_fakeenv_step: info_mean/info_std go together");
  hipStream_t s = (hipStream_t)stream;
  FwdArgs f{};
  const size_t es = a->obs_f64 ? 8 : 4;
  (void)es;
  f.in = FwdIn{a->d_obs, a->obs_f64, h->O, a->d_act, 0, h->A};
  f.B = a->B;
  f.mean = a->d_ens_mean;
  f.var = a->d_ens_var;
  if (launch_bnn_fwd(h, FWD_PREDICT, f, s)) return -1;
  hipLaunchKernelGGL(fakeenv_post_kernel, dim3(ceil_div((int)a->B, 256)), dim3(256), 0, s, *a, h->E, h->O,
                     h->A);
  MOPO_HIP(hipGetLastError());
  return 0;
}
