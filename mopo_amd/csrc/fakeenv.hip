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

__global__ __launch_bounds__(256) void fakeenv_post_kernel(const mopo_fakeenv_args a, int E, int O, int A) {
  const int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (b >= a.B) return;
  const int D = O + 1;
  const int64_t B = a.B;
  double obs[MAXD];
  for (int d = 0; d < O; ++d)
    obs[d] = a.obs_f64 ? reinterpret_cast<const double*>(a.d_obs)[b * O + d]
                       : (double)reinterpret_cast<const float*>(a.d_obs)[b * O + d];
  auto mean_at = [&](int e, int d) -> float {  // fake_env.py:66 (f64 add, stored back to f32)
    float m = a.d_ens_mean[((int64_t)e * B + b) * D + d];
    return d >= 1 ? (float)((double)m + obs[d - 1]) : m;
  };
  double sample[MAXD];
  float mmean[MAXD], mstd[MAXD];
  if (!a.deterministic) {
    const int sel = (int)a.d_model_inds[b];  // bnn.py:343 / fake_env.py:77-81
    for (int d = 0; d < D; ++d) {
      float m = mean_at(sel, d);
      float s = sqrtf(a.d_ens_var[((int64_t)sel * B + b) * D + d]);
      mmean[d] = m;
      mstd[d] = s;
      sample[d] = (double)m + a.d_noise_sel[b * D + d] * (double)s;  // fake_env.py:72 (f64)
    }
  } else {  // fake_env.py:69-70, 84-86: plain f32 means over all members
    for (int d = 0; d < D; ++d) {
      float sm = 0.f, ss = 0.f;
      for (int e = 0; e < E; ++e) {
        sm += mean_at(e, d);
        ss += sqrtf(a.d_ens_var[((int64_t)e * B + b) * D + d]);
      }
      mmean[d] = sm / (float)E;
      mstd[d] = ss / (float)E;
      sample[d] = (double)mmean[d];
    }
  }
  // _get_logprob (fake_env.py:20-35): log-sum-exp over ALL members, naive exp then log
  if (a.d_log_prob || a.d_dev) {
    double prob = 0.0;
    const double k_log2pi = (double)D * log(2.0 * M_PI);
    for (int e = 0; e < E; ++e) {
      double slv = 0.0, sq = 0.0;
      for (int d = 0; d < D; ++d) {
        float v = a.d_ens_var[((int64_t)e * B + b) * D + d];
        slv += (double)logf(v);
        double df = sample[d] - (double)mean_at(e, d);
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
  const bool term = term_fn(a.term_kind, sample + 1, O);
  // penalty (fake_env.py:97-115)
  float pen = 0.f;
  if (a.penalty_coeff != 0.f) {
    if (a.penalty_learned_var) {
      for (int e = 0; e < E; ++e) {
        float s2 = 0.f;
        for (int d = 0; d < D; ++d) {
          float s = sqrtf(a.d_ens_var[((int64_t)e * B + b) * D + d]);
          s2 += s * s;
        }
        pen = fmaxf(pen, sqrtf(s2));
      }
    } else {
      float mu[MAXD];
      for (int d = 1; d < D; ++d) {
        float sm = 0.f;
        for (int e = 0; e < E; ++e) sm += mean_at(e, d);
        mu[d] = sm / (float)E;
      }
      for (int e = 0; e < E; ++e) {
        float s2 = 0.f;
        for (int d = 1; d < D; ++d) {
          float df = mean_at(e, d) - mu[d];
          s2 += df * df;
        }
        pen = fmaxf(pen, sqrtf(s2));
      }
    }
  }
  const double rew = sample[0];
  const double pen_rew = a.penalty_coeff != 0.f ? rew - (double)a.penalty_coeff * (double)pen : rew;
  for (int d = 0; d < O; ++d) a.d_next_obs[b * O + d] = sample[d + 1];
  a.d_rewards[b] = pen_rew;
  a.d_terminals[b] = term ? 1 : 0;
  if (a.d_penalty) a.d_penalty[b] = pen;
  if (a.d_unpenalized) a.d_unpenalized[b] = rew;
  if (a.d_info_mean) {  // fake_env.py:94-95
    float* im = a.d_info_mean + b * (D + 1);
    float* is = a.d_info_std + b * (D + 1);
    im[0] = mmean[0]; im[1] = term ? 1.f : 0.f;
    is[0] = mstd[0]; is[1] = 0.f;
    for (int d = 1; d < D; ++d) { im[d + 1] = mmean[d]; is[d + 1] = mstd[d]; }
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
  if (a->B == 0) return 0;  // empty batch: nothing to read or write (empty buffers may be NULL)
  MOPO_REQUIRE(a->d_ens_mean && a->d_ens_var, "mopo_fakeenv_step: ensemble workspaces required");
  MOPO_REQUIRE(a->deterministic || (a->d_noise_sel && a->d_model_inds),
               "mopo_fakeenv_step: noise and model_inds required unless deterministic");
  MOPO_REQUIRE(a->d_next_obs && a->d_rewards && a->d_terminals, "mopo_fakeenv_step: NULL output");
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
