#pragma once
#include "internal.h"

namespace mopo {

struct ActorArgs {
  const float* P;    // flat SAC params; pi block at offset 0 (TF [in,out] layout) -- biases read here
  const float* Wpk;  // pi weights repacked fragment-major by pack_actor
  int O, A, Hp;
  const void* obs; int obs_f64;
  int64_t B;               // grid rows
  const int* d_count;      // optional device row count
  const float* eps;        // [B, A] injected normals or NULL (Philox)
  uint64_t seed; uint32_t step;
  const int64_t* d_uid;    // optional per-row global id (Philox counter)
  int64_t uid_offset;
  float* act;              // [B, A]
  float* mu;               // [B, A] tanh(mu) or NULL
  // rollout: write the obs/act half of the pool row and clear the penalty accumulator
  float* pool_obs; float* pool_act; const int64_t* pool_state; int64_t pool_max;
  int64_t stage_base;      // >= 0: staged layout, row goes to stage_base + row
  int64_t pool_off;        // pool layout: row goes to (pool_state[0] + pool_off + row) % pool_max
  uint32_t* pen_zero;
  // rollout: member selection per row (bnn.py:343): injected sel_in or Philox choice over elites
  int32_t* sel_out; const int32_t* sel_in; const int32_t* elites; int n_elites;
  // rollout: the ensemble's scaled input row (utils.py:96) [B][32] in slot_feat(., xs_in) order,
  // (concat(obs, act) - mu) / sigma, so the ensemble reads 128 contiguous bytes per row and member
  float* xs; const float* xs_mu; const float* xs_sigma; int xs_in;
  // rollout_random (mopo.py:736-738): the actions are U(-1, 1) draws -- injected act_uni [B, A] or
  // Philox -- and replace the policy's (still computed, as the reference calls get_action_meta first)
  int rand_act; const float* act_uni;
  // 0: f32 MFMA on the fragment-major f32 packing; 4 (DT_F16X3): the f16x3 split (mlp_tile.h) on the
  // f16 packing (pack_actor with split = 1); 3 (DT_BF16X6): the exact 3-part bf16 split (split = 2)
  int dtype;
  // 1: no other launch runs beside this one (an unsplit rollout): the f16x3 ring actor (actor_f16q_kernel,
  // 203 VGPRs), faster alone, slower beside the other row part's ensemble launch
  int alone;
};

int launch_actor(const ActorArgs& a, hipStream_t s);
__host__ __device__ int64_t actor_packed_floats(int O, int Hp, int split = 0);
int pack_actor(const float* P, int O, int A, int Hp, float* dst, hipStream_t s, int split = 0);

}  // namespace mopo
