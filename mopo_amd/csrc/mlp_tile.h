// Register-resident MLP tiles on f32 MFMA with LDS-staged weight slices (shared by bnn.hip, actor.hip).
#pragma once
#include <type_traits>

#include "internal.h"

namespace mopo {

// ---- slot -> feature map of a width-F dimension tiled in 16-slot blocks -----------------------
// Slot s = 4g + t of a block is MFMA lane group g, register (= k-step) t.  Full blocks are the
// identity.  The last partial block (rem = F mod 16 features) packs its features into the first
// q = ceil(rem / 4) registers of every lane group -- feature 16 blk + q g + t for t < q -- so its
// registers t >= q hold only padding and a layer consuming it skips those k-steps (TQ below).
// Weights (both K and N sides of hidden layers), biases and the layer-0 inputs all use it; the
// head's outputs keep the natural order.  H = 200: 52 -> 50 k-steps per layer; 23 inputs: 8 -> 6.
__host__ __device__ __forceinline__ int slot_feat(int slot, int F) {
  const int blk = slot >> 4, rem = F - 16 * blk;
  if (rem >= 16) return slot;
  if (rem <= 0) return -1;
  const int q = (rem + 3) >> 2, g = (slot >> 2) & 3, t = slot & 3, f = q * g + t;
  return (t < q && f < rem) ? 16 * blk + f : -1;
}

// Head output slots.  Slot s = 16 nb + 4 g + t of the fused head (lane group g, register t) with
// j = 4 nb + t and Q = ceil(D / 4): j < Q holds log-var d = g + 4 j, Q <= j < 2Q holds mean
// d = g + 4 (j - Q), the rest is padding.  The kind of a register is then uniform across the
// wave (no divergent mean / log-var branches in the epilogue) and each register's 4 lane groups
// cover 4 consecutive d.  Returns the column of the fused [mean | log-var] head, or -1.
__host__ __device__ __forceinline__ int head_col(int slot, int D) {
  const int nb = slot >> 4, g = (slot >> 2) & 3, t = slot & 3, j = 4 * nb + t, Q = (D + 3) >> 2;
  if (j < Q) return g + 4 * j < D ? D + g + 4 * j : -1;
  if (j < 2 * Q) return g + 4 * (j - Q) < D ? g + 4 * (j - Q) : -1;
  return -1;
}

// k-steps a consumer must run in the last 16-deep k-group of a width-F input (4: no skip)
__host__ __device__ constexpr int tail_steps(int F) { return (F & 15) == 0 ? 4 : ((F & 15) + 3) >> 2; }

// ---- LDS-staged weight streaming ------------------------------------------------------------
// A workgroup of WAVES waves shares one member; every k-group slice of a layer (NB fragments,
// 1 KiB each, contiguous in HBM) is copied HBM->LDS once per workgroup with global_load_lds
// (no VGPR round trip), double-buffered: the slice for k-group kg+1 is in flight while the waves
// run the 4*NB*R MFMAs of k-group kg.  One barrier per k-group (its implicit vmcnt(0) retires the
// slice issued one k-group earlier, so the copy latency hides behind a full k-group of MFMAs).
typedef __attribute__((address_space(3))) void* lds_void_t;

template <int NB, int WAVES>
struct Stage {
  static constexpr int PER = (NB + WAVES - 1) / WAVES;  // fragments per wave (uniform vmcnt)
  static constexpr int SLOTS = PER * WAVES;
};

// One wave-wide 16-B-per-lane copy HBM -> LDS (lane l's quad lands at lds + 4 l): global_load_lds with a
// 64-bit per-lane address (one v_lshl_add_u64 per copy).  MOPO_LDS_BUF = 1 issues it as buffer_load ...
// lds with the wave-uniform part of the address in SGPRs (descriptor + soffset) and only lane * 16 in a
// VGPR -- no VALU per copy, but measured 5 % slower on the headline rollout (same-box A/B: 122.7 vs
// 129.2M transitions/s, ensemble 0.347 vs 0.333 ms), so it stays off.
#ifndef MOPO_LDS_BUF
#define MOPO_LDS_BUF 0
#endif
__device__ __forceinline__ void copy_lds16(const float* __restrict__ base, int lane_quad, int uni_quads, float* lds) {
#if MOPO_LDS_BUF
  const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t)lds, 16, lane_quad * 16, uni_quads * 16, 0, 0);
#else
  __builtin_amdgcn_global_load_lds((const void*)(base + (uni_quads + lane_quad) * 4), (lds_void_t)lds, 16, 0, 0);
#endif
}

template <int NB, int WAVES>
__device__ __forceinline__ void stage_slice(const float* __restrict__ src, float* lds, int w, int lane) {
#pragma unroll
  for (int i = 0; i < Stage<NB, WAVES>::PER; ++i) {
    const int f = w + i * WAVES;
// pad slots re-read a valid fragment (never consumed); measured: skipping them with a wave-uniform
    // branch is ~1.5 % slower for H = 200 (13 of 16 slots used)
    const int fs = f < NB ? f : NB - 1;
    copy_lds16(src, lane, fs * 64, lds + f * 256);
  }
}

// acc[r][nb] = sum over KG k-groups of W(kg, nb) x in[r][kg]; wf = this member's layer fragments.
// If `bias` is given, the layer's BQ*4 bias values (default NB*16) are copied to lds_bias (1 KiB global_load_lds
// pieces, one per wave) together with the last k-group's slice, so the barrier that publishes that slice
// also publishes the bias for the epilogue (bias_swish reads it from LDS).
template <int BQ, int WAVES>
__device__ __forceinline__ void stage_bias(const float* __restrict__ bias, float* lds_bias, int w, int lane) {
  constexpr int PIECES = (BQ + 63) / 64;  // BQ quads; 1 KiB (64 quads) per wave-wide copy
  static_assert(PIECES <= WAVES, "bias larger than one copy per wave");
  if (w < PIECES) {
    const int q = min(w * 64 + lane, BQ - 1);
    copy_lds16(bias, q, 0, lds_bias + w * 256);
  }
}

// One pipeline block: KPB k-groups x NB output tiles of a layer whose k-group slices lie NBS
// fragments apart (NBS > NB: a subset of the output tiles), fragment (j, nb) into LDS slot j*NB + nb.
// Every wave issues the same number of copies (pad slots re-read a valid fragment, never consumed):
// measured faster than skipping them with a wave-uniform branch.  kg_valid: k-groups left in the layer.
template <int NB, int KPB, int NBS, int WAVES>
__device__ __forceinline__ void stage_block(const float* __restrict__ src, float* lds, int w, int lane, int kg_valid) {
  constexpr int NF = KPB * NB, PER = (NF + WAVES - 1) / WAVES;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int f = w + i * WAVES;
    int j = (f < NF ? f : NF - 1) / NB, nb = (f < NF ? f : NF - 1) % NB;
    if (j >= kg_valid) j = kg_valid - 1;
    copy_lds16(src, lane, (j * NBS + nb) * 64, lds + f * 256);
  }
}

// TQ: k-steps run in the last k-group (slot_feat tail; 4 = all).
// Cross-layer prefetch: NBN > 0 stages the NEXT layer's first slice (wf_next, NBN fragments) during
// this layer's last k-group, and that layer is then called with PRE = true (no initial barrier +
// exposed copy).  `par` is the buffer of block 0 (block b uses buffer (b + par) & 1).
// NBS: fragments per k-group slice in memory (NB < NBS: this call covers output tiles [0, NB) of a
// wider layer whose slices start at wf + kg * NBS fragments); ACC: accumulate into acc (no zeroing).
// KPBN / NBSN: pipeline-block shape of the next call (its first block is what NBN > 0 prefetches).
template <int KG, int NB, int R, int WAVES, int SLOT, int BQ = NB * 4, int KPB = 1, int TQ = 4, int NBN = 0,
          bool PRE = false, int NBS = NB, bool ACC = false, int KPBN = 1, int NBSN = NBN>
__device__ __forceinline__ void layer_lds(const float* __restrict__ wf, const f32x4 (&in)[R][KG], f32x4 (&acc)[R][NB],
                                          float* lds, int w, int lane, const float* __restrict__ bias = nullptr,
                                          float* lds_bias = nullptr, int par = 0,
                                          const float* __restrict__ wf_next = nullptr) {
  static_assert(!PRE || KG >= 2, "a prestaged layer stages its bias with a later slice");
  static_assert(((KPB * NB + WAVES - 1) / WAVES) * WAVES * 256 <= SLOT, "pipeline block larger than its buffer");
  if (!ACC)
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) acc[r][nb] = zero4();
  constexpr int NBLK = (KG + KPB - 1) / KPB;
  // BNN_KNOB_* (scripts/micro/bnn_knobs.hip): timing-only builds with one part removed
  if (!PRE) {
#ifndef BNN_KNOB_NOBARRIER
    __syncthreads();  // every wave is done reading both buffers (previous layer)
#endif
#ifndef BNN_KNOB_NOSTAGE
    stage_block<NB, KPB, NBS, WAVES>(wf, lds + par * SLOT, w, lane, KG);
    if (NBLK == 1 && bias) stage_bias<BQ, WAVES>(bias, lds_bias, w, lane);
#endif
  }
#pragma unroll
  for (int blk = 0; blk < NBLK; ++blk) {
#ifndef BNN_KNOB_NOBARRIER
    __syncthreads();  // vmcnt(0): block blk landed (all waves); buffer (blk+1)&1 free
#endif
#ifndef BNN_KNOB_NOSTAGE
    if (blk + 1 < NBLK) {
      stage_block<NB, KPB, NBS, WAVES>(wf + (blk + 1) * KPB * NBS * 256, lds + ((blk + 1 + par) & 1) * SLOT, w, lane,
                                       KG - (blk + 1) * KPB);
    } else {
      if constexpr (NBN > 0)
        stage_block<NBN, KPBN, NBSN, WAVES>(wf_next, lds + ((blk + 1 + par) & 1) * SLOT, w, lane, KPBN);
    }
    if (blk + 2 == NBLK && bias) stage_bias<BQ, WAVES>(bias, lds_bias, w, lane);
#endif
#ifndef BNN_KNOB_NOPIN
    // keep the next slice's copies issued here, ahead of this k-group's MFMAs: left alone, the
    // scheduler sinks every other k-group's copies to just before the next barrier, whose
    // vmcnt(0) then exposes their whole latency
    __builtin_amdgcn_sched_barrier(0);
#endif
#ifdef BNN_KNOB_PRIO
    __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
    for (int j = 0; j < KPB; ++j) {
      const int kg = blk * KPB + j;
      if (kg < KG) {
        const float* b = lds + ((blk + par) & 1) * SLOT + j * NB * 256;
        // fragment nb + 1 is read before the MFMAs of fragment nb (one LDS read in flight)
        f32x4 fr_next = *reinterpret_cast<const f32x4*>(b + lane * 4);
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          const f32x4 fr = fr_next;
          if (nb + 1 < NB) fr_next = *reinterpret_cast<const f32x4*>(b + ((nb + 1) * 64 + lane) * 4);
#pragma unroll
          for (int t = 0; t < (kg + 1 == KG ? TQ : 4); ++t)
#pragma unroll
            for (int r = 0; r < R; ++r) {
#ifndef BNN_KNOB_NOMFMA
              acc[r][nb] = mfma4(fr[t], in[r][kg][t], acc[r][nb]);
#else
              acc[r][nb][t] += fr[t] * in[r][kg][t];
#endif
            }
        }
      }
    }
#ifdef BNN_KNOB_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
  }
}

// ---- bf16 variant (v_mfma_f32_16x16x32_bf16, f32 accumulate) --------------------------------
// A k-group is 32 deep; lane (row m, group g) supplies 8 bf16 of its row.  The k order inside a
// group is permuted so the B operand comes straight from the previous layer's two accumulator
// blocks 2c, 2c+1 (feature 16*nb + 4g + r held by lane (m, g) in register r):
//   element j of lane group g  <->  feature 32c + (j < 4 ? 4g + j : 16 + 4g + (j - 4)).
// The weight fragments are packed with the same permutation (pack_frags_bf16_kernel).
typedef short bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f32x4 mfma_bf16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// the same 16x16x32 shape on f16 operands (the "f16x3" split: fp16 parts, stored as their bits)
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ f32x4 mfma_f16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

template <bool F16>
__device__ __forceinline__ f32x4 mfma_16x16x32(bf16x8 a, bf16x8 b, f32x4 c) {
  if constexpr (F16) return mfma_f16(a, b, c);
  else return mfma_bf16(a, b, c);
}

// k-half MFMA (16x16x16) on the low 4 elements of 16x16x32 operands: by bf16_kperm those are k = 4 g + j,
// j < 4, i.e. the first 16 of the k-group.  Used for a k-group whose upper 16 are all padding.
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
template <bool F16>
__device__ __forceinline__ f32x4 mfma_16x16x16_lo(bf16x8 a, bf16x8 b, f32x4 c) {
  const s16x4 al = __builtin_shufflevector(a, a, 0, 1, 2, 3), bl = __builtin_shufflevector(b, b, 0, 1, 2, 3);
  if constexpr (F16)
    return __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(f16x4, al), __builtin_bit_cast(f16x4, bl), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(al, bl, c, 0, 0, 0);
}

__host__ __device__ __forceinline__ int bf16_kperm(int g, int j) { return j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4); }

__device__ __forceinline__ short to_bf16(float x) { return __builtin_bit_cast(short, (__bf16)x); }

#ifndef MOPO_BF16_PF
#define MOPO_BF16_PF 4   // layer_lds_bf16: fragment reads in flight
#endif
template <int KG, int NB, int WAVES, int SLOT, int NBU = NB, bool KH = false>
__device__ __forceinline__ void layer_lds_bf16(const float* __restrict__ wf, const bf16x8 (&in)[KG], f32x4 (&acc)[NB],
                                               float* lds, int w, int lane, const float* __restrict__ bias = nullptr,
                                               float* lds_bias = nullptr) {
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) acc[nb] = zero4();
#ifndef BNN_KNOB_NOBARRIER
  __syncthreads();
#endif
#ifndef BNN_KNOB_NOSTAGE
  stage_slice<NB, WAVES>(wf, lds, w, lane);
  if (bias) stage_bias<NB * 4, WAVES>(bias, lds_bias, w, lane);  // published by the first barrier below
#endif
#pragma unroll
  for (int kg = 0; kg < KG; ++kg) {
#ifndef BNN_KNOB_NOBARRIER
    __syncthreads();
#endif
#ifndef BNN_KNOB_NOSTAGE
    if (kg + 1 < KG) stage_slice<NB, WAVES>(wf + (kg + 1) * NB * 256, lds + ((kg + 1) & 1) * SLOT, w, lane);
#endif
    const float* b = lds + (kg & 1) * SLOT;
    // fragments read MOPO_BF16_PF ahead, each read pinned ahead of the MFMAs that follow it (one MFMA per
    // fragment: left to the scheduler, every read sits right before its use)
    constexpr int PF = MOPO_BF16_PF < NBU ? MOPO_BF16_PF : NBU;
    bf16x8 fq[PF];
#pragma unroll
    for (int k = 0; k < PF; ++k) fq[k] = *reinterpret_cast<const bf16x8*>(b + (k * 64 + lane) * 4);
#pragma unroll
    for (int nb = 0; nb < NBU; ++nb) {  // blocks >= NBU: padding output block, skipped
      const bf16x8 fr = fq[nb % PF];
      if (nb + PF < NBU) fq[nb % PF] = *reinterpret_cast<const bf16x8*>(b + ((nb + PF) * 64 + lane) * 4);
      if constexpr (MOPO_BF16_PF > 1) __builtin_amdgcn_sched_barrier(0x0406);
#ifndef BNN_KNOB_NOMFMA
      // KH: the last k-group's upper 16 are padding (odd input-block count), so a 16-deep MFMA
      if (KH && kg + 1 == KG) acc[nb] = mfma_16x16x16_lo<false>(fr, in[kg], acc[nb]);
      else acc[nb] = mfma_bf16(fr, in[kg], acc[nb]);
#else
      acc[nb][0] += (float)fr[0];
#endif
    }
  }
}

// ---- split-bf16 variant: f32 operands as P bf16 parts (x = x0 + x1 [+ x2]) ---------------------
// Part p of a value is the round-to-nearest-even bf16 of its residual after parts 0..p-1 (each residual is
// exact in f32).  P = 3 is an EXACT split: x0 + x1 + x2 == x for every f32 with 2^-100 <= |x| < 2^127 (and
// x = 0): x0 takes the top 8 significand bits, the residual x - x0 is a multiple of ulp(x) of at most 2^15
// ulps, x1 takes its top 8 bits, and what is left is a multiple of ulp(x) of at most 2^7 ulps -- 8 bits, so
// x2 holds it exactly (above 2^-100 every part is a normal bf16).  The layer runs the products W_p x X_q
// with p + q < P (P = 2: 3 MFMAs, P = 3: 6 MFMAs per k-group and block) on v_mfma_f32_16x16x32_bf16 with f32
// accumulate; the three dropped products x1 w2 + x2 w1 + x2 w2 are <= (2^-24 + 2^-24 + 2^-32) |x w| with
// RN parts (|x1| <= 2^-8 |x|, |x2| <= 2^-16 |x|), under f32's own rounding of the sums.  Weight fragments
// are packed [kg][p][nb] (pack_frags_bf16_kernel with P parts), so the pipeline streams KG * P slices of NB
// fragments through the same LDS slots as the bf16 layer: slice (kg, p) feeds the (P - p) activation parts
// of k-group kg.  (tests/test_split.py holds the CPU restatement of this split to the exactness claim.)
__device__ __forceinline__ float from_bf16(short s) { return __builtin_bit_cast(float, (uint32_t)(uint16_t)s << 16); }
template <int P>
__device__ __forceinline__ void split_bf16(float v, short (&out)[P]) {
  float r = v;
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const short s = to_bf16(r);
    out[p] = s;
    if (p + 1 < P) r -= from_bf16(s);
  }
}
// two values at once into whole dwords (part p of a in the low half, of b in the high half): v_cvt_pk_bf16_f32
// rounds to nearest even; the residuals are exact subtractions of the parts' f32 values (a v_dot2_f32_bf16
// form of the subtraction, a + (-1) * part, measured WRONG on gfx950: errors of 0.03-1 in the ensemble output)
template <int P>
__device__ __forceinline__ void split_bf16_pair(float a, float b, uint32_t (&out)[P]) {
#pragma unroll
  for (int p = 0; p < P; ++p) {
    uint32_t h;
    asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(h) : "v"(a), "v"(b));
    out[p] = h;
    if (p + 1 < P) {
      a -= __builtin_bit_cast(float, h << 16);
      b -= __builtin_bit_cast(float, h & 0xffff0000u);
    }
  }
}

// PS: parts staged per slice (P: one slice of P * NB fragments per k-group; 1: P slices of NB).
// F16: the parts are fp16 ("f16x3", split_f16_scaled) and the products run on the f16 MFMA.
// bias / lds_bias: the layer's NB * 16 bias values are copied to LDS with the first slice (published by
// the first k-group's barrier), so the epilogue reads them from LDS instead of global memory.
template <int KG, int NB, int WAVES, int SLOT, int P, int PS = P, bool F16 = false, int NBU = NB, bool KH = false>
__device__ __forceinline__ void layer_lds_split(const float* __restrict__ wf, const bf16x8 (&in)[P][KG],
                                                f32x4 (&acc)[NB], float* lds, int w, int lane,
                                                const float* __restrict__ bias = nullptr, float* lds_bias = nullptr) {
  static_assert(P % PS == 0, "parts per slice must divide the parts");
  constexpr int SPK = P / PS, S = KG * SPK, NF = PS * NB;
  static_assert(Stage<NF, WAVES>::SLOTS * 256 <= SLOT, "slice larger than its buffer");
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) acc[nb] = zero4();
  __syncthreads();
  stage_slice<NF, WAVES>(wf, lds, w, lane);
  if (bias) stage_bias<NB * 4, WAVES>(bias, lds_bias, w, lane);
#pragma unroll
  for (int s = 0; s < S; ++s) {
    __syncthreads();
    if (s + 1 < S) stage_slice<NF, WAVES>(wf + (s + 1) * NF * 256, lds + ((s + 1) & 1) * SLOT, w, lane);
    __builtin_amdgcn_sched_barrier(0);
    const int kg = s / SPK;
    const float* b = lds + (s & 1) * SLOT;
#ifndef BNN_SPLIT_NOPF
    // fragment i + 1 is read before the MFMAs of fragment i (one LDS read in flight)
    bf16x8 fr_next = *reinterpret_cast<const bf16x8*>(b + lane * 4);
#endif
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      const int pp = i / NB, nb = i % NB, p = (s % SPK) * PS + pp;
      if (nb >= NBU) continue;  // padding output block (odd hidden-block count)
#ifndef BNN_SPLIT_NOPF
      const bf16x8 fr = fr_next;
      const int nx = i + 1 + (((i + 1) % NB) >= NBU ? NB - NBU : 0);
      if (nx < NF) fr_next = *reinterpret_cast<const bf16x8*>(b + (nx * 64 + lane) * 4);
#else
      const bf16x8 fr = *reinterpret_cast<const bf16x8*>(b + (i * 64 + lane) * 4);
#endif
#pragma unroll
      for (int q = P - 1 - p; q >= 0; --q)
        acc[nb] = (KH && kg + 1 == KG) ? mfma_16x16x16_lo<F16>(fr, in[q][kg], acc[nb])
                                       : mfma_16x16x32<F16>(fr, in[q][kg], acc[nb]);
    }
  }
}

// ---- "f16x3": f32 operands as 2 fp16 parts under a power-of-two scale ---------------------------
// v ~ (x0 + x1) / s with x0 = RN_f16(v s), x1 = RN_f16(v s - x0): |v - (x0 + x1)/s| <= 2^-22 |v| (fp16
// unit roundoff 2^-11, squared), and the products x0 w0 + x0 w1 + x1 w0 drop x1 w1 <= 2^-22 |v w|:
// the same ~22-bit class as the 3-part bf16 split (whose truncated parts leave 2^-22 and whose dropped
// products x1 w2, x2 w1 are 2^-21 each) at half its MFMAs.  The scale keeps fp16's range out of the
// way: weights carry one 2^k per layer and member (packed on the device), activations one per row
// (row_scale: the row's max |v| lands in [2^14, 2^15), so nothing overflows and an element far below
// the row max loses at most 2^-38 of it, below f32 rounding of the sums); acc * (2^-k / s) undoes it.
struct F16Parts {
  short hi, lo;
};
__device__ __forceinline__ F16Parts split_f16_scaled(float v, float s) {
  const float vs = v * s;
  const _Float16 h = (_Float16)vs;
  const _Float16 l = (_Float16)(vs - (float)h);
  return {__builtin_bit_cast(short, h), __builtin_bit_cast(short, l)};
}

// Two elements at once into whole dwords (hi parts, lo parts) with v_cvt_pk_f16_f32 (round to nearest):
// every write of an MFMA operand register is a full 32-bit write.  Left to itself the compiler folds the
// split into v_fma_mix{lo,hi}_f16 half-register writes, and an MFMA issued right after a mixhi write
// of its B operand was measured to read a stale half (nondeterministic 2^-11 errors).
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
struct F16Pair {
  uint32_t hi, lo;
};
// The remainders v - f32(hi) come from ONE v_fma_mix_f32 each (the fp16 half read in place, times -1,
// plus v; a full 32-bit result): exact, as the subtraction is (hi = RN16(v) is within half an fp16 ulp of
// v), so the parts are bit-identical to the convert + subtract form, one VALU op per value fewer
// (MOPO_F16_MIXSUB=0: that form)
#ifndef MOPO_F16_MIXSUB
#define MOPO_F16_MIXSUB 1
#endif
__device__ __forceinline__ F16Pair split_f16_pair_prescaled(float as, float bs) {
  uint32_t h;
  asm volatile("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(h) : "v"(as), "v"(bs));
  float la, lb;
  if (MOPO_F16_MIXSUB) {
    asm volatile("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(la) : "v"(h), "v"(as));
    asm volatile("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(lb) : "v"(h), "v"(bs));
  } else {
    la = as - (float)__builtin_bit_cast(_Float16, (uint16_t)(h & 0xffffu));
    lb = bs - (float)__builtin_bit_cast(_Float16, (uint16_t)(h >> 16));
  }
  uint32_t l;
  asm volatile("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(l) : "v"(la), "v"(lb));
  return {h, l};
}

__device__ __forceinline__ F16Pair split_f16_pair(float a, float b, float s) {
  return split_f16_pair_prescaled(a * s, b * s);
}

// power-of-two scale s with max |v| * s in [2^14, 2^15) (mx >= 0; zero / tiny rows clamp, inf / NaN
// stay inf / NaN as in f32) and its exact inverse
__device__ __forceinline__ void row_scale(float mx, float& s, float& inv) {
  uint32_t eb = (__float_as_uint(mx) >> 23) & 0xffu;
  eb = eb < 15u ? 15u : (eb > 254u ? 254u : eb);
  s = __uint_as_float((268u - eb) << 23);
  inv = __uint_as_float((eb - 14u) << 23);
}

#ifndef MOPO_SPLIT_PF
#define MOPO_SPLIT_PF 3  // LDS fragment reads in flight in layer_lds_split_f32 (pinned: MOPO_SPLIT_PIN)
#endif
#ifndef MOPO_SPLIT_PIN
#define MOPO_SPLIT_PIN 1
#endif
// layer_lds_split with f32 activations held (8 VGPRs per k-group instead of 4 * P): each k-group's P
// bf16 parts are split when its first slice is consumed, so only one k-group's parts are live.
// F16: the 2 fp16 parts of in * s (split_f16_scaled; s = the row scale) on the f16 MFMA.
// NBS > NB (PS = 1): the layer's slices hold NBS output blocks, of which this call computes the NB starting at
// wf (a column subset: the H = 400 f16x3 kernel's column halves); BQ: bias quads staged with the first slice
template <int KG, int NB, int WAVES, int SLOT, int P, int PS = P, bool F16 = false, int NBU = NB, bool KH = false,
          int NBS = NB, int BQ = NB * 4>
__device__ __forceinline__ void layer_lds_split_f32(const float* __restrict__ wf, const float (&in)[KG][8],
                                                    f32x4 (&acc)[NB], float* lds, int w, int lane, float sc = 1.f,
                                                    const float* __restrict__ bias = nullptr,
                                                    float* lds_bias = nullptr) {
  static_assert(P % PS == 0, "parts per slice must divide the parts");
  static_assert(NBS == NB || PS == 1, "a column subset needs one part per slice");
  constexpr int SPK = P / PS, S = KG * SPK, NF = PS * NB, SSTR = PS * NBS;   // SSTR: slice stride (fragments)
  static_assert(Stage<NF, WAVES>::SLOTS * 256 <= SLOT, "slice larger than its buffer");
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) acc[nb] = zero4();
  bf16x8 cur[P];
  __syncthreads();
  stage_slice<NF, WAVES>(wf, lds, w, lane);
  if (bias) stage_bias<BQ, WAVES>(bias, lds_bias, w, lane);  // published by the first barrier below
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int kg = s / SPK;
    if (s % SPK == 0) {
      if constexpr (F16) {
        static_assert(!F16 || P == 2, "f16 split has 2 parts");
        u32x4v h4, l4;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const F16Pair pr = split_f16_pair(in[kg][2 * q], in[kg][2 * q + 1], sc);
          h4[q] = pr.hi;
          l4[q] = pr.lo;
        }
        cur[0] = __builtin_bit_cast(bf16x8, h4);
        cur[P - 1] = __builtin_bit_cast(bf16x8, l4);
      }
      if constexpr (!F16) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          short parts[P];
          split_bf16<P>(in[kg][j], parts);
#pragma unroll
          for (int p = 0; p < P; ++p) cur[p][j] = parts[p];
        }
      }
    }
    __syncthreads();
    if (s + 1 < S) stage_slice<NF, WAVES>(wf + (s + 1) * SSTR * 256, lds + ((s + 1) & 1) * SLOT, w, lane);
    __builtin_amdgcn_sched_barrier(0);
    const float* b = lds + (s & 1) * SLOT;
#if MOPO_SPLIT_PF <= 1
    // fragment i's successor is read before fragment i's MFMAs (one LDS read in flight); output
    // blocks nb >= NBU (the padding block of an odd hidden-block count) are skipped
    bf16x8 fr_next = *reinterpret_cast<const bf16x8*>(b + lane * 4);
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      const int pp = i / NB, nb = i % NB, p = (s % SPK) * PS + pp;
      if (nb >= NBU) continue;
      const bf16x8 fr = fr_next;
      const int nx = i + 1 + (((i + 1) % NB) >= NBU ? NB - NBU : 0);
      if (nx < NF) fr_next = *reinterpret_cast<const bf16x8*>(b + (nx * 64 + lane) * 4);
#pragma unroll
      for (int q = P - 1 - p; q >= 0; --q)
        acc[nb] = (KH && kg + 1 == KG) ? mfma_16x16x16_lo<F16>(fr, cur[q], acc[nb])
                                       : mfma_16x16x32<F16>(fr, cur[q], acc[nb]);
    }
#else
    // MOPO_SPLIT_PF = D reads in flight: the used fragments of the slice (padding blocks skipped) are
    // consumed in order u = 0, 1, ... and fragment u + D is read before fragment u's MFMAs
    constexpr int D = MOPO_SPLIT_PF;
    constexpr int NU = (NF / NB) * NBU;  // used fragments of the slice
    auto frag_at = [&](int u) { return (u / NBU) * NB + u % NBU; };
    bf16x8 ring[D];
#pragma unroll
    for (int u = 0; u < D && u < NU; ++u) ring[u] = *reinterpret_cast<const bf16x8*>(b + (frag_at(u) * 64 + lane) * 4);
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int i = frag_at(u);
      const int pp = i / NB, nb = i % NB, p = (s % SPK) * PS + pp;
      const bf16x8 fr = ring[u % D];
      if (u + D < NU) ring[u % D] = *reinterpret_cast<const bf16x8*>(b + (frag_at(u + D) * 64 + lane) * 4);
      // the read stays ahead of the MFMAs that follow it (bnn_fwd_ring_kernel's BNN_RING_PIN)
      if constexpr (MOPO_SPLIT_PIN) __builtin_amdgcn_sched_barrier(0x0406);
#pragma unroll
      for (int q = P - 1 - p; q >= 0; --q)
        acc[nb] = (KH && kg + 1 == KG) ? mfma_16x16x16_lo<F16>(fr, cur[q], acc[nb])
                                       : mfma_16x16x32<F16>(fr, cur[q], acc[nb]);
    }
#endif
  }
}

// layer_lds_split_f32's f16 form over R row blocks per wave: every weight fragment read from LDS feeds
// the MFMAs of all R row blocks (R = 2 halves the LDS reads, the barriers and the staged bytes per row).
// in[r]: row block r's f32 activations (scaled by sc[r] when split); parts made when a k-group is consumed.
// NBN > 0: during the last slice, stage the NEXT layer's first slice (NBN fragments at wf_next) into the
// other buffer; that layer is then called with PRE = true (no initial barrier + exposed copy; its bias
// goes out with its second slice).  Every layer here has an even slice count, so slice s always uses
// buffer s & 1.
template <int KG, int NB, int R, int WAVES, int SLOT, int NBU = NB, bool KH = false, int NBN = 0, bool PRE = false>
__device__ __forceinline__ void layer_f16_rows(const float* __restrict__ wf, const float (&in)[R][KG][8],
                                               f32x4 (&acc)[R][NB], float* lds, int w, int lane, const float (&sc)[R],
                                               const float* __restrict__ bias = nullptr, float* lds_bias = nullptr,
                                               const float* __restrict__ wf_next = nullptr) {
  constexpr int P = 2, S = KG * P;
  static_assert(Stage<NB, WAVES>::SLOTS * 256 <= SLOT, "slice larger than its buffer");
  static_assert(Stage<NBN, WAVES>::SLOTS * 256 <= SLOT, "next slice larger than its buffer");
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[r][nb] = zero4();
  bf16x8 cur[R][P];
  if (!PRE) {
    __syncthreads();
    stage_slice<NB, WAVES>(wf, lds, w, lane);
    if (bias) stage_bias<NB * 4, WAVES>(bias, lds_bias, w, lane);  // published by the first barrier below
  }
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int kg = s / P, p = s % P;
    if (p == 0) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        u32x4v h4, l4;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const F16Pair pr = split_f16_pair(in[r][kg][2 * q], in[r][kg][2 * q + 1], sc[r]);
          h4[q] = pr.hi;
          l4[q] = pr.lo;
        }
        cur[r][0] = __builtin_bit_cast(bf16x8, h4);
        cur[r][1] = __builtin_bit_cast(bf16x8, l4);
      }
    }
    __syncthreads();
    if (s + 1 < S) stage_slice<NB, WAVES>(wf + (s + 1) * NB * 256, lds + ((s + 1) & 1) * SLOT, w, lane);
    else if constexpr (NBN > 0) stage_slice<NBN, WAVES>(wf_next, lds + (S & 1) * SLOT, w, lane);
    if (PRE && s == 0 && bias) stage_bias<NB * 4, WAVES>(bias, lds_bias, w, lane);  // published at s = 1
    __builtin_amdgcn_sched_barrier(0);
    const float* b = lds + (s & 1) * SLOT;
    bf16x8 fr_next = *reinterpret_cast<const bf16x8*>(b + lane * 4);
#pragma unroll
    for (int nb = 0; nb < NBU; ++nb) {
      const bf16x8 fr = fr_next;
      if (nb + 1 < NBU) fr_next = *reinterpret_cast<const bf16x8*>(b + ((nb + 1) * 64 + lane) * 4);
      // part 0 of W meets both activation parts, part 1 only the high part (the x1 w1 product is dropped)
#pragma unroll
      for (int q = P - 1 - p; q >= 0; --q)
#pragma unroll
        for (int r = 0; r < R; ++r)
          acc[r][nb] = (KH && kg + 1 == KG) ? mfma_16x16x16_lo<true>(fr, cur[r][q], acc[r][nb])
                                            : mfma_16x16x32<true>(fr, cur[r][q], acc[r][nb]);
    }
  }
}

// A narrow f16x3 layer (one 16-wide output block: the actor's [mu | log_std] head) whose 2 KG weight
// fragments sit in ONE staged slice (buffer `buf`, copied beforehand, e.g. as layer_f16_rows' NBN
// prefetch): one barrier for the whole layer instead of one per (k-group, part) slice.
template <int KG, int R>
__device__ __forceinline__ void head_f16_rows(const float (&in)[R][KG][8], f32x4 (&acc)[R], const float* lds_buf,
                                              int lane, const float (&sc)[R]) {
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = zero4();
  __syncthreads();   // vmcnt(0): the slice landed (every wave's copies), and is visible to all
#pragma unroll
  for (int kg = 0; kg < KG; ++kg) {
    const bf16x8 f0 = *reinterpret_cast<const bf16x8*>(lds_buf + ((2 * kg) * 64 + lane) * 4);
    const bf16x8 f1 = *reinterpret_cast<const bf16x8*>(lds_buf + ((2 * kg + 1) * 64 + lane) * 4);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      u32x4v h4, l4;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const F16Pair pr = split_f16_pair(in[r][kg][2 * q], in[r][kg][2 * q + 1], sc[r]);
        h4[q] = pr.hi;
        l4[q] = pr.lo;
      }
      const bf16x8 c0 = __builtin_bit_cast(bf16x8, h4), c1 = __builtin_bit_cast(bf16x8, l4);
      acc[r] = mfma_16x16x32<true>(f0, c1, acc[r]);   // the product order of layer_f16_rows
      acc[r] = mfma_16x16x32<true>(f0, c0, acc[r]);
      acc[r] = mfma_16x16x32<true>(f1, c0, acc[r]);
    }
  }
}

// ---- LDS-ring pipelines (bnn.hip bnn_fwd_f16q_kernel, actor.hip actor_f16q_kernel) --------------
template <int J, int JEND>
struct RingRun {  // f(integral_constant<J>) for J in [J, JEND), unrolled at compile time
  template <class F>
  __device__ __forceinline__ static void run(F&& f) {
    f(std::integral_constant<int, J>{});
    RingRun<J + 1, JEND>::run(f);
  }
};
template <int JEND>
struct RingRun<JEND, JEND> {
  template <class F>
  __device__ __forceinline__ static void run(F&&) {}
};

// s_waitcnt vmcnt(N) expcnt(7) lgkmcnt(0) (gfx9 encoding: vmcnt [3:0] + [15:14], expcnt [6:4], lgkmcnt [11:8])
template <int N>
__device__ __forceinline__ void wait_vm_lgkm0() {
  static_assert(N >= 0 && N < 64, "vmcnt out of range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | ((N >> 4) << 14));
}

}  // namespace mopo
