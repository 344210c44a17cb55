// The actor-critic MLP forward on the matrix cores, shared by the policy
// launches of rx_ppo.hip (k_policy_act, k_selfplay_act, k_ppo_grad's forward),
// so every launch that evaluates the policy does exactly the same arithmetic (DESIGN.md §3:
// v_mfma_f32_16x16x4_f32 is a k-ordered fmaf chain; the layouts below fix
// every summation order).  agent/ppo.py:11-62, :105-110.
#pragma once
#include <hip/hip_runtime.h>

#include "rx.h"
#include "rx_policy.h"

#ifndef PPO_STAMP
#define PPO_STAMP(j) \
  do {               \
  } while (0)
#endif

namespace {

using rx_policy::kH;
using rx_policy::kNA;
using rx_policy::Lay;
using rx_policy::normal_logp;
using f4 = float __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 mma(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// bf16 precision (rx_ppo_batch / rx_policy_io .precision = RX_PREC_BF16,
// config["policy_dtype"] = "bf16"): the same products on
// v_mfma_f32_16x16x32_bf16, operands rounded to bf16, f32 accumulation.
// Lane l holds A[row l & 15][k = 8(l >> 4) + j] and B[k][col l & 15], j < 8.
// A k-step of 32 hidden units is ordered so that its B fragment is lane-local
// in the transposed register layout: slot (q, j) <-> hidden unit
// h = 32s + 16(j >> 2) + 4q + (j & 3), i.e. tile 2s + (j >> 2), register j & 3.
using bf8 = __bf16 __attribute__((ext_vector_type(8)));
constexpr int kF32 = RX_PREC_FP32, kBF16 = RX_PREC_BF16;

__device__ __forceinline__ f4 mma16(bf8 a, bf8 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ bf8 to_bf8(float4 lo, float4 hi) {
  bf8 v;
  v[0] = (__bf16)lo.x, v[1] = (__bf16)lo.y, v[2] = (__bf16)lo.z, v[3] = (__bf16)lo.w;
  v[4] = (__bf16)hi.x, v[5] = (__bf16)hi.y, v[6] = (__bf16)hi.z, v[7] = (__bf16)hi.w;
  return v;
}
__device__ __forceinline__ bf8 to_bf8(const f4& lo, const f4& hi) {
  return to_bf8(make_float4(lo[0], lo[1], lo[2], lo[3]), make_float4(hi[0], hi[1], hi[2], hi[3]));
}

template <int D>
struct Geo {
  static constexpr int KS1 = (D + 3) / 4;   // layer-1 k-steps: d = 4s + q, zero beyond D (15 -> 4, 19 -> 5)
  static constexpr int DP = 4 * KS1 + 1;    // LDS row stride of W1 (odd)
  static constexpr int NT1 = (D + 16) / 16;  // dW1 column tiles including the ones column d = D (1 / 2)
  static constexpr int XS = 16 * NT1 + 1;   // LDS row stride of the per-wave [row][d] input tile
  // input fragment per lane: fp32 x[s] = X[row][4s + q] (s < KS1); bf16 x[j] = X[row][8q + j] (j < 8)
  template <int PREC>
  static constexpr int XN = PREC == kBF16 ? 8 : KS1;
  template <int PREC>
  __device__ static constexpr int d_of(int s, int q) { return PREC == kBF16 ? 8 * q + s : 4 * s + q; }
};

// Weights of one trunk, read either from the flat parameter buffer (global,
// L2-resident) or from the workgroup's LDS copy (same element order, padded
// row strides).  o = output unit, i / d = input unit.
struct WGlobal {
  const float* __restrict__ W1;  // [64][D]
  const float* __restrict__ b1;
  const float* __restrict__ W2;  // [64][64]
  const float* __restrict__ b2;
  const float* __restrict__ W3;  // [n_out][64]
  const float* __restrict__ b3;
  int D;
  __device__ float w1(int o, int d) const { return d < D ? W1[o * D + d] : 0.0f; }
  __device__ float4 w2row4(int o, int i0) const { return *reinterpret_cast<const float4*>(W2 + o * kH + i0); }
  __device__ float w2(int o, int i) const { return W2[o * kH + i]; }
  __device__ float w3(int j, int h) const { return W3[j * kH + h]; }
};
// Forward of one trunk for the wave's 16 rows: x = the lane's input fragment
// (Geo::d_of).  H1 / H2 tiles in the transposed register layout; y = head
// pre-activations: lane (q = 0, l15) holds output j in y[j].
template <int D, int NOUT, int PREC, class Wt>
__device__ __forceinline__ void mlp_forward(const Wt& w, const float (&x)[Geo<D>::template XN<PREC>], f4 (&H1)[4],
                                            f4 (&H2)[4], f4& y, int l15, int q, int stamp = -1) {
  constexpr int KS1 = Geo<D>::KS1;
  const int j3 = l15 < NOUT ? l15 : 0;
  const float on = l15 < NOUT ? 1.0f : 0.0f;
  if constexpr (PREC == kBF16) {
    const bf8 bx = to_bf8(make_float4(x[0], x[1], x[2], x[3]), make_float4(x[4], x[5], x[6], x[7]));
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {  // layer 1: one k-step (d = 8q + j < 32)
      const int o = 16 * mt + l15;
      const float4 lo = make_float4(w.w1(o, 8 * q), w.w1(o, 8 * q + 1), w.w1(o, 8 * q + 2), w.w1(o, 8 * q + 3));
      const float4 hi = make_float4(w.w1(o, 8 * q + 4), w.w1(o, 8 * q + 5), w.w1(o, 8 * q + 6), w.w1(o, 8 * q + 7));
      const f4 z = mma16(to_bf8(lo, hi), bx, f4{0.0f, 0.0f, 0.0f, 0.0f});
#pragma unroll
      for (int r = 0; r < 4; ++r) H1[mt][r] = rx_policy::tanh_fast(z[r] + w.b1[16 * mt + 4 * q + r]);
    }
    const bf8 bh[2] = {to_bf8(H1[0], H1[1]), to_bf8(H1[2], H1[3])};
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      f4 z = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int s = 0; s < 2; ++s)
        z = mma16(to_bf8(w.w2row4(16 * mt + l15, 32 * s + 4 * q), w.w2row4(16 * mt + l15, 32 * s + 16 + 4 * q)),
                  bh[s], z);
#pragma unroll
      for (int r = 0; r < 4; ++r) H2[mt][r] = rx_policy::tanh_fast(z[r] + w.b2[16 * mt + 4 * q + r]);
    }
    y = f4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float v[8];
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) v[jj] = on * w.w3(j3, 32 * s + 16 * (jj >> 2) + 4 * q + (jj & 3));
      y = mma16(to_bf8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7])),
                to_bf8(H2[2 * s], H2[2 * s + 1]), y);
    }
  } else {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      f4 z = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int s = 0; s < KS1; ++s) z = mma(w.w1(16 * mt + l15, 4 * s + q), x[s], z);
#pragma unroll
      for (int r = 0; r < 4; ++r) H1[mt][r] = rx_policy::tanh_fast(z[r] + w.b1[16 * mt + 4 * q + r]);
    }
    if (stamp >= 0) PPO_STAMP(stamp);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      f4 z = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float4 a = w.w2row4(16 * mt + l15, 16 * t + 4 * q);
        z = mma(a.x, H1[t][0], z);
        z = mma(a.y, H1[t][1], z);
        z = mma(a.z, H1[t][2], z);
        z = mma(a.w, H1[t][3], z);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) H2[mt][r] = rx_policy::tanh_fast(z[r] + w.b2[16 * mt + 4 * q + r]);
    }
    if (stamp >= 0) PPO_STAMP(stamp + 1);
    // head on the VALU (NOUT <= 2 of an MFMA tile's 16 output rows would be
    // used): lane (q, l15) sums its own hidden units h = 16t + 4q + r in the
    // order t, r, then the 4 q-lanes of the row combine as (p0 + p1) + (p2 + p3)
    // (xor 16, then xor 32; k_rollout repeats this order).  Every lane of the
    // row ends with output j in y[j].
    y = f4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int j = 0; j < NOUT; ++j) {
      float acc = 0.0f;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc = fmaf(w.w3(j, 16 * t + 4 * q + r), H2[t][r], acc);
      acc += __shfl_xor(acc, 16, 64);
      acc += __shfl_xor(acc, 32, 64);
      y[j] = acc;
    }
    (void)j3;
    (void)on;
  }
}

// The bf16 forward of mlp_forward on PREBUILT operand fragments (16 bytes per
// lane per MFMA operand, in exactly the element order mlp_forward's bf16 path
// converts): F1[mt][lane] layer 1, F2[2 mt + s][lane] layer 2, F3[s][lane] the head
// (rows >= NOUT zero).  Same bf16 values, same MFMAs in the same order as
// mlp_forward<.., kBF16>: bit-identical.  The pointers may be LDS (k_ppo_grad_bf)
// or global (the rollout's per-rollout image, k_policy_frag).
template <int NOUT>
__device__ __forceinline__ void mlp_forward_frag(const bf8* F1, const bf8* F2, const bf8* F3, const float* b1,
                                                 const float* b2, const float (&x)[8], f4 (&H1)[4], f4 (&H2)[4],
                                                 f4& y, int lane, int q) {
  const bf8 bx = to_bf8(make_float4(x[0], x[1], x[2], x[3]), make_float4(x[4], x[5], x[6], x[7]));
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    const f4 z = mma16(F1[mt * 64 + lane], bx, f4{0.0f, 0.0f, 0.0f, 0.0f});
#pragma unroll
    for (int r = 0; r < 4; ++r) H1[mt][r] = rx_policy::tanh_fast(z[r] + b1[16 * mt + 4 * q + r]);
  }
  const bf8 bh[2] = {to_bf8(H1[0], H1[1]), to_bf8(H1[2], H1[3])};
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    f4 z = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int s = 0; s < 2; ++s) z = mma16(F2[(2 * mt + s) * 64 + lane], bh[s], z);
#pragma unroll
    for (int r = 0; r < 4; ++r) H2[mt][r] = rx_policy::tanh_fast(z[r] + b2[16 * mt + 4 * q + r]);
  }
  y = f4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int s = 0; s < 2; ++s) y = mma16(F3[s * 64 + lane], to_bf8(H2[2 * s], H2[2 * s + 1]), y);
}
// one trunk's fragment image in global memory (k_policy_frag): F1 | F2 | F3
constexpr int kFragF1 = 0, kFragF2 = 4 * 64, kFragF3 = kFragF2 + 8 * 64, kFragTrunk = kFragF3 + 2 * 64;  // bf8 units

// Rollout policy step (agent/ppo.py:105-110, get_action_and_value on obs[t]):
// per row  action = clamp(eps * std + mu, -1, 1)   (Normal.sample() = normal_() * std + mu)
//          logp   = sum_j Normal(mu, std).log_prob(action_j),  value = critic(obs).
// eps [N][2] is drawn by the caller with torch's normal_() so the sampling
// stream is torch's.  Wave = 16 rows of one trunk, weights straight from the
// (L2-resident) parameter buffer.
template <int D, int PREC, bool FRAG = false>
__device__ __forceinline__ void policy_rows(const rx_policy_io& io, const float* __restrict__ P, bool critic,
                                            int64_t rb, const bf8* __restrict__ frag = nullptr) {
  using L = Lay<D>;
  constexpr int XN = Geo<D>::template XN<PREC>;
  const int lane = threadIdx.x & 63, l15 = lane & 15, q = lane >> 4;
  const int64_t row = rb * 16 + l15;
  if (rb * 16 >= io.n) return;
  const bool live = row < io.n;
  const int64_t os = io.obs_stride > 0 ? io.obs_stride : D, as = io.act_stride > 0 ? io.act_stride : kNA;
  float x[XN];
#pragma unroll
  for (int s = 0; s < XN; ++s) {
    const int d = Geo<D>::template d_of<PREC>(s, q);
    x[s] = (live && d < D) ? io.obs[row * os + d] : 0.0f;
  }
  f4 H1[4], H2[4], y;
  if (!critic) {
    const WGlobal w{P + L::aW1, P + L::ab1, P + L::aW2, P + L::ab2, P + L::aW3, P + L::ab3, D};
    if constexpr (FRAG && PREC == kBF16)
      mlp_forward_frag<kNA>(frag + kFragF1, frag + kFragF2, frag + kFragF3, w.b1, w.b2, x, H1, H2, y, lane, q);
    else
      mlp_forward<D, kNA, PREC>(w, x, H1, H2, y, l15, q);
    if (q != 0 || !live) return;
    float logp = 0.0f;
#pragma unroll
    for (int j = 0; j < kNA; ++j) {
      const float mu = rx_policy::tanh_fast(y[j] + P[L::ab3 + j]);
      const float scale = expf(io.log_std[j]);
      const float var = scale * scale;
      const float smp = io.eps[row * kNA + j] * scale + mu;  // mul_(std).add_(mu): two roundings
      const float a = fminf(fmaxf(smp, -1.0f), 1.0f);
      io.actions[row * as + j] = a;
      if (io.actions2) io.actions2[row * (io.act2_stride > 0 ? io.act2_stride : kNA) + j] = a;
      logp += normal_logp(a - mu, var, logf(scale));
    }
    if (io.logprobs) io.logprobs[row] = logp;
  } else {
    const WGlobal w{P + L::cW1, P + L::cb1, P + L::cW2, P + L::cb2, P + L::cW3, P + L::cb3, D};
    if constexpr (FRAG && PREC == kBF16) {
      const bf8* fc = frag + kFragTrunk;
      mlp_forward_frag<1>(fc + kFragF1, fc + kFragF2, fc + kFragF3, w.b1, w.b2, x, H1, H2, y, lane, q);
    } else {
      mlp_forward<D, 1, PREC>(w, x, H1, H2, y, l15, q);
    }
    if (q != 0 || !live) return;
    io.values[row] = y[0] + P[L::cb3];
  }
}

}  // namespace
