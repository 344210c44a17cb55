// rx_policy.h -- the actor-critic MLP's flat parameter layout (agent/ppo.py:11-62)
// and the per-action-dim log-density, shared by the fused PPO kernels
// (rx_ppo.hip) and the persistent small-N rollout (k_rollout, rx_kernels.hip),
// so both evaluate the policy with the same operations.
#pragma once
#include <hip/hip_runtime.h>

namespace rx_policy {

constexpr int kH = 64;   // hidden width (agent/ppo.py:20-29)
constexpr int kNA = 2;   // action dims

template <int D>
struct Lay {  // flat parameter offsets, module.parameters() order; Pp = partial row stride
  static constexpr int aW1 = 0, ab1 = aW1 + kH * D, aW2 = ab1 + kH, ab2 = aW2 + kH * kH, aW3 = ab2 + kH,
                       ab3 = aW3 + kNA * kH, cW1 = ab3 + kNA, cb1 = cW1 + kH * D, cW2 = cb1 + kH,
                       cb2 = cW2 + kH * kH, cW3 = cb2 + kH, cb3 = cW3 + kH, P = cb3 + 1, Pp = (P + 63) / 64 * 64;
};

// tanh for the policy's hidden and head activations: sign(x) * (1 - 2 / (exp(2|x|)
// + 1)) with the hardware exp2 and reciprocal -- 5 VALU (4 plus the sign copy)
// where ocml's tanhf takes ~30 and a small-|x| polynomial branch ~15.  Absolute
// error <= 1.4e-7 over the whole range (float32 emulation with correctly rounded
// exp2 / reciprocal: tools/tanh_error.py), i.e. float rounding of the
// activations.  Relative error: the form cancels as |x| -> 0 (1 - 2/(e + 1)
// with e ~ 1), so below |x| = 2^-12 the result is x itself (tanh x = x (1 -
// x^2/3 + ...): relative error < 2^-25, i.e. exact in float32 up to rounding);
// between 2^-12 and ~0.1 the bound is the absolute 1.4e-7, a relative error of
// up to 1.4e-7 / |x| (6e-4 at 2^-12, 1.4e-6 at 0.1).  tests/test_ppo_fused_gpu.py
// ::test_policy_act_near_zero_preactivations checks torch parity there with
// that combined bound.  The policy's outputs stay within float rounding of
// torch's forward (tests/test_ppo_fused_gpu.py, tests/test_bf16_gpu.py).  Every
// kernel that evaluates the policy uses this one function, so k_rollout and
// rx_policy_act stay bit-identical.  (The VALU count matters: k_ppo_grad's
// forward phase issued ~770 VALU per pass with the polynomial form, 500 with
// this one, beside 96 MFMAs; the small-|x| select adds 2.)
__device__ __forceinline__ float tanh_fast(float x) {
  const float ax = __builtin_fabsf(x);
  const float e = __builtin_amdgcn_exp2f(ax * 2.8853900817779268f);  // exp(2|x|); inf past ~44
  const float t = __builtin_copysignf(fmaf(__builtin_amdgcn_rcpf(e + 1.0f), -2.0f, 1.0f), x);
  return ax < 0x1p-12f ? x : t;
}

// Normal(mu, exp(log_std)).log_prob(a) for one action dim, in torch's operation
// order (torch/distributions/normal.py: -((a-mu)**2)/(2*var) - log(scale) - log(sqrt(2*pi))).
__device__ __forceinline__ float normal_logp(float diff, float var, float log_scale) {
  return -(diff * diff) / (2.0f * var) - log_scale - 0.91893853320467274178f;
}

}  // namespace rx_policy
