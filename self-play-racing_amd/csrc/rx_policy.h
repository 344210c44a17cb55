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

// tanh for the policy's hidden and head activations: ocml's split (an odd
// polynomial below |x| = 0.625, 1 - 2 / (exp(2|x|) + 1) above, sign copied
// back) with the hardware exp2 / reciprocal instead of ocml's range-reduced
// exp and full-precision division: ~15 VALU instead of ~30, within a few ulp
// of tanhf (the policy's outputs stay within float rounding of torch's forward,
// tests/test_ppo_fused_gpu.py).  Every kernel that evaluates the policy uses
// this one function, so k_rollout and rx_policy_act stay bit-identical.
__device__ __forceinline__ float tanh_fast(float x) {
  const float ax = __builtin_fabsf(x);
  const float x2 = x * x;
  float p = fmaf(__int_as_float(0xbbbac73d), x2, __int_as_float(0x3ca908c9));
  p = fmaf(x2, p, __int_as_float(0xbd5c1c4e));
  p = fmaf(x2, p, __int_as_float(0x3e088382));
  p = fmaf(x2, p, __int_as_float(0xbeaaaa99));
  const float small = fmaf(x2, ax * p, ax);
  const float e = __builtin_amdgcn_exp2f(ax * 2.8853900817779268f);  // exp(2|x|) = 2^(2|x| log2 e); inf past ~44
  const float large = fmaf(__builtin_amdgcn_rcpf(e + 1.0f), -2.0f, 1.0f);
  return __builtin_copysignf(ax < 0.625f ? small : large, x);
}

// Normal(mu, exp(log_std)).log_prob(a) for one action dim, in torch's operation
// order (torch/distributions/normal.py: -((a-mu)**2)/(2*var) - log(scale) - log(sqrt(2*pi))).
__device__ __forceinline__ float normal_logp(float diff, float var, float log_scale) {
  return -(diff * diff) / (2.0f * var) - log_scale - 0.91893853320467274178f;
}

}  // namespace rx_policy
