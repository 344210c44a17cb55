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

// Normal(mu, exp(log_std)).log_prob(a) for one action dim, in torch's operation
// order (torch/distributions/normal.py: -((a-mu)**2)/(2*var) - log(scale) - log(sqrt(2*pi))).
__device__ __forceinline__ float normal_logp(float diff, float var, float log_scale) {
  return -(diff * diff) / (2.0f * var) - log_scale - 0.91893853320467274178f;
}

}  // namespace rx_policy
