// Fused gradient clipping + Adam step for the PPO update (agent/ppo.py:204-207):
//   nn.utils.clip_grad_norm_(params, max_grad_norm); optimizer.step()
// with torch.optim.Adam(lr, eps=1e-5) (agent/ppo.py:83).  The policy has ~11k
// parameters, so the eager torch path is ~40 launches of a few hundred
// elements each; here it is ONE workgroup of 1024 threads (16 wave64s):
// per-tensor squared norms -> global norm -> clip coefficient -> Adam, with
// the step count, lr and an early-stop flag read from device memory so the
// launch can sit inside a captured graph.
#include <hip/hip_runtime.h>

#include "rx.h"

namespace {

constexpr int kThreads = 1024;
constexpr int kWaves = kThreads / 64;

struct adam_args {
  rx_adam_config cfg;
  float* p;
  float* g;
  float* m;
  float* v;
  float* step;
  const double* lr;
  const uint8_t* stop;
};

__global__ __launch_bounds__(kThreads) void k_adam_clip(adam_args a) {
  if (a.stop && *a.stop) return;  // uniform: KL early stop already hit
  __shared__ float sq[RX_ADAM_MAX_TENSORS][kThreads];  // per-thread partial sums of squares, per tensor
  __shared__ float norms[RX_ADAM_MAX_TENSORS];
  const int n_t = a.cfg.n_tensors;
  const int64_t n = a.cfg.offsets[n_t];
  float coef = 1.0f;
  if (a.cfg.max_grad_norm > 0.0) {
    // torch.nn.utils.clip_grad_norm_: total = ||(||g_0||, ..., ||g_k||)||_2,
    // coef = clamp(max_norm / (total + 1e-6), max=1), grads *= coef.
    // Pass 1: coalesced, independent loads; each thread adds g^2 into its own
    // slot of its element's tensor.  Pass 2: wave t reduces tensor t's slots.
    for (int t = 0; t < n_t; ++t) sq[t][threadIdx.x] = 0.0f;
    int t = 0;
#pragma unroll 4
    for (int64_t i = threadIdx.x; i < n; i += kThreads) {
      while (i >= a.cfg.offsets[t + 1]) ++t;
      const float x = a.g[i];
      sq[t][threadIdx.x] = fmaf(x, x, sq[t][threadIdx.x]);
    }
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int u = wave; u < n_t; u += kWaves) {
      float s = 0.0f;
      for (int k = lane; k < kThreads; k += 64) s += sq[u][k];
      for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      if (lane == 0) norms[u] = sqrtf(s);
    }
    __syncthreads();
    float tot2 = 0.0f;
    for (int u = 0; u < n_t; ++u) tot2 += norms[u] * norms[u];
    const float total = sqrtf(tot2);
    coef = fminf((float)a.cfg.max_grad_norm / (total + 1e-6f), 1.0f);
  }
  // torch.optim.Adam (foreach, non-capturable) with step count s:
  //   m = lerp(m, g, 1-b1); v = v*b2 + (1-b2)*g*g;
  //   p += (-lr/(1-b1^s)) * m / (sqrt(v)/sqrt(1-b2^s) + eps)
  const double s = (double)*a.step + 1.0;
  const double b1 = a.cfg.beta1, b2 = a.cfg.beta2;
  const float w1 = (float)(1.0 - b1);
  const float fb2 = (float)b2, w2 = (float)(1.0 - b2);
  const float step_size = (float)(-(*a.lr / (1.0 - pow(b1, s))));
  const float bc2_sqrt = (float)sqrt(1.0 - pow(b2, s));
  const float eps = (float)a.cfg.eps;
#pragma unroll 4
  for (int64_t i = threadIdx.x; i < n; i += kThreads) {
    const float g = a.g[i] * coef;
    a.g[i] = g;
    float m = a.m[i];
    m = m + w1 * (g - m);  // torch.lerp, weight < 0.5 branch
    float v = a.v[i] * fb2;
    v = v + w2 * g * g;
    a.m[i] = m;
    a.v[i] = v;
    const float den = sqrtf(v) / bc2_sqrt + eps;
    a.p[i] = a.p[i] + step_size * (m / den);
  }
  if (threadIdx.x == 0) *a.step = (float)s;
}

}  // namespace

extern "C" int rx_launch_adam(const rx_adam_config* cfg, float* p, float* g, float* m, float* v, float* step,
                              const double* lr, const uint8_t* stop, hipStream_t s) {
  adam_args a{*cfg, p, g, m, v, step, lr, stop};
  hipLaunchKernelGGL(k_adam_clip, dim3(1), dim3(kThreads), 0, s, a);
  return (int)hipGetLastError();
}
