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

__device__ double block_sum(double x, double* red) {
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  const int w = threadIdx.x >> 6;
  __syncthreads();  // red[] may still be read by the previous call
  if ((threadIdx.x & 63) == 0) red[w] = x;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < kWaves; ++i) s += red[i];  // same order in every thread
  return s;
}

__global__ __launch_bounds__(kThreads) void k_adam_clip(adam_args a) {
  if (a.stop && *a.stop) return;  // uniform: KL early stop already hit
  __shared__ double red[kWaves];
  const int n_t = a.cfg.n_tensors;
  const int64_t n = a.cfg.offsets[n_t];
  float coef = 1.0f;
  if (a.cfg.max_grad_norm > 0.0) {
    // torch.nn.utils.clip_grad_norm_: total = ||(||g_0||, ..., ||g_k||)||_2,
    // coef = clamp(max_norm / (total + 1e-6), max=1), grads *= coef
    float tot2 = 0.0f;
    for (int t = 0; t < n_t; ++t) {
      double s = 0.0;
      for (int64_t i = a.cfg.offsets[t] + threadIdx.x; i < a.cfg.offsets[t + 1]; i += kThreads) {
        const double x = a.g[i];
        s += x * x;
      }
      const float nt = (float)sqrt(block_sum(s, red));
      tot2 += nt * nt;
    }
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
