// Fused gradient clipping + Adam step for the PPO update (agent/ppo.py:204-207):
//   nn.utils.clip_grad_norm_(params, max_grad_norm); optimizer.step()
// with torch.optim.Adam(lr, eps=1e-5) (agent/ppo.py:83).  The policy has ~11k
// parameters, so the eager torch path is ~40 launches of a few hundred
// elements each; here it is two launches, each one memory round trip wide:
//   k_adam_norm   one workgroup per 1024 elements: per-tensor sums of squares
//                 of its slice -> ws[block][tensor]; bumps the step count;
//   k_adam_apply  one thread per element: every workgroup folds ws in the same
//                 order (per-tensor norms -> global norm -> clip coefficient,
//                 identical in all of them), then clips the gradient and
//                 applies Adam to its element.
// The step count, lr and an early-stop flag live in device memory, so the pair
// can sit inside a captured graph.
#include <hip/hip_runtime.h>

#include "rx.h"

namespace {

constexpr int kT = 256;                 // threads per workgroup (4 waves)
constexpr int kNormElems = RX_ADAM_NORM_ELEMS;  // elements per k_adam_norm workgroup
constexpr int kPer = kNormElems / kT;

struct adam_args {
  rx_adam_config cfg;
  float* p;
  float* g;
  float* m;
  float* v;
  float* step;
  const double* lr;
  const uint8_t* stop;
  float* ws;  // [ceil(n / kNormElems)][n_tensors] partial sums of squares
};

__global__ __launch_bounds__(kT) void k_adam_norm(adam_args a) {
  if (a.stop && *a.stop) return;  // uniform: KL early stop already hit
  if (blockIdx.x == 0 && threadIdx.x == 0) *a.step += 1.0f;  // k_adam_apply reads the new count
  if (!(a.cfg.max_grad_norm > 0.0)) return;
  __shared__ float sq[RX_ADAM_MAX_TENSORS][kT];  // per-thread sums of squares, per tensor
  const int n_t = a.cfg.n_tensors;
  const int64_t n = a.cfg.offsets[n_t];
  const int64_t base = (int64_t)blockIdx.x * kNormElems + threadIdx.x;
  float x[kPer];
#pragma unroll
  for (int k = 0; k < kPer; ++k) {  // independent coalesced loads, one round trip
    const int64_t i = base + (int64_t)k * kT;
    x[k] = i < n ? a.g[i] : 0.0f;
  }
  for (int t = 0; t < n_t; ++t) sq[t][threadIdx.x] = 0.0f;
  int t = 0;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int64_t i = base + (int64_t)k * kT;
    if (i < n) {
      while (i >= a.cfg.offsets[t + 1]) ++t;
      sq[t][threadIdx.x] = fmaf(x[k], x[k], sq[t][threadIdx.x]);
    }
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int u = wave; u < n_t; u += kT / 64) {
    float s = 0.0f;
    for (int k = lane; k < kT; k += 64) s += sq[u][k];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) a.ws[(int64_t)blockIdx.x * n_t + u] = s;
  }
}

__global__ __launch_bounds__(kT) void k_adam_apply(adam_args a) {
  if (a.stop && *a.stop) return;
  const int n_t = a.cfg.n_tensors;
  const int64_t n = a.cfg.offsets[n_t];
  float coef = 1.0f;
  if (a.cfg.max_grad_norm > 0.0) {
    // torch.nn.utils.clip_grad_norm_: total = ||(||g_0||, ..., ||g_k||)||_2,
    // coef = clamp(max_norm / (total + 1e-6), max=1), grads *= coef.
    __shared__ float norms[RX_ADAM_MAX_TENSORS];
    const int nb = (int)((n + kNormElems - 1) / kNormElems);
    if (threadIdx.x < n_t) {
      float s = 0.0f;
      for (int b = 0; b < nb; ++b) s += a.ws[(int64_t)b * n_t + threadIdx.x];
      norms[threadIdx.x] = sqrtf(s);
    }
    __syncthreads();
    float tot2 = 0.0f;
    for (int u = 0; u < n_t; ++u) tot2 += norms[u] * norms[u];
    const float total = sqrtf(tot2);
    coef = fminf((float)a.cfg.max_grad_norm / (total + 1e-6f), 1.0f);
  }
  const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  // torch.optim.Adam (foreach, non-capturable) with step count s (already
  // incremented by k_adam_norm):
  //   m = lerp(m, g, 1-b1); v = v*b2 + (1-b2)*g*g;
  //   p += (-lr/(1-b1^s)) * m / (sqrt(v)/sqrt(1-b2^s) + eps)
  const double s = (double)*a.step;
  const double b1 = a.cfg.beta1, b2 = a.cfg.beta2;
  const float w1 = (float)(1.0 - b1);
  const float fb2 = (float)b2, w2 = (float)(1.0 - b2);
  const float step_size = (float)(-(*a.lr / (1.0 - pow(b1, s))));
  const float bc2_sqrt = (float)sqrt(1.0 - pow(b2, s));
  const float eps = (float)a.cfg.eps;
  const float g = a.g[i] * coef;
  float m = a.m[i];
  float v = a.v[i];
  const float p = a.p[i];
  a.g[i] = g;
  m = m + w1 * (g - m);  // torch.lerp, weight < 0.5 branch
  v = v * fb2;
  v = v + w2 * g * g;
  a.m[i] = m;
  a.v[i] = v;
  const float den = sqrtf(v) / bc2_sqrt + eps;
  a.p[i] = p + step_size * (m / den);
}

}  // namespace

extern "C" int rx_launch_adam(const rx_adam_config* cfg, float* p, float* g, float* m, float* v, float* step,
                              const double* lr, const uint8_t* stop, float* ws, hipStream_t s) {
  adam_args a{*cfg, p, g, m, v, step, lr, stop, ws};
  const int64_t n = cfg->offsets[cfg->n_tensors];
  const int nb_norm = n > 0 ? (int)((n + kNormElems - 1) / kNormElems) : 1;
  hipLaunchKernelGGL(k_adam_norm, dim3(nb_norm), dim3(kT), 0, s, a);
  if (n > 0) hipLaunchKernelGGL(k_adam_apply, dim3((unsigned)((n + kT - 1) / kT)), dim3(kT), 0, s, a);
  return (int)hipGetLastError();
}
