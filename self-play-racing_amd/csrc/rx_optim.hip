// Fused gradient clipping + Adam step for the PPO update (agent/ppo.py:204-207):
//   nn.utils.clip_grad_norm_(params, max_grad_norm); optimizer.step()
// with torch.optim.Adam(lr, eps=1e-5) (agent/ppo.py:83).  The policy has ~11k
// parameters, so the eager torch path is ~40 launches of a few hundred
// elements each; here it is two launches, each one memory round trip wide:
//   k_adam_norm   per-tensor sums of squares of every 64-entry block of the
//                 gradient -> ws[block][tensor]; bumps the step count;
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

struct adam_args {
  rx_adam_config cfg;
  float* p;
  float* g;
  float* m;
  float* v;
  float* step;
  const double* lr;
  const uint8_t* stop;
  float* ws;  // [nb][n_tensors] partial sums of squares
  int nb;     // partial rows in ws
};

// Per-tensor sums of squares in blocks of 64 gradient entries: 16 lanes x 4
// consecutive entries, an fmaf chain per lane, then a 16-lane xor tree --
// exactly the partials k_ppo_reduce writes in the fused minibatch update
// (rx_ppo.hip), so both optimizer paths clip with bit-identical norms.
constexpr int kNormBlock = 64;
__global__ __launch_bounds__(kT) void k_adam_norm(adam_args a) {
  if (a.stop && *a.stop) return;  // uniform: KL early stop already hit
  if (blockIdx.x == 0 && threadIdx.x == 0) *a.step += 1.0f;  // k_adam_apply reads the new count
  if (!(a.cfg.max_grad_norm > 0.0)) return;
  const int n_t = a.cfg.n_tensors;
  const int64_t n = a.cfg.offsets[n_t];
  const int64_t blk = (int64_t)blockIdx.x * (kT / 16) + (threadIdx.x >> 4);  // 64-entry block of this lane group
  if (blk >= a.nb) return;  // whole 16-lane groups
  const int64_t p4 = blk * kNormBlock + 4 * (threadIdx.x & 15);
  float g[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) g[k] = p4 + k < n ? a.g[p4 + k] : 0.0f;
  const int64_t b0 = blk * kNormBlock, b1 = b0 + kNormBlock;
  for (int u = 0; u < n_t; ++u) {
    const int64_t lo = a.cfg.offsets[u], hi = a.cfg.offsets[u + 1];
    if (hi <= b0 || lo >= b1) {  // tensor outside this block (uniform over the 16 lanes)
      if ((threadIdx.x & 15) == 0) a.ws[blk * n_t + u] = 0.0f;
      continue;
    }
    float sq = 0.0f;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (p4 + k < n && p4 + k >= lo && p4 + k < hi) sq = fmaf(g[k], g[k], sq);
    for (int off = 1; off < 16; off <<= 1) sq += __shfl_xor(sq, off, 16);
    if ((threadIdx.x & 15) == 0) a.ws[blk * n_t + u] = sq;
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
    // Every workgroup folds the nb partial rows in the same fixed order.
    // Every workgroup folds the nb partial rows the same way: the [nb][n_t]
    // partials staged in LDS (coalesced, all loads in flight), then wave w sums
    // tensors w, w + 4, ...: lane l adds rows l, l + 64, ... in order, a 64-lane
    // xor tree finishes.
    constexpr int kMaxPart = 8192;  // LDS floats for the partials
    __shared__ float part[kMaxPart];
    __shared__ float norms[RX_ADAM_MAX_TENSORS];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int tot = a.nb * n_t;
    for (int c0 = 0; c0 < tot; c0 += kMaxPart) {  // one chunk unless nb * n_t > kMaxPart
      const int c1 = min(tot, c0 + kMaxPart);
      for (int e = c0 + threadIdx.x; e < c1; e += kT) part[e - c0] = a.ws[e];
      __syncthreads();
      for (int u = wave; u < n_t; u += kT / 64) {
        float s = c0 ? norms[u] : 0.0f;  // running total over the chunks
        float l = 0.0f;
        for (int b = lane; b < a.nb; b += 64) {
          const int e = b * n_t + u;
          if (e >= c0 && e < c1) l += part[e - c0];
        }
        for (int o = 32; o > 0; o >>= 1) l += __shfl_xor(l, o, 64);
        if (lane == 0) norms[u] = s + l;
      }
      __syncthreads();
    }
    if (threadIdx.x < n_t) norms[threadIdx.x] = sqrtf(norms[threadIdx.x]);
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
  const int64_t n = cfg->offsets[cfg->n_tensors];
  const int nb = n > 0 ? (int)((n + kNormBlock - 1) / kNormBlock) : 1;  // 64-entry norm blocks
  adam_args a{*cfg, p, g, m, v, step, lr, stop, ws, nb};
  hipLaunchKernelGGL(k_adam_norm, dim3((nb + kT / 16 - 1) / (kT / 16)), dim3(kT), 0, s, a);
  if (n > 0) hipLaunchKernelGGL(k_adam_apply, dim3((unsigned)((n + kT - 1) / kT)), dim3(kT), 0, s, a);
  return (int)hipGetLastError();
}

// The optimizer half of rx_ppo_minibatch_update: the step count was bumped and
// the per-tensor sums of squares written (ws[nb][n_tensors]) by k_ppo_reduce.
extern "C" int rx_launch_adam_apply(const rx_adam_config* cfg, float* p, float* g, float* m, float* v, float* step,
                                    const double* lr, const uint8_t* stop, float* ws, int nb, hipStream_t s) {
  const int64_t n = cfg->offsets[cfg->n_tensors];
  adam_args a{*cfg, p, g, m, v, step, lr, stop, ws, nb};
  if (n > 0) hipLaunchKernelGGL(k_adam_apply, dim3((unsigned)((n + kT - 1) / kT)), dim3(kT), 0, s, a);
  return (int)hipGetLastError();
}
