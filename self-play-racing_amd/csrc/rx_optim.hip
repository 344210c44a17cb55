// Fused gradient clipping + Adam step for the PPO update (agent/ppo.py:204-207):
//   nn.utils.clip_grad_norm_(params, max_grad_norm); optimizer.step()
// with torch.optim.Adam(lr, eps=1e-5) (agent/ppo.py:83).  The policy has ~11k
// parameters, so the eager torch path is ~40 launches of a few hundred
// elements each; here it is two launches, each one memory round trip wide:
//   k_adam_norm   per-tensor sums of squares of every 64-entry block of the
//                 gradient -> ws[block][tensor]; bumps the step count and
//                 writes Adam's two bias-correction scalars -> ws[nb * n_t ..];
//   k_adam_apply  one thread per element: its gradient / moment / parameter
//                 loads go out first, then every workgroup folds the norm
//                 partials of each tensor's own blocks in the same order
//                 (per-tensor norms -> global norm -> clip coefficient,
//                 identical in all of them), clips the gradient and applies
//                 Adam to its element.
// The step count, lr and an early-stop flag live in device memory, so the pair
// can sit inside a captured graph.  The fused PPO minibatch update writes the
// same ws (partials + scalars) from k_ppo_reduce (rx_ppo.hip) and launches only
// k_adam_apply.
#include <hip/hip_runtime.h>

#include "rx.h"
#include "rx_internal.h"

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
  float* ws;  // [nb][n_tensors] partial sums of squares, then the 2 Adam scalars
  int nb;     // partial rows in ws
};

// Per-tensor sums of squares in blocks of 64 gradient entries: 16 lanes x 4
// consecutive entries, an fmaf chain per lane, then a 16-lane xor tree --
// exactly the partials k_ppo_reduce writes in the fused minibatch update
// (rx_ppo.hip), so both optimizer paths clip with bit-identical norms.
constexpr int kNormBlock = RX_ADAM_NORM_ELEMS;
__global__ __launch_bounds__(kT) void k_adam_norm(adam_args a) {
  if (a.stop && *a.stop) return;  // uniform: KL early stop already hit
  const int n_t = a.cfg.n_tensors;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const float s = *a.step + 1.0f;
    *a.step = s;  // k_adam_apply reads the new count through the scalars
    rx_adam_scalars(a.cfg, s, *a.lr, a.ws + (size_t)a.nb * n_t);
  }
  if (!(a.cfg.max_grad_norm > 0.0)) return;
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
  const int n_t = a.cfg.n_tensors;
  const int64_t n = a.cfg.offsets[n_t];
  const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
  const bool live = i < n;
  // the element's operands and the step scalars first: one memory round trip
  // that overlaps the norm fold below
  float g = live ? a.g[i] : 0.0f, m = live ? a.m[i] : 0.0f, v = live ? a.v[i] : 0.0f, p = live ? a.p[i] : 0.0f;
  const float step_size = a.ws[(size_t)a.nb * n_t], bc2_sqrt = a.ws[(size_t)a.nb * n_t + 1];
  __shared__ int s_stopped;
  if (threadIdx.x == 0) s_stopped = a.stop ? (int)*a.stop : 0;
  float coef = 1.0f;
  if (a.cfg.max_grad_norm > 0.0) {
    // torch.nn.utils.clip_grad_norm_: total = ||(||g_0||, ..., ||g_k||)||_2,
    // coef = clamp(max_norm / (total + 1e-6), max=1), grads *= coef.
    // Thread group u (16 lanes, u < n_t) folds tensor u: lane j adds the
    // tensor's norm blocks b = b_lo + j, b_lo + j + 16, ... in ascending order
    // (every load of the fold in flight at once: one memory round trip), then a
    // 16-lane xor tree.  Only the blocks the tensor overlaps are read -- every
    // other partial row holds an exact 0 for it -- at nb + n_t loads instead of
    // nb * n_t.  Every workgroup folds identically.
    __shared__ float norms[RX_ADAM_MAX_TENSORS];
    constexpr int kFold = 8;  // blocks per lane in flight (tensors of up to 16 * 8 * 64 entries in one round)
    const int u = threadIdx.x >> 4, j = threadIdx.x & 15;
    float l = 0.0f;
    if (u < n_t) {
      const int64_t lo = a.cfg.offsets[u], hi = a.cfg.offsets[u + 1];
      if (hi > lo) {
        const int b_lo = (int)(lo / kNormBlock), b_hi = (int)((hi - 1) / kNormBlock);
        for (int b0 = b_lo + j; b0 <= b_hi; b0 += 16 * kFold) {
          float v[kFold];
#pragma unroll
          for (int k = 0; k < kFold; ++k) {
            const int b = b0 + 16 * k;
            v[k] = b <= b_hi ? a.ws[(size_t)b * n_t + u] : 0.0f;
          }
#pragma unroll
          for (int k = 0; k < kFold; ++k) l += v[k];
        }
      }
    }
    for (int o = 1; o < 16; o <<= 1) l += __shfl_xor(l, o, 16);
    if (j == 0 && u < n_t) norms[u] = sqrtf(l);
    if (n_t > kT / 16) {  // more tensors than 16-lane groups (rx.h allows 32): the rest, one group each, in turn
      for (int u2 = u + kT / 16; u2 < n_t; u2 += kT / 16) {
        const int64_t lo = a.cfg.offsets[u2], hi = a.cfg.offsets[u2 + 1];
        float l2 = 0.0f;
        if (hi > lo) {
          const int b_lo = (int)(lo / kNormBlock), b_hi = (int)((hi - 1) / kNormBlock);
          for (int b = b_lo + j; b <= b_hi; b += 16) l2 += a.ws[(size_t)b * n_t + u2];
        }
        for (int o = 1; o < 16; o <<= 1) l2 += __shfl_xor(l2, o, 16);
        if (j == 0) norms[u2] = sqrtf(l2);
      }
    }
    __syncthreads();
    float tot2 = 0.0f;
    for (int t = 0; t < n_t; ++t) tot2 += norms[t] * norms[t];
    const float total = sqrtf(tot2);
    coef = fminf((float)a.cfg.max_grad_norm / (total + 1e-6f), 1.0f);
  } else {
    __syncthreads();
  }
  if (s_stopped || !live) return;  // block-uniform stop: KL early stop already hit
  // torch.optim.Adam (foreach, non-capturable) with step count s (the scalars
  // step_size = -lr / (1 - b1^s), bc2_sqrt = sqrt(1 - b2^s) come from ws):
  //   m = lerp(m, g, 1-b1); v = v*b2 + (1-b2)*g*g;
  //   p += step_size * m / (sqrt(v)/bc2_sqrt + eps)
  const double b1 = a.cfg.beta1, b2 = a.cfg.beta2;
  const float w1 = (float)(1.0 - b1);
  const float fb2 = (float)b2, w2 = (float)(1.0 - b2);
  const float eps = (float)a.cfg.eps;
  rx_adam_elem(g, m, v, p, coef, w1, fb2, w2, eps, step_size, bc2_sqrt);
  a.g[i] = g;
  a.m[i] = m;
  a.v[i] = v;
  a.p[i] = p;
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

// The optimizer half of rx_ppo_minibatch_update: the step count was bumped,
// the per-tensor sums of squares written (ws[nb][n_tensors]) and the two Adam
// scalars after them by k_ppo_reduce.
extern "C" int rx_launch_adam_apply(const rx_adam_config* cfg, float* p, float* g, float* m, float* v, float* step,
                                    const double* lr, const uint8_t* stop, float* ws, int nb, hipStream_t s) {
  const int64_t n = cfg->offsets[cfg->n_tensors];
  adam_args a{*cfg, p, g, m, v, step, lr, stop, ws, nb};
  if (n > 0) hipLaunchKernelGGL(k_adam_apply, dim3((unsigned)((n + kT - 1) / kT)), dim3(kT), 0, s, a);
  return (int)hipGetLastError();
}
