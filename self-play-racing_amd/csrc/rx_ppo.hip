// Fused PPO minibatch gradient (agent/ppo.py:170-203) for the actor-critic MLP
// (agent/ppo.py:11-62): gather -> actor/critic forward -> clipped PG + clipped
// value loss -> backward -> weight gradients, in one kernel, plus a
// deterministic split-K reduce.  Replaces ~100 torch launches per minibatch
// whose weight-gradient GEMMs (M=N<=64, K=minibatch) hipBLASLt runs on a
// handful of workgroups (profiles/r01/ppo_update_kernel_stats.csv).
//
// Layout: one thread = one minibatch row.  Weights are wave-uniform and are
// read through scalar loads (SGPR operands of the FMAs); per-row activations
// live in VGPRs.  Weight gradients dW = sum_r dZ[r] (x) H[r] are formed per
// workgroup (kRows rows) by staging dZ and H in LDS and accumulating register
// tiles, written as one partial per workgroup; k_ppo_reduce sums partials in
// a fixed order (run-to-run deterministic, no float atomics).
#include <hip/hip_runtime.h>

#include "rx.h"

namespace {

constexpr int kH = 64;       // hidden width (agent/ppo.py:20-29)
constexpr int kNA = 2;       // action dims
constexpr int kRows = 256;   // rows per workgroup = threads per workgroup

template <int D>
struct Lay {  // flat parameter offsets, module.parameters() order
  static constexpr int aW1 = 0, ab1 = aW1 + kH * D, aW2 = ab1 + kH, ab2 = aW2 + kH * kH, aW3 = ab2 + kH,
                       ab3 = aW3 + kNA * kH, cW1 = ab3 + kNA, cb1 = cW1 + kH * D, cW2 = cb1 + kH,
                       cb2 = cW2 + kH * kH, cW3 = cb2 + kH, cb3 = cW3 + kH, P = cb3 + 1;
};

struct ppo_args {
  rx_ppo_batch b;
  int32_t m;          // minibatch index within the epoch
  const uint8_t* stop;
  float* partial;     // [n_wg][P]
  double* kl_partial; // [n_wg]
};

// h = tanh(W x + b) for a 64-wide layer; W row-major [64][K] (scalar loads)
template <int K>
__device__ __forceinline__ void dense_tanh(const float* __restrict__ W, const float* __restrict__ bias,
                                           const float* in, float* out) {
#pragma unroll
  for (int i = 0; i < kH; ++i) {
    float z = 0.0f;
#pragma unroll
    for (int k = 0; k < K; ++k) z = fmaf(W[i * K + k], in[k], z);
    out[i] = tanhf(z + bias[i]);
  }
}

// Phase helper: dW[I][J] (+)= sum_r dZ[r][i] * H[r][j] with dZ, H staged in LDS
// ([kRows][I] and [kRows][J]); 4x4 register tiles over (i, j).
template <int I, int J>
__device__ __forceinline__ void acc_tile(const float* __restrict__ dZ, const float* __restrict__ Hs, float* dst,
                                         float* dbias) {
  static_assert(I % 4 == 0 && J % 4 == 0, "tile");
  constexpr int TI = I / 4, TJ = J / 4, NT = TI * TJ;
  for (int t = threadIdx.x; t < NT; t += kRows) {
    const int i0 = (t / TJ) * 4, j0 = (t % TJ) * 4;
    float acc[4][4] = {};
    float bacc[4] = {};
    for (int r = 0; r < kRows; ++r) {
      const float4 z = *reinterpret_cast<const float4*>(dZ + r * I + i0);
      const float4 h = *reinterpret_cast<const float4*>(Hs + r * J + j0);
      const float zz[4] = {z.x, z.y, z.z, z.w}, hh[4] = {h.x, h.y, h.z, h.w};
#pragma unroll
      for (int a = 0; a < 4; ++a) {
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[a][c] = fmaf(zz[a], hh[c], acc[a][c]);
        bacc[a] += zz[a];
      }
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) {
#pragma unroll
      for (int c = 0; c < 4; ++c) dst[(i0 + a) * J + j0 + c] = acc[a][c];
      if (j0 == 0 && dbias) dbias[i0 + a] = bacc[a];
    }
  }
}

// dW1[64][D] with D not a multiple of 4: thread -> (i, d) pairs.
template <int D>
__device__ __forceinline__ void acc_first(const float* __restrict__ dZ, const float* __restrict__ X, float* dst,
                                          float* dbias) {
  for (int e = threadIdx.x; e < kH * D + kH; e += kRows) {
    float s = 0.0f;
    if (e < kH * D) {
      const int i = e / D, d = e % D;
      for (int r = 0; r < kRows; ++r) s = fmaf(dZ[r * kH + i], X[r * D + d], s);
      dst[e] = s;
    } else {
      const int i = e - kH * D;
      for (int r = 0; r < kRows; ++r) s += dZ[r * kH + i];
      dbias[i] = s;
    }
  }
}

// W and partial are separate __restrict__ kernel arguments: the weights are then
// provably never written by this kernel, so the compiler reads them with
// scalar loads (SGPR operands) instead of per-lane vector loads.
template <int D>
__global__ __launch_bounds__(kRows) void k_ppo_grad(ppo_args a, const float* __restrict__ W,
                                                    float* __restrict__ partial) {
  using L = Lay<D>;
  if (a.stop && *a.stop) return;  // KL early stop already hit: nothing to compute
  __shared__ float sA[kRows * kH];
  __shared__ float sB[kRows * kH];
  __shared__ float sX[kRows * D];
  __shared__ double sKL[kRows / 64];
  const rx_ppo_batch& b = a.b;
  float* __restrict__ out = partial + (size_t)blockIdx.x * L::P;
  const int r = threadIdx.x;
  const int row = blockIdx.x * kRows + r;
  int64_t src = row < b.mb ? b.perm[(int64_t)a.m * b.mb + row] : -1;
  const bool live = src >= 0 && src < b.n_rows;  // out-of-range indices contribute nothing
  if (!live) src = 0;

  float x[D];
#pragma unroll
  for (int d = 0; d < D; ++d) x[d] = live ? b.obs[src * D + d] : 0.0f;
  // advantage normalisation with this minibatch's (mean, std), agent/ppo.py:187
  const float mean = b.adv_stats[2 * a.m], sd = b.adv_stats[2 * a.m + 1];
  const float An = live ? (b.advantages[src] - mean) / (sd + 1e-8f) : 0.0f;
  const float invM = 1.0f / (float)b.mb;
  const float lo = 1.0f - b.clip_coef, hi = 1.0f + b.clip_coef;

  // ------------------------------------------------ actor
  float h1[kH], h2[kH];
  dense_tanh<D>(W + L::aW1, W + L::ab1, x, h1);
  dense_tanh<kH>(W + L::aW2, W + L::ab2, h1, h2);
  float mu[kNA];
#pragma unroll
  for (int j = 0; j < kNA; ++j) {
    float z = 0.0f;
#pragma unroll
    for (int k = 0; k < kH; ++k) z = fmaf(W[L::aW3 + j * kH + k], h2[k], z);
    mu[j] = tanhf(z + W[L::ab3 + j]);
  }
  // Normal(mu, exp(log_std)).log_prob(action).sum(-1)  (torch.distributions.Normal)
  float logp = 0.0f, diff[kNA], var[kNA];
#pragma unroll
  for (int j = 0; j < kNA; ++j) {
    const float scale = expf(b.log_std[j]);
    var[j] = scale * scale;
    const float act = live ? b.actions[src * kNA + j] : 0.0f;
    diff[j] = act - mu[j];
    logp += -(diff[j] * diff[j]) / (2.0f * var[j]) - logf(scale) - 0.91893853320467274178f;
  }
  const float oldlp = live ? b.logprobs[src] : 0.0f;
  const float ratio = expf(logp - oldlp);
  // clipped surrogate: max(-A*ratio, -A*clamp(ratio)), torch.max splits ties
  const float u1 = -An * ratio, u2 = -An * fminf(fmaxf(ratio, lo), hi);
  const float g1 = u1 > u2 ? 1.0f : (u1 == u2 ? 0.5f : 0.0f), g2 = 1.0f - g1;
  const float inr = (ratio >= lo && ratio <= hi) ? 1.0f : 0.0f;
  const float dlogp = live ? invM * (g1 * -An + g2 * -An * inr) * ratio : 0.0f;
  float dz3[kNA];
#pragma unroll
  for (int j = 0; j < kNA; ++j) dz3[j] = dlogp * diff[j] / var[j] * (1.0f - mu[j] * mu[j]);

  // KL partial: sum(old_logp - new_logp) over live rows
  {
    double kl = live ? (double)(oldlp - logp) : 0.0;
    for (int o = 32; o > 0; o >>= 1) kl += __shfl_xor(kl, o, 64);
    if ((r & 63) == 0) sKL[r >> 6] = kl;
  }
  // layer 3: dW3 = dz3 (x) h2
#pragma unroll
  for (int k = 0; k < kH; ++k) sA[r * kH + k] = live ? h2[k] : 0.0f;
#pragma unroll
  for (int j = 0; j < kNA; ++j) sB[r * kNA + j] = dz3[j];
#pragma unroll
  for (int d = 0; d < D; ++d) sX[r * D + d] = x[d];
  __syncthreads();
  if (r == 0) {
    double s = 0.0;
    for (int w = 0; w < kRows / 64; ++w) s += sKL[w];
    a.kl_partial[blockIdx.x] = s;
  }
  if (r < kNA * kH) {
    const int j = r / kH, k = r % kH;
    float s = 0.0f;
    for (int q = 0; q < kRows; ++q) s = fmaf(sB[q * kNA + j], sA[q * kH + k], s);
    out[L::aW3 + j * kH + k] = s;
  } else if (r < kNA * kH + kNA) {
    const int j = r - kNA * kH;
    float s = 0.0f;
    for (int q = 0; q < kRows; ++q) s += sB[q * kNA + j];
    out[L::ab3 + j] = s;
  }
  // dz2 = (W3^T dz3) * (1 - h2^2)
#pragma unroll
  for (int k = 0; k < kH; ++k) {
    float s = 0.0f;
#pragma unroll
    for (int j = 0; j < kNA; ++j) s = fmaf(W[L::aW3 + j * kH + k], dz3[j], s);
    h2[k] = live ? s * (1.0f - h2[k] * h2[k]) : 0.0f;  // h2 now holds dz2
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kH; ++k) {
    sA[r * kH + k] = h2[k];                  // dz2
    sB[r * kH + k] = live ? h1[k] : 0.0f;    // h1
  }
  __syncthreads();
  acc_tile<kH, kH>(sA, sB, out + L::aW2, out + L::ab2);
  // dz1 = (W2^T dz2) * (1 - h1^2)
  float dz1[kH];
#pragma unroll
  for (int k = 0; k < kH; ++k) dz1[k] = 0.0f;
#pragma unroll
  for (int i = 0; i < kH; ++i) {
#pragma unroll
    for (int k = 0; k < kH; ++k) dz1[k] = fmaf(W[L::aW2 + i * kH + k], h2[i], dz1[k]);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kH; ++k) sA[r * kH + k] = live ? dz1[k] * (1.0f - h1[k] * h1[k]) : 0.0f;
  __syncthreads();
  acc_first<D>(sA, sX, out + L::aW1, out + L::ab1);

  // ------------------------------------------------ critic
  dense_tanh<D>(W + L::cW1, W + L::cb1, x, h1);
  dense_tanh<kH>(W + L::cW2, W + L::cb2, h1, h2);
  float v = 0.0f;
#pragma unroll
  for (int k = 0; k < kH; ++k) v = fmaf(W[L::cW3 + k], h2[k], v);
  v += W[L::cb3];
  // clipped value loss 0.5 * max((v-R)^2, (v_clip-R)^2), agent/ppo.py:194-198
  const float R = live ? b.returns[src] : 0.0f, ov = live ? b.values[src] : 0.0f;
  const float vd = v - ov;
  const float vc = ov + fminf(fmaxf(vd, -b.clip_coef), b.clip_coef);
  const float e1 = v - R, e2 = vc - R;
  const float q1 = e1 * e1, q2 = e2 * e2;
  const float gq1 = q1 > q2 ? 1.0f : (q1 == q2 ? 0.5f : 0.0f), gq2 = 1.0f - gq1;
  const float vin = (vd >= -b.clip_coef && vd <= b.clip_coef) ? 1.0f : 0.0f;
  const float dv = live ? b.vf_coef * 0.5f * invM * (gq1 * 2.0f * e1 + gq2 * 2.0f * e2 * vin) : 0.0f;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kH; ++k) sA[r * kH + k] = live ? h2[k] : 0.0f;
  sB[r] = dv;
  __syncthreads();
  if (r < kH) {
    float s = 0.0f;
    for (int q = 0; q < kRows; ++q) s = fmaf(sB[q], sA[q * kH + r], s);
    out[L::cW3 + r] = s;
  } else if (r == kH) {
    float s = 0.0f;
    for (int q = 0; q < kRows; ++q) s += sB[q];
    out[L::cb3] = s;
  }
#pragma unroll
  for (int k = 0; k < kH; ++k) h2[k] = live ? W[L::cW3 + k] * dv * (1.0f - h2[k] * h2[k]) : 0.0f;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kH; ++k) {
    sA[r * kH + k] = h2[k];
    sB[r * kH + k] = live ? h1[k] : 0.0f;
  }
  __syncthreads();
  acc_tile<kH, kH>(sA, sB, out + L::cW2, out + L::cb2);
#pragma unroll
  for (int k = 0; k < kH; ++k) dz1[k] = 0.0f;
#pragma unroll
  for (int i = 0; i < kH; ++i) {
#pragma unroll
    for (int k = 0; k < kH; ++k) dz1[k] = fmaf(W[L::cW2 + i * kH + k], h2[i], dz1[k]);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kH; ++k) sA[r * kH + k] = live ? dz1[k] * (1.0f - h1[k] * h1[k]) : 0.0f;
  __syncthreads();
  acc_first<D>(sA, sX, out + L::cW1, out + L::cb1);
}

// grad[p] = sum_w partial[w][p] (fixed order); block 0 also folds the KL
// partials into approx_kl and raises the early-stop flag (agent/ppo.py:178-182).
__global__ __launch_bounds__(256) void k_ppo_reduce(const float* __restrict__ partial, const double* __restrict__ klp,
                                                    int n_wg, int P, int mb, float kl_target, float* grad,
                                                    uint8_t* stop, float* kl_at_stop) {
  if (*stop) return;
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p < P) {
    float s = 0.0f;
    for (int w = 0; w < n_wg; ++w) s += partial[(size_t)w * P + p];
    grad[p] = s;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    double s = 0.0;
    for (int w = 0; w < n_wg; ++w) s += klp[w];
    const float kl = (float)(s / (double)mb);
    if (kl > kl_target) {
      *kl_at_stop = kl;
      *stop = 1;  // read by the optimizer launch that follows on the stream
    }
  }
}

// Per-minibatch (mean, unbiased std) of the advantages, one workgroup per minibatch.
__global__ __launch_bounds__(1024) void k_adv_stats(const float* __restrict__ adv, const int64_t* __restrict__ perm,
                                                    int mb, int64_t n_rows, float* stats) {
  __shared__ double red[2][16];
  const int64_t base = (int64_t)blockIdx.x * mb;
  double s = 0.0, s2 = 0.0;
  for (int i = threadIdx.x; i < mb; i += 1024) {
    const int64_t k = perm[base + i];
    const double x = (k >= 0 && k < n_rows) ? adv[k] : 0.0;
    s += x;
    s2 += x * x;
  }
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o, 64);
    s2 += __shfl_xor(s2, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s;
    red[1][threadIdx.x >> 6] = s2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0, q = 0.0;
    for (int w = 0; w < 16; ++w) {
      a += red[0][w];
      q += red[1][w];
    }
    const double mean = a / mb;
    const double var = mb > 1 ? fmax(q - a * mean, 0.0) / (mb - 1) : 0.0;
    stats[2 * blockIdx.x] = (float)mean;
    stats[2 * blockIdx.x + 1] = (float)sqrt(var);
  }
}

}  // namespace

extern "C" size_t rx_ppo_partial_floats(int obs_dim, int mb) {
  const int P = obs_dim == 15 ? Lay<15>::P : Lay<19>::P;
  return (size_t)((mb + kRows - 1) / kRows) * P;
}

extern "C" int rx_ppo_n_params(int32_t obs_dim) {
  return obs_dim == 15 ? Lay<15>::P : obs_dim == 19 ? Lay<19>::P : 0;
}

extern "C" int rx_launch_adv_stats(const rx_ppo_batch* b, int n_mb, float* stats, hipStream_t s) {
  hipLaunchKernelGGL(k_adv_stats, dim3(n_mb), dim3(1024), 0, s, b->advantages, b->perm, b->mb, b->n_rows, stats);
  return (int)hipGetLastError();
}

extern "C" int rx_launch_ppo_grad(const rx_ppo_batch* b, int m, uint8_t* stop, float* kl_at_stop, float* partial,
                                  double* klp, float* grad, hipStream_t s) {
  const int n_wg = (b->mb + kRows - 1) / kRows;
  ppo_args a{*b, m, stop, partial, klp};
  int P;
  if (b->obs_dim == 15) {
    hipLaunchKernelGGL(k_ppo_grad<15>, dim3(n_wg), dim3(kRows), 0, s, a, b->params, partial);
    P = Lay<15>::P;
  } else {
    hipLaunchKernelGGL(k_ppo_grad<19>, dim3(n_wg), dim3(kRows), 0, s, a, b->params, partial);
    P = Lay<19>::P;
  }
  hipLaunchKernelGGL(k_ppo_reduce, dim3((P + 255) / 256), dim3(256), 0, s, partial, klp, n_wg, P, b->mb,
                     b->kl_target, grad, stop, kl_at_stop);
  return (int)hipGetLastError();
}
