// Fused PPO minibatch gradient (agent/ppo.py:170-203) for the actor-critic MLP
// (agent/ppo.py:11-62): gather -> actor/critic forward -> clipped PG + clipped
// value loss -> backward -> weight gradients, in one kernel, plus a
// deterministic split-K reduce.  Replaces ~100 torch launches per minibatch
// whose weight-gradient GEMMs (M=N<=64, K=minibatch) hipBLASLt runs on a
// handful of workgroups (profiles/r01/ppo_update_kernel_stats.csv).
//
// Layout: lane = minibatch row, the 4 waves of a workgroup split the hidden
// columns; weights are wave-uniform and read through scalar loads (SGPR
// operands of the FMAs); activations are staged in LDS (row stride 65, so
// lane-per-row reads are bank-conflict free).  Weight gradients
// dW = sum_r dZ[r] (x) H[r] are register tiles over the LDS-staged rows, added
// into one partial per workgroup (<= 512 per minibatch); k_ppo_reduce sums the
// partials in a fixed order (run-to-run deterministic, no float atomics).
#include <hip/hip_runtime.h>

#include "rx.h"
#include "rx_policy.h"

namespace {

using rx_policy::kH;   // hidden width (agent/ppo.py:20-29)
using rx_policy::kNA;  // action dims
constexpr int kT = 256;  // threads per workgroup (4 waves)
constexpr int kRP = 64;  // rows per pass (lane = row)
constexpr int kS = 65;   // LDS row stride of the [64][64] tiles (lane-per-row reads hit distinct banks)
constexpr int kMaxWG = 512;  // partials per minibatch (rows per workgroup grow beyond that)
constexpr int kSplitNetsBelow = 256;  // workgroups per minibatch below which actor / critic get their own
#ifndef RX_PPO_KQ
#define RX_PPO_KQ 4
#endif
constexpr int kQ = RX_PPO_KQ;  // hidden columns per weight-load group (SGPR budget vs load batching)

using rx_policy::Lay;
using rx_policy::normal_logp;

struct ppo_args {
  rx_ppo_batch b;
  int32_t m;            // minibatch index within the epoch
  int32_t rows_per_wg;  // multiple of kRP
  const uint8_t* stop;
  double* kl_partial;   // [n_wg]
};

__device__ __forceinline__ void put(float* p, float v, bool first) { *p = first ? v : *p + v; }

// The two 64-wide tanh layers of one trunk (agent/ppo.py:20-29) for kRP rows:
// lane = row, wave w computes hidden columns [16w, 16w+16) with the weights as
// SGPR operands; h1 -> sH1, h2 -> sH2 (row stride kS).  Ends with the
// barrier that publishes sH2.
template <int D>
__device__ __forceinline__ void hidden_layers(const float* __restrict__ W, int oW1, int ob1, int oW2, int ob2,
                                              const float* sX, float* sH1, float* sH2, int lane, int w) {
  constexpr int XS = D + 1;
  {
    float x[D];
#pragma unroll
    for (int d = 0; d < D; ++d) x[d] = sX[lane * XS + d];
    for (int cg = 0; cg < 16 / kQ; ++cg) {
      const int c0 = w * 16 + cg * kQ;
      float z[kQ] = {};
#pragma unroll
      for (int d = 0; d < D; ++d) {
#pragma unroll
        for (int q = 0; q < kQ; ++q) z[q] = fmaf(W[oW1 + (c0 + q) * D + d], x[d], z[q]);
      }
#pragma unroll
      for (int q = 0; q < kQ; ++q) sH1[lane * kS + c0 + q] = tanhf(z[q] + W[ob1 + c0 + q]);
    }
  }
  __syncthreads();
  {
    float h[kH];
#pragma unroll
    for (int k = 0; k < kH; ++k) h[k] = sH1[lane * kS + k];
    for (int cg = 0; cg < 16 / kQ; ++cg) {
      const int c0 = w * 16 + cg * kQ;
      float z[kQ] = {};
#pragma unroll
      for (int k = 0; k < kH; ++k) {
#pragma unroll
        for (int q = 0; q < kQ; ++q) z[q] = fmaf(W[oW2 + (c0 + q) * kH + k], h[k], z[q]);
      }
#pragma unroll
      for (int q = 0; q < kQ; ++q) sH2[lane * kS + c0 + q] = tanhf(z[q] + W[ob2 + c0 + q]);
    }
  }
  __syncthreads();
}

// One workgroup = rows_per_wg minibatch rows, processed kRP at a time, of both
// networks (actor, then critic) -- or, when the minibatch gives fewer than
// kSplitNetsBelow workgroups, of ONE network (blockIdx.y: 0 = actor, 1 =
// critic; their losses share no parameter, so the two backward passes are
// independent workgroups writing disjoint ranges of the same partial row: a
// latency-bound small minibatch then runs twice the workgroups, each half the
// chain).  Per pass and network:
//   forward  : wave w computes hidden columns [16w, 16w+16) for the 64 rows
//              (lane = row), weights as SGPR operands, outputs to LDS;
//   head     : wave 0 computes mu / value and the loss gradient per row;
//   backward : dZ2 / dZ1 likewise column-split over waves;
//   dW       : LDS-staged register tiles over the pass's rows, added into the
//              workgroup's partial (each entry owned by one thread).
template <int D>
__global__ __launch_bounds__(kT, 2) void k_ppo_grad(ppo_args a, const float* __restrict__ W,
                                                    float* __restrict__ partial) {
  using L = Lay<D>;
  constexpr int XS = D + 1;
  if (a.stop && *a.stop) return;  // KL early stop already hit: nothing to compute
  __shared__ float sX[kRP * XS];
  __shared__ float sH1[kRP * kS];
  __shared__ float sH2[kRP * kS];
  __shared__ float sDZ[kRP * kS];
  __shared__ float sHead[kRP * kNA];
  __shared__ int64_t sSrc[kRP];
  const rx_ppo_batch& b = a.b;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);  // wave index, provably uniform
  float* __restrict__ out = partial + (size_t)blockIdx.x * L::Pp;
  const int64_t row0 = (int64_t)blockIdx.x * a.rows_per_wg;
  const int64_t row_end = min(row0 + (int64_t)a.rows_per_wg, (int64_t)b.mb);
  const float mean = b.adv_stats[2 * a.m], sd = b.adv_stats[2 * a.m + 1];
  const float invM = 1.0f / (float)b.mb;
  const float clip = b.clip_coef, lo = 1.0f - clip, hi = 1.0f + clip;
  double kl = 0.0;
  bool first = true;
  // gridDim.y == 2: this workgroup's network only (small minibatches: twice the
  // workgroups, half the chain each); 1: both networks, actor then critic
  const int net0 = gridDim.y == 2 ? (int)blockIdx.y : 0, net1 = gridDim.y == 2 ? net0 + 1 : 2;
  for (int64_t base = row0; base < row_end; base += kRP, first = false) {
    if (t < kRP) {
      int64_t src = base + t < row_end ? b.perm[(int64_t)a.m * b.mb + base + t] : -1;
      sSrc[t] = (src >= 0 && src < b.n_rows) ? src : -1;  // out-of-range indices contribute nothing
    }
    __syncthreads();
    for (int e = t; e < kRP * D; e += kT) {
      const int r = e / D, d = e - r * D;
      const int64_t src = sSrc[r];
      sX[r * XS + d] = src >= 0 ? b.obs[src * D + d] : 0.0f;
    }
    const int64_t src = sSrc[lane];
    const bool live = src >= 0;
    __syncthreads();
    for (int net = net0; net < net1; ++net) {
      const int oW1 = net ? L::cW1 : L::aW1, ob1 = net ? L::cb1 : L::ab1;
      const int oW2 = net ? L::cW2 : L::aW2, ob2 = net ? L::cb2 : L::ab2;
      const int oW3 = net ? L::cW3 : L::aW3, ob3 = net ? L::cb3 : L::ab3;
      const int n_out = net ? 1 : kNA;
      hidden_layers<D>(W, oW1, ob1, oW2, ob2, sX, sH1, sH2, lane, w);
      // ---- head and loss gradient (wave 0, lane = row)
      if (w == 0) {
        float h[kH];
#pragma unroll
        for (int k = 0; k < kH; ++k) h[k] = sH2[lane * kS + k];
        if (net == 0) {
          // Normal(mu, exp(log_std)).log_prob(action).sum(-1); clipped surrogate
          float mu[kNA], diff[kNA], var[kNA], logp = 0.0f;
#pragma unroll
          for (int j = 0; j < kNA; ++j) {
            float z = 0.0f;
#pragma unroll
            for (int k = 0; k < kH; ++k) z = fmaf(W[oW3 + j * kH + k], h[k], z);
            mu[j] = tanhf(z + W[ob3 + j]);
            const float scale = expf(b.log_std[j]);
            var[j] = scale * scale;
            diff[j] = (live ? b.actions[src * kNA + j] : 0.0f) - mu[j];
            logp += normal_logp(diff[j], var[j], logf(scale));
          }
          const float oldlp = live ? b.logprobs[src] : 0.0f;
          const float An = live ? (b.advantages[src] - mean) / (sd + 1e-8f) : 0.0f;
          const float ratio = expf(logp - oldlp);
          const float u1 = -An * ratio, u2 = -An * fminf(fmaxf(ratio, lo), hi);
          const float g1 = u1 > u2 ? 1.0f : (u1 == u2 ? 0.5f : 0.0f), g2 = 1.0f - g1;  // torch.max splits ties
          const float inr = (ratio >= lo && ratio <= hi) ? 1.0f : 0.0f;
          const float dlogp = live ? invM * (g1 * -An + g2 * -An * inr) * ratio : 0.0f;
#pragma unroll
          for (int j = 0; j < kNA; ++j) sHead[lane * kNA + j] = dlogp * diff[j] / var[j] * (1.0f - mu[j] * mu[j]);
          if (live) kl += (double)(oldlp - logp);
        } else {
          float v = 0.0f;
#pragma unroll
          for (int k = 0; k < kH; ++k) v = fmaf(W[oW3 + k], h[k], v);
          v += W[ob3];
          // 0.5 * max((v-R)^2, (v_clip-R)^2), agent/ppo.py:194-198
          const float R = live ? b.returns[src] : 0.0f, ov = live ? b.values[src] : 0.0f;
          const float vd = v - ov;
          const float vc = ov + fminf(fmaxf(vd, -clip), clip);
          const float e1 = v - R, e2 = vc - R;
          const float q1 = e1 * e1, q2 = e2 * e2;
          const float gq1 = q1 > q2 ? 1.0f : (q1 == q2 ? 0.5f : 0.0f), gq2 = 1.0f - gq1;
          const float vin = (vd >= -clip && vd <= clip) ? 1.0f : 0.0f;
          sHead[lane] = live ? b.vf_coef * 0.5f * invM * (gq1 * 2.0f * e1 + gq2 * 2.0f * e2 * vin) : 0.0f;
        }
      }
      __syncthreads();
      // ---- dW3 / db3 = sum_r head[r] (x) h2[r]
      if (t < n_out * kH) {
        const int j = t / kH, k = t - j * kH;
        float s = 0.0f;
        for (int r = 0; r < kRP; ++r) s = fmaf(sHead[r * n_out + j], sH2[r * kS + k], s);
        put(out + oW3 + t, s, first);
      } else if (t < n_out * kH + n_out) {
        const int j = t - n_out * kH;
        float s = 0.0f;
        for (int r = 0; r < kRP; ++r) s += sHead[r * n_out + j];
        put(out + ob3 + j, s, first);
      }
      // ---- dz2 = (W3^T head) * (1 - h2^2), columns [16w, 16w+16)
      for (int q = 0; q < 16; ++q) {
        const int k = w * 16 + q;
        float dh = 0.0f;
        for (int j = 0; j < n_out; ++j) dh = fmaf(sHead[lane * n_out + j], W[oW3 + j * kH + k], dh);
        const float h2 = sH2[lane * kS + k];
        sDZ[lane * kS + k] = dh * (1.0f - h2 * h2);
      }
      __syncthreads();
      // ---- dW2 / db2 = sum_r dz2[r] (x) h1[r]: 4x4 tile per thread
      {
        const int c0 = (t >> 4) * 4, k0 = (t & 15) * 4;
        float acc[4][4] = {}, bacc[4] = {};
        for (int r = 0; r < kRP; ++r) {
          float dz[4], hh[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            dz[q] = sDZ[r * kS + c0 + q];
            hh[q] = sH1[r * kS + k0 + q];
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) {
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[i][q] = fmaf(dz[i], hh[q], acc[i][q]);
            bacc[i] += dz[i];
          }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
          for (int q = 0; q < 4; ++q) put(out + oW2 + (c0 + i) * kH + k0 + q, acc[i][q], first);
          if (k0 == 0) put(out + ob2 + c0 + i, bacc[i], first);
        }
      }
      // ---- dz1 = (W2^T dz2) * (1 - h1^2), columns [16w, 16w+16) -> sH2 (h2 is dead)
      {
        float dz[kH];
#pragma unroll
        for (int c = 0; c < kH; ++c) dz[c] = sDZ[lane * kS + c];
        for (int kg = 0; kg < 16 / kQ; ++kg) {
          const int k0 = w * 16 + kg * kQ;
          float acc[kQ] = {};
#pragma unroll
          for (int c = 0; c < kH; ++c) {
#pragma unroll
            for (int q = 0; q < kQ; ++q) acc[q] = fmaf(W[oW2 + c * kH + k0 + q], dz[c], acc[q]);
          }
#pragma unroll
          for (int q = 0; q < kQ; ++q) {
            const float h1 = sH1[lane * kS + k0 + q];
            sH2[lane * kS + k0 + q] = acc[q] * (1.0f - h1 * h1);
          }
        }
      }
      __syncthreads();
      // ---- dW1 / db1 = sum_r dz1[r] (x) x[r]
      for (int e = t; e < kH * D + kH; e += kT) {
        float s = 0.0f;
        if (e < kH * D) {
          const int c = e / D, d = e - c * D;
          for (int r = 0; r < kRP; ++r) s = fmaf(sH2[r * kS + c], sX[r * XS + d], s);
          put(out + oW1 + e, s, first);
        } else {
          const int c = e - kH * D;
          for (int r = 0; r < kRP; ++r) s += sH2[r * kS + c];
          put(out + ob1 + c, s, first);
        }
      }
      __syncthreads();
    }
  }
  if (w == 0 && net0 == 0) {
    for (int o = 32; o > 0; o >>= 1) kl += __shfl_xor(kl, o, 64);
    if (lane == 0) a.kl_partial[blockIdx.x] = kl;
  }
}

// Rollout policy step (agent/ppo.py:105-110, get_action_and_value on obs[t]):
// actor + critic forward for kRP rows per workgroup, then per row
//   action = clamp(eps * std + mu, -1, 1)        (Normal.sample() = normal_() * std + mu)
//   logp   = sum_j Normal(mu, std).log_prob(action_j),  value = critic(obs)
// eps [N][2] is drawn by the caller with torch's normal_() so the sampling
// stream is torch's.  Outputs go straight into the rollout buffers.
template <int D>
__global__ __launch_bounds__(kT, 2) void k_policy_act(rx_policy_io io, const float* __restrict__ W) {
  // blockIdx.y = trunk: 0 = actor (mu -> action, log-prob), 1 = critic (value);
  // the two trunks are independent, so they run as separate workgroups
  using L = Lay<D>;
  constexpr int XS = D + 1;
  __shared__ float sX[kRP * XS];
  __shared__ float sH1[kRP * kS];
  __shared__ float sH2[kRP * kS];
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const bool critic = blockIdx.y != 0;
  const int64_t base = (int64_t)blockIdx.x * kRP;
  const int64_t row = base + lane;
  const bool live = row < io.n;
  const int64_t os = io.obs_stride > 0 ? io.obs_stride : D, as = io.act_stride > 0 ? io.act_stride : kNA;
  for (int e = t; e < kRP * D; e += kT) {
    const int r = e / D, d = e - r * D;
    sX[r * XS + d] = base + r < io.n ? io.obs[(base + r) * os + d] : 0.0f;
  }
  __syncthreads();
  if (!critic) {
    hidden_layers<D>(W, L::aW1, L::ab1, L::aW2, L::ab2, sX, sH1, sH2, lane, w);
    if (w != 0 || !live) return;
    float h[kH];
#pragma unroll
    for (int k = 0; k < kH; ++k) h[k] = sH2[lane * kS + k];
    float logp = 0.0f;
#pragma unroll
    for (int j = 0; j < kNA; ++j) {
      float z = 0.0f;
#pragma unroll
      for (int k = 0; k < kH; ++k) z = fmaf(W[L::aW3 + j * kH + k], h[k], z);
      const float mu = tanhf(z + W[L::ab3 + j]);
      const float scale = expf(io.log_std[j]);
      const float var = scale * scale;
      const float smp = io.eps[row * kNA + j] * scale + mu;  // mul_(std).add_(mu): two roundings
      const float a = fminf(fmaxf(smp, -1.0f), 1.0f);
      io.actions[row * as + j] = a;
      logp += normal_logp(a - mu, var, logf(scale));
    }
    io.logprobs[row] = logp;
  } else {
    hidden_layers<D>(W, L::cW1, L::cb1, L::cW2, L::cb2, sX, sH1, sH2, lane, w);
    if (w != 0 || !live) return;
    float v = 0.0f;
#pragma unroll
    for (int k = 0; k < kH; ++k) v = fmaf(W[L::cW3 + k], sH2[lane * kS + k], v);
    io.values[row] = v + W[L::cb3];
  }
}

// grad[p] = sum_w partial[w][p] in a fixed order.  One workgroup owns 64
// parameters (16 float4 columns) and reads the partial rows in 64 interleaved
// slices (a wave reads four 256-byte row pieces), so the ~Pp/64 workgroups
// stream the partials from most CUs; the slices are combined in slice order.
// Block 0's wave 1 also folds the KL partials into approx_kl and raises the
// early-stop flag (agent/ppo.py:178-182).  Partials have row stride Pp (P
// rounded up to 64) so every row is float4-aligned.
constexpr int kRedCols = 16;                    // float4 columns per workgroup
constexpr int kRedSlices = 1024 / kRedCols;     // 64
constexpr int kRedBatch = 8;                    // partial rows loaded per thread per round trip
__global__ __launch_bounds__(1024) void k_ppo_reduce(const float* __restrict__ partial,
                                                     const double* __restrict__ klp, int n_wg, int P, int Pp, int mb,
                                                     float kl_target, float scale, float* grad, uint8_t* stop,
                                                     float* kl_at_stop, float* kl_out) {
  if (*stop) return;
  __shared__ float4 red[kRedSlices][kRedCols];
  const int c = threadIdx.x % kRedCols, sl = threadIdx.x / kRedCols;
  const int p4 = blockIdx.x * (4 * kRedCols) + c * 4;  // first of this thread's 4 parameters
  float4 s = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  if (p4 < Pp)
    for (int w0 = sl; w0 < n_wg; w0 += kRedBatch * kRedSlices) {
      float4 v[kRedBatch];  // independent loads first: one memory round trip per batch
#pragma unroll
      for (int k = 0; k < kRedBatch; ++k) {
        const int w = w0 + k * kRedSlices;
        v[k] = w < n_wg ? *reinterpret_cast<const float4*>(partial + (size_t)w * Pp + p4)
                        : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      }
#pragma unroll
      for (int k = 0; k < kRedBatch; ++k) {
        s.x += v[k].x;
        s.y += v[k].y;
        s.z += v[k].z;
        s.w += v[k].w;
      }
    }
  red[sl][c] = s;
  __syncthreads();
  // slices -> 8 groups (group q sums slices q, q+8, ...) -> column total, in order
  __shared__ float4 red2[8][kRedCols];
  if (sl < 8) {
    float4 t = red[sl][c];
    for (int k = sl + 8; k < kRedSlices; k += 8) {
      const float4 v = red[k][c];
      t.x += v.x;
      t.y += v.y;
      t.z += v.z;
      t.w += v.w;
    }
    red2[sl][c] = t;
  }
  __syncthreads();
  if (threadIdx.x < kRedCols && p4 < P) {
    float4 t = red2[0][c];
    for (int k = 1; k < 8; ++k) {
      const float4 v = red2[k][c];
      t.x += v.x;
      t.y += v.y;
      t.z += v.z;
      t.w += v.w;
    }
    const float o[4] = {t.x, t.y, t.z, t.w};
    for (int q = 0; q < 4 && p4 + q < P; ++q) grad[p4 + q] = o[q] * scale;
  }
  const int lane = threadIdx.x & 63;
  if (blockIdx.x == 0 && (threadIdx.x >> 6) == 1) {
    double k = 0.0;
    for (int w = lane; w < n_wg; w += 64) k += klp[w];
    for (int o = 32; o > 0; o >>= 1) k += __shfl_xor(k, o, 64);
    const float kl = (float)(k / (double)mb);
    if (kl_out) {  // shard mode: this rank's share of the global KL, decided after the all-reduce
      if (lane == 0) *kl_out = kl * scale;
    } else if (lane == 0 && kl > kl_target) {
      *kl_at_stop = kl;
      *stop = 1;  // read by the optimizer launch that follows on the stream
    }
  }
}

// Per-minibatch (mean, unbiased std) of the advantages, one workgroup per
// minibatch; with ``moments`` set it writes the raw (sum, square-sum) instead,
// for the cross-rank all-reduce of a data-parallel update (same summation
// order, so moments -> k_adv_finalize == this kernel's stats bit for bit).
__device__ __forceinline__ void adv_write(double a, double q, double count, float* stats, int i) {
  const double mean = a / count;
  const double var = count > 1.0 ? fmax(q - a * mean, 0.0) / (count - 1.0) : 0.0;
  stats[2 * i] = (float)mean;
  stats[2 * i + 1] = (float)sqrt(var);
}

__global__ __launch_bounds__(1024) void k_adv_stats(const float* __restrict__ adv, const int64_t* __restrict__ perm,
                                                    int mb, int64_t n_rows, float* stats, double* moments) {
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
    if (moments) {
      moments[2 * blockIdx.x] = a;
      moments[2 * blockIdx.x + 1] = q;
    } else {
      adv_write(a, q, (double)mb, stats, blockIdx.x);
    }
  }
}

// (mean, unbiased std) of every minibatch from all-reduced moments over ``count`` rows.
__global__ __launch_bounds__(64) void k_adv_finalize(const double* __restrict__ moments, int n_mb, double count,
                                                     float* stats) {
  for (int i = threadIdx.x; i < n_mb; i += 64) adv_write(moments[2 * i], moments[2 * i + 1], count, stats, i);
}

// The data-parallel KL early stop (agent/ppo.py:178-182) on the all-reduced
// mean KL: raise *stop for the rx_adam_clip_step that follows.
__global__ __launch_bounds__(64) void k_kl_check(const float* __restrict__ kl, float kl_target, uint8_t* stop,
                                                 float* kl_at_stop) {
  if (threadIdx.x == 0 && !*stop && *kl > kl_target) {
    *kl_at_stop = *kl;
    *stop = 1;
  }
}

}  // namespace

static int rows_per_wg(int mb) {
  const int passes = (mb + kRP * kMaxWG - 1) / (kRP * kMaxWG);
  return kRP * (passes < 1 ? 1 : passes);
}

extern "C" int rx_ppo_n_wg(int mb) {
  const int rp = rows_per_wg(mb);
  return (mb + rp - 1) / rp;
}

extern "C" size_t rx_ppo_partial_floats(int obs_dim, int mb) {
  const int P = obs_dim == 15 ? Lay<15>::Pp : Lay<19>::Pp;
  const int rp = rows_per_wg(mb);
  return (size_t)((mb + rp - 1) / rp) * P;
}

extern "C" int rx_ppo_n_params(int32_t obs_dim) {
  return obs_dim == 15 ? Lay<15>::P : obs_dim == 19 ? Lay<19>::P : 0;
}

extern "C" int rx_launch_adv_stats(const rx_ppo_batch* b, int n_mb, float* stats, double* moments, hipStream_t s) {
  hipLaunchKernelGGL(k_adv_stats, dim3(n_mb), dim3(1024), 0, s, b->advantages, b->perm, b->mb, b->n_rows, stats,
                     moments);
  return (int)hipGetLastError();
}

extern "C" int rx_launch_adv_finalize(const double* moments, int n_mb, int64_t count, float* stats, hipStream_t s) {
  hipLaunchKernelGGL(k_adv_finalize, dim3(1), dim3(64), 0, s, moments, n_mb, (double)count, stats);
  return (int)hipGetLastError();
}

extern "C" int rx_launch_kl_check(const float* kl, float kl_target, uint8_t* stop, float* kl_at_stop, hipStream_t s) {
  hipLaunchKernelGGL(k_kl_check, dim3(1), dim3(64), 0, s, kl, kl_target, stop, kl_at_stop);
  return (int)hipGetLastError();
}

extern "C" int rx_launch_ppo_grad(const rx_ppo_batch* b, int m, float scale, uint8_t* stop, float* kl_at_stop,
                                  float* kl_out, float* partial, double* klp, float* grad, hipStream_t s) {
  const int rp = rows_per_wg(b->mb);
  const int n_wg = (b->mb + rp - 1) / rp;
  const int ny = n_wg < kSplitNetsBelow ? 2 : 1;
  ppo_args a{*b, m, rp, stop, klp};
  int P, Pp;
  if (b->obs_dim == 15) {
    hipLaunchKernelGGL(k_ppo_grad<15>, dim3(n_wg, ny), dim3(kT), 0, s, a, b->params, partial);
    P = Lay<15>::P, Pp = Lay<15>::Pp;
  } else {
    hipLaunchKernelGGL(k_ppo_grad<19>, dim3(n_wg, ny), dim3(kT), 0, s, a, b->params, partial);
    P = Lay<19>::P, Pp = Lay<19>::Pp;
  }
  hipLaunchKernelGGL(k_ppo_reduce, dim3((Pp + 4 * kRedCols - 1) / (4 * kRedCols)), dim3(1024), 0, s, partial, klp, n_wg, P, Pp, b->mb,
                     b->kl_target, scale, grad, stop, kl_at_stop, kl_out);
  return (int)hipGetLastError();
}

extern "C" int rx_launch_policy_act(const rx_policy_io* io, hipStream_t s) {
  const int n_wg = (int)((io->n + kRP - 1) / kRP);
  if (io->obs_dim == 15)
    hipLaunchKernelGGL(k_policy_act<15>, dim3(n_wg, 2), dim3(kT), 0, s, *io, io->params);
  else
    hipLaunchKernelGGL(k_policy_act<19>, dim3(n_wg, 2), dim3(kT), 0, s, *io, io->params);
  return (int)hipGetLastError();
}
