// Fused PPO minibatch gradient (agent/ppo.py:170-203) and the rollout policy
// step (agent/ppo.py:105-110) for the actor-critic MLP (agent/ppo.py:11-62),
// on the f32-input matrix cores: v_mfma_f32_16x16x4_f32 is bit for bit a
// k-ordered fmaf chain (exact f32, 64 FLOP/clk/SIMD), so every dot product
// here is a DEFINED fmaf chain whose order k_rollout (rx_kernels.hip) repeats
// with VALU fmaf to stay bit-identical with rx_policy_act.
//
// Orientation: activations are kept TRANSPOSED, hidden unit = MFMA row, batch
// row = MFMA column.  A 16x16 output tile leaves lane l holding batch row
// l & 15 and hidden units 16*tile + 4*(l >> 4) + r in its 4 registers, which
// is exactly the B-operand fragment of the next layer if that layer's k-steps
// are ordered (tile t, register r) and an MFMA's 4-wide k index is the lane
// group q = l >> 4: hidden unit h = 16t + 4q + r.  So Z1 -> H1 -> Z2 -> H2 ->
// head, and dZ2 -> dH1, chain in registers with no LDS transposes; the weight
// operand of each step is read in the matching permuted order.  Every sum
// over hidden units therefore runs in the order t, r, q (h = 16t + 4q + r);
// over input features in the natural order d = 0 .. D-1 (zero-padded to 4k).
//
// k_ppo_grad: a workgroup (4 waves) owns rows_per_wg minibatch rows of ONE
// trunk (blockIdx.y: actor or critic), 64 per pass, 16 per wave for the
// forward / loss / dZ2 / dH1 chains.  Weight gradients sum over batch rows,
// which sit on lanes, so their operands go through LDS transposes of the
// pass's 64 rows ([hidden][row]) and the MFMA k index becomes the row; wave w
// owns output rows [16w, 16w+16) of dW2 and of dW1 (+ db1: a ones column at
// d = D of the input tile), so the tile accumulators go straight to the
// workgroup's partial row.  db2, dW3, db3 and the KL are per-wave sums (lane =
// hidden unit) folded in a fixed order; k_ppo_reduce sums the partial rows in a
// fixed order (run-to-run deterministic, no float atomics).
#include <hip/hip_runtime.h>

#include "rx.h"
#include "rx_internal.h"
#include "rx_policy.h"

// Profiling build only (-DRX_PPO_STAMPS, tools/ppo_stamps.py): per-wave
// s_memtime stamps at k_ppo_grad's phase boundaries into a device array read
// by rx_ppo_stamps_read (exported by that build only).  The product library has
// no stamps.
#ifdef RX_PPO_STAMPS
constexpr int kStampW = 24, kStampMaxWaves = 8192;
__device__ unsigned long long g_ppo_stamps[kStampMaxWaves * kStampW];
#define PPO_STAMP(j)                                                                                       \
  do {                                                                                                     \
    const int sw_ = ((int)(blockIdx.y * gridDim.x + blockIdx.x) * (int)(blockDim.x >> 6) + (int)(threadIdx.x >> 6)); \
    if ((threadIdx.x & 63) == 0 && sw_ < kStampMaxWaves && (j) < kStampW)                                \
      g_ppo_stamps[sw_ * kStampW + (j)] = __builtin_amdgcn_s_memtime();                                   \
  } while (0)
#else
#define PPO_STAMP(j) \
  do {               \
  } while (0)
#endif

#include "rx_policy_mfma.h"

namespace {

using rx_policy::kH;   // hidden width (agent/ppo.py:20-29)
using rx_policy::kNA;  // action dims
constexpr int kT = 256;      // k_policy_act: threads per workgroup (4 waves)
// k_ppo_grad workgroup: RX_PPO_NW waves (4 or 8), 16 rows each per pass.  With
// 8 waves one workgroup per CU stages its trunk's weights (half the prologue
// traffic of two 4-wave workgroups) and the minibatch has half the partial rows;
// measured no faster (the 8-wave barriers wait longer: minibatch step 39.5-40.3
// vs 40.5-40.7 us, profiles/r03/ab_ppo_grad_8_waves.json), so 4 is the default
// and 8 an A/B build (bit-exact tests pass with either).
#ifndef RX_PPO_NW
#define RX_PPO_NW 4
#endif
constexpr int kGW = RX_PPO_NW;
static_assert(kGW == 4 || kGW == 8, "k_ppo_grad: 4 or 8 waves per workgroup");
constexpr int kGT = 64 * kGW;  // k_ppo_grad threads per workgroup
constexpr int kRP = 16 * kGW;  // rows per workgroup pass (16 per wave)
#ifndef RX_PPO_MAXWG
#define RX_PPO_MAXWG (RX_PPO_NW == 8 ? 128 : 256)
#endif
constexpr int kMaxWG = RX_PPO_MAXWG;  // row workgroups per minibatch and trunk (rows per workgroup grow beyond that)
constexpr int kWS = 68;      // LDS row stride of W2 [o][i] (float4-aligned; transposed reads conflict-free)
constexpr int kTS = kRP + 2;  // LDS row stride of the [hidden][row] transposes (= 2 mod 64: operand reads conflict-free)
#ifndef RX_PPO_MINW
#define RX_PPO_MINW 2  // k_ppo_grad: min waves per SIMD (register budget 512 / RX_PPO_MINW)
#endif

using rx_policy::Lay;
using rx_policy::normal_logp;
// 8 consecutive floats of an LDS row (8-byte aligned) as a bf16 fragment
__device__ __forceinline__ bf8 rows8(const float* p) {
  const float2 a = *reinterpret_cast<const float2*>(p), b = *reinterpret_cast<const float2*>(p + 2),
               c = *reinterpret_cast<const float2*>(p + 4), d = *reinterpret_cast<const float2*>(p + 6);
  return to_bf8(make_float4(a.x, a.y, b.x, b.y), make_float4(c.x, c.y, d.x, d.y));
}

struct ppo_args {
  rx_ppo_batch b;
  int32_t m;            // minibatch index within the epoch
  int32_t rows_per_wg;  // multiple of kRP
  const uint8_t* stop;
  double* kl_partial;   // [n_wg]
};

struct WLds {
  const float* W1;  // [64][DP], zero beyond D
  const float* b1;
  const float* W2;  // [64][kWS]
  const float* b2;
  const float* W3;  // [n_out][64]
  const float* b3;
  int DP;
  __device__ float w1(int o, int d) const { return d < DP ? W1[o * DP + d] : 0.0f; }  // zero-padded to DP
  __device__ float4 w2row4(int o, int i0) const { return *reinterpret_cast<const float4*>(W2 + o * kWS + i0); }
  __device__ float w2(int o, int i) const { return W2[o * kWS + i]; }
  __device__ float w3(int j, int h) const { return W3[j * kH + h]; }
};

template <int D, int PREC, bool FRAG = false>
__global__ __launch_bounds__(kT) void k_policy_act(rx_policy_io io, const float* __restrict__ P,
                                                   const bf8* __restrict__ frag) {
  // a workgroup's 4 waves run ONE trunk (even workgroups actor, odd critic) on
  // 4 consecutive 16-row blocks, so a CU's L1 holds one trunk's 21 KB of weights
  const bool critic = blockIdx.x & 1;
  const int64_t rb = (int64_t)(blockIdx.x >> 1) * (kT / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  policy_rows<D, PREC, FRAG>(io, P, critic, rb, frag);
}

// The bf16 rollout's fragment image (rx_rollout_steps, once per rollout: the
// parameters do not change inside it): per trunk (workgroup y) F1 | F2 | F3 in
// mlp_forward_frag's layout, the same bf16 conversions mlp_forward's bf16 path
// does per use -- so every rollout policy launch reads one 16-byte fragment per
// MFMA operand from L2 instead of 8 scalar loads and 4 conversions.
template <int D>
__global__ __launch_bounds__(256) void k_policy_frag(const float* __restrict__ P, bf8* __restrict__ img) {
  using L = Lay<D>;
  const bool critic = blockIdx.x == 1;
  const float* W1 = P + (critic ? L::cW1 : L::aW1);
  const float* W2 = P + (critic ? L::cW2 : L::aW2);
  const float* W3 = P + (critic ? L::cW3 : L::aW3);
  const int nout = critic ? 1 : kNA;
  bf8* out = img + (critic ? kFragTrunk : 0);
  for (int sl = threadIdx.x; sl < kFragTrunk; sl += 256) {
    const int ln = sl & 63, l15 = ln & 15, q = ln >> 4;
    float v[8];
    if (sl < kFragF2) {  // F1[mt][lane] = W1[16 mt + l15][8 q + j] (zero beyond D)
      const int o = 16 * (sl >> 6) + l15;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = 8 * q + j < D ? W1[o * D + 8 * q + j] : 0.0f;
    } else if (sl < kFragF3) {  // F2[2 mt + s][lane] = W2[16 mt + l15][h(s, q, j)]
      const int k = (sl - kFragF2) >> 6, mt = k >> 1, s = k & 1, o = 16 * mt + l15;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = W2[o * kH + 32 * s + 16 * (j >> 2) + 4 * q + (j & 3)];
    } else {  // F3[s][lane] = W3[l15][h(s, q, j)] for l15 < n_out, else 0
      const int s = (sl - kFragF3) >> 6;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = l15 < nout ? W3[l15 * kH + 32 * s + 16 * (j >> 2) + 4 * q + (j & 3)] : 0.0f;
    }
    out[sl] = to_bf8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]));
  }
}

// One self-play rollout step's policies in ONE launch (rx_selfplay_rollout_steps):
// workgroup kind b % 3 = the learning agent's actor, its critic, the frozen
// opponent's actor (its log-prob and value are never read, so it has no critic
// workgroups) -- each exactly k_policy_act's rows.  The agent's critic
// workgroups also copy the agent's observation rows they read into the
// rollout's obs[t] and the previous step's agent reward into rewards[t - 1]
// (what k_agent_rows did after each step), when copy.obs_out is set.
struct selfplay_copy {
  float* obs_out;        // [N][D] rollout rows, or nullptr
  const float* rew_src;  // the env's [N][2] rewards
  float* rew_out;        // [N]
  int32_t agent;
};
template <int D, int PA, int PO>
__global__ __launch_bounds__(kT) void k_selfplay_act(rx_policy_io ag, rx_policy_io op, selfplay_copy cp) {
  const int kind = (int)blockIdx.x % 3;
  const int64_t rb = (int64_t)(blockIdx.x / 3) * (kT / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (kind == 2) {
    policy_rows<D, PO>(op, op.params, false, rb);
    return;
  }
  policy_rows<D, PA>(ag, ag.params, kind == 1, rb);
  if (kind != 1 || !cp.obs_out || rb * 16 >= ag.n) return;
  const int lane = threadIdx.x & 63;
  const int64_t os = ag.obs_stride > 0 ? ag.obs_stride : D;
  const int64_t r0 = rb * 16, nr = min((int64_t)16, ag.n - r0);
  for (int i = lane; i < nr * D; i += 64) {
    const int64_t r = r0 + i / D;
    cp.obs_out[r * D + i % D] = ag.obs[r * os + i % D];
  }
  if (lane < nr) cp.rew_out[r0 + lane] = cp.rew_src[(r0 + lane) * 2 + cp.agent];
}

// LDS words of k_ppo_grad's workgroup
template <int D>
struct GradLds {
  static constexpr int W1 = 0, B1 = W1 + 64 * Geo<D>::DP, W2 = B1 + 64, B2 = W2 + 64 * kWS, W3 = B2 + 64,
                       B3 = W3 + kNA * 64, WEND = B3 + 4;  // trunk weights
  // the pass's 64 rows: [hidden][row] transposes (dZ2 then dZ1; H1 then H2), [row][d] = [X | 1], [row][j] = g
  static constexpr int SZ = WEND, SH = SZ + 64 * kTS, SX = SH + 64 * kTS, SG = SX + kRP * Geo<D>::XS;
  // per-wave db2, dW3, db3, kl: written after the last pass, over the dZ transpose
  static constexpr int SMALL = SZ, SMALL_PER = 64 + kNA * 64 + kNA + 2, TOTAL = SG + kRP * kNA;
  static_assert(kGW * SMALL_PER <= 64 * kTS, "per-wave sums must fit in the dZ transpose");
};

// d loss / d head pre-activation g of the lane's row (every lane of the row) from
// the head outputs y (lane (0, l15) holds output j in y[j]) and the row's inputs
// s0..s3 (actor: actions 0 / 1, old log-prob, advantage; critic: return, old
// value); the actor also adds old_logp - logp to kl on its q = 0 lanes.
// agent/ppo.py:170-198 (clipped surrogate, clipped value loss); shared by both
// precisions' trunks.
template <int NET>
__device__ __forceinline__ void head_grad(const rx_ppo_batch& b, float s0, float s1, float s2, float s3, bool live,
                                          const f4& y, const float* b3, int l15, int q, const float (&var)[kNA],
                                          const float (&lsc)[kNA], float mean, float sd, float invM, float clip,
                                          float (&g)[NET ? 1 : kNA], double& kl) {
  constexpr int NOUT = NET ? 1 : kNA;
  const float lo = 1.0f - clip, hi = 1.0f + clip;
  if constexpr (NET == 0) {
    float mu[kNA], diff[kNA], logp = 0.0f;
#pragma unroll
    for (int j = 0; j < kNA; ++j) {
      mu[j] = rx_policy::tanh_fast(__shfl(y[j], l15, 64) + b3[j]);
      diff[j] = (j ? s1 : s0) - mu[j];
      logp += normal_logp(diff[j], var[j], lsc[j]);
    }
    const float oldlp = s2;
    const float An = live ? (s3 - mean) / (sd + 1e-8f) : 0.0f;
    const float ratio = expf(logp - oldlp);
    const float u1 = -An * ratio, u2 = -An * fminf(fmaxf(ratio, lo), hi);
    const float g1 = u1 > u2 ? 1.0f : (u1 == u2 ? 0.5f : 0.0f), g2 = 1.0f - g1;  // torch.max splits ties
    const float inr = (ratio >= lo && ratio <= hi) ? 1.0f : 0.0f;
    const float dlogp = live ? invM * (g1 * -An + g2 * -An * inr) * ratio : 0.0f;
#pragma unroll
    for (int j = 0; j < NOUT; ++j) g[j] = dlogp * diff[j] / var[j] * (1.0f - mu[j] * mu[j]);
    if (live && q == 0) kl += (double)(oldlp - logp);
  } else {
    const float v = __shfl(y[0], l15, 64) + b3[0];
    // 0.5 * max((v-R)^2, (v_clip-R)^2), agent/ppo.py:194-198
    const float R = s0, ov = s1;
    const float vd = v - ov;
    const float vc = ov + fminf(fmaxf(vd, -clip), clip);
    const float e1 = v - R, e2 = vc - R;
    const float q1 = e1 * e1, q2 = e2 * e2;
    const float gq1 = q1 > q2 ? 1.0f : (q1 == q2 ? 0.5f : 0.0f), gq2 = 1.0f - gq1;
    const float vin = (vd >= -clip && vd <= clip) ? 1.0f : 0.0f;
    g[0] = live ? b.vf_coef * 0.5f * invM * (gq1 * 2.0f * e1 + gq2 * 2.0f * e2 * vin) : 0.0f;
  }
}

// One trunk (NET: 0 = actor, 1 = critic) of one workgroup: rows_per_wg rows,
// kRP = 64 per pass.  Per pass:
//   A  each wave: forward, loss gradient g and dZ2 for its 16 rows (registers);
//      dZ2^T, H1^T, [X | 1] and g of its rows -> LDS;                  barrier
//   B  wave w: dW2 rows [16w, 16w+16) over the pass's 64 rows (k = row);
//      db2 of its rows (lane = hidden unit); dH1 = W2^T dZ2, dZ1 (registers); barrier
//   C  each wave: dZ1^T, H2^T of its rows -> LDS;                       barrier
//   D  wave w: dW1 (+ db1) rows [16w, 16w+16); dW3 / db3 of its rows;   barrier
// Each wave owns distinct output tiles, so the tile accumulators go straight
// to the partial row; the per-wave db2 / dW3 / db3 / KL sums are folded in a
// fixed order ((w0 + w2) + (w1 + w3)).
template <int D, int NET, int PREC>
__device__ __forceinline__ void ppo_grad_trunk(const ppo_args& a, const float* __restrict__ W, float* lds,
                                               float* __restrict__ out) {
  using L = Lay<D>;
  using G = Geo<D>;
  using S = GradLds<D>;
  constexpr int NOUT = NET ? 1 : kNA, NT1 = G::NT1, XN = G::template XN<PREC>;
  constexpr int oW1 = NET ? L::cW1 : L::aW1, ob1 = NET ? L::cb1 : L::ab1, oW2 = NET ? L::cW2 : L::aW2,
                ob2 = NET ? L::cb2 : L::ab2, oW3 = NET ? L::cW3 : L::aW3, ob3 = NET ? L::cb3 : L::ab3;
  const rx_ppo_batch& b = a.b;
  const int t0 = threadIdx.x, lane = t0 & 63, l15 = lane & 15, q = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(t0 >> 6);
  const int rr = 16 * wv + l15;  // this lane's row within the pass
  // weight-gradient tiles of this wave: output rows [16 rb, 16 rb + 16) of dW2 /
  // dW1; dW2 column tiles c2 + i (i < NT2); dW1 column tiles c1 + i (i < NA1)
  // over k-steps [k1_lo, k1_hi) of the pass (8 waves and one dW1 column tile:
  // the two wave halves split the pass's rows and add at the end)
  constexpr int NT2 = kGW == 4 ? 4 : 2, NA1 = kGW == 4 ? NT1 : 1;
  const int rb = kGW == 4 ? wv : (wv & 3), hh = kGW == 4 ? 0 : (wv >> 2);
  const int c2 = NT2 * hh, c1 = (kGW == 8 && NT1 == 2) ? hh : 0;
  constexpr bool KSPLIT = kGW == 8 && NT1 == 1;
  const int64_t row0 = (int64_t)blockIdx.x * a.rows_per_wg;
  const int64_t row_end = min(row0 + (int64_t)a.rows_per_wg, (int64_t)b.mb);
  // wave-uniform operands in SGPRs: scalar loads through the constant address
  // space (a plain load through a pointer the compiler cannot prove unclobbered
  // is a vector load, and its result would hold VGPRs across every pass)
  auto sgpr = [](float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); };
  auto sload = [](const float* p) { return *(const __attribute__((address_space(4))) float*)p; };
  const float mean = sload(b.adv_stats + 2 * a.m), sd = sload(b.adv_stats + 2 * a.m + 1);
  const float invM = 1.0f / (float)b.mb;
  const float clip = b.clip_coef;
  float var[kNA], lsc[kNA];
#pragma unroll
  for (int j = 0; j < kNA; ++j) {
    const float scale = expf(sload(b.log_std + j));
    var[j] = sgpr(scale * scale);
    lsc[j] = sgpr(logf(scale));
  }
  f4 acc2[NT2], acc1[NA1];  // dW2 / dW1 (+ db1) tiles of rows [16 rb, +16)
#pragma unroll
  for (int k = 0; k < NT2; ++k) acc2[k] = f4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int k = 0; k < NA1; ++k) acc1[k] = f4{0.0f, 0.0f, 0.0f, 0.0f};
  float db2 = 0.0f, dw3[NOUT] = {}, db3 = 0.0f;  // lane = hidden unit (db2, dW3), output (db3)
  double kl = 0.0;
  // inputs of a row, loaded one pass ahead (the perm index two passes ahead):
  // the dependent gathers perm -> obs / actions / ... never stall a pass
  struct RowIn {
    float x[XN], s0, s1, s2, s3;  // actor: action 0/1, old log-prob, advantage; critic: return, value
  };
  auto src_of = [&](int64_t base) -> int64_t {
    const int64_t r_mb = base + rr;
    if (r_mb >= row_end) return -1;
    const int64_t v = b.perm[(int64_t)a.m * b.mb + r_mb];
    return (v >= 0 && v < b.n_rows) ? v : -1;  // out-of-range indices contribute nothing
  };
  auto load_row = [&](int64_t src) -> RowIn {
    RowIn in;
    const bool ok = src >= 0;
#pragma unroll
    for (int s = 0; s < XN; ++s) {
      const int d = G::template d_of<PREC>(s, q);
      in.x[s] = (ok && d < D) ? b.obs[src * D + d] : 0.0f;
    }
    if (NET == 0) {
      in.s0 = ok ? b.actions[src * kNA] : 0.0f;
      in.s1 = ok ? b.actions[src * kNA + 1] : 0.0f;
      in.s2 = ok ? b.logprobs[src] : 0.0f;
      in.s3 = ok ? b.advantages[src] : 0.0f;
    } else {
      in.s0 = ok ? b.returns[src] : 0.0f;
      in.s1 = ok ? b.values[src] : 0.0f;
      in.s2 = in.s3 = 0.0f;
    }
    return in;
  };
  // ---- stage the trunk's weights (zero-padded rows) while the first pass's
  // rows are gathered.  Issue order matters (vector loads complete in order):
  // the perm indices first, then EVERY staging load into registers, then the
  // row gathers (which wait only for the perm loads), then the LDS stores --
  // one memory latency for all of it instead of one round trip per staged
  // element (stamps: staging 11 k -> see DESIGN.md §3, k_ppo_grad)
  int64_t src = src_of(row0), src_n = src_of(row0 + kRP);
  constexpr int kW1N = (64 * G::DP + kGT - 1) / kGT, kW2N = 64 * 64 / kGT;
  float w1v[kW1N], w2v[kW2N], bv[2];
#pragma unroll
  for (int j = 0; j < kW1N; ++j) {
    const int e = t0 + kGT * j, o = e / G::DP, d = e - o * G::DP;
    w1v[j] = (e < 64 * G::DP && d < D) ? W[oW1 + o * D + d] : 0.0f;
  }
#pragma unroll
  for (int j = 0; j < kW2N; ++j) w2v[j] = W[oW2 + t0 + kGT * j];
  bv[0] = t0 < 64 ? W[ob1 + t0] : (t0 < 128 ? W[ob2 + t0 - 64] : 0.0f);
  bv[1] = t0 < NOUT * 64 ? W[oW3 + t0] : 0.0f;
  const float b3v = t0 < NOUT ? W[ob3 + t0] : 0.0f;
  RowIn cur = load_row(src);
#pragma unroll
  for (int j = 0; j < kW1N; ++j)
    if (t0 + kGT * j < 64 * G::DP) lds[S::W1 + t0 + kGT * j] = w1v[j];
#pragma unroll
  for (int j = 0; j < kW2N; ++j) {
    const int e = t0 + kGT * j;
    lds[S::W2 + (e >> 6) * kWS + (e & 63)] = w2v[j];
  }
  if (t0 < 64)
    lds[S::B1 + t0] = bv[0];
  else if (t0 < 128)
    lds[S::B2 + t0 - 64] = bv[0];
  if (t0 < NOUT * 64) lds[S::W3 + t0] = bv[1];
  if (t0 < NOUT) lds[S::B3 + t0] = b3v;
  __syncthreads();
  const WLds w{lds + S::W1, lds + S::B1, lds + S::W2, lds + S::B2, lds + S::W3, lds + S::B3, G::DP};
  PPO_STAMP(1);
  int pass_ = 0;
  float* sZ = lds + S::SZ;  // [hidden][row]
  float* sH = lds + S::SH;  // [hidden][row]
  float* sX = lds + S::SX;  // [row][d]
  float* sG = lds + S::SG;  // [row][j]

  for (int64_t base = row0; base < row_end; base += kRP) {
    // ================================================================ A
    const int64_t src_nn = src_of(base + 2 * kRP);
    const RowIn nxt = load_row(src_n);
    const bool live = src >= 0;
    float x[XN];
#pragma unroll
    for (int s = 0; s < XN; ++s) {
      const int d = G::template d_of<PREC>(s, q);
      x[s] = cur.x[s];
      if (d <= D) sX[rr * G::XS + d] = d == D ? 1.0f : x[s];  // the ones column (d = D) carries db1
    }
    f4 H1[4], H2[4], y;
    mlp_forward<D, NOUT, PREC>(w, x, H1, H2, y, l15, q, pass_ == 0 ? 16 : -1);
    if (pass_ == 0) PPO_STAMP(18);
    float g[NOUT];  // d loss / d head pre-activation, row rr (every lane of the row)
    head_grad<NET>(b, cur.s0, cur.s1, cur.s2, cur.s3, live, y, w.b3, l15, q, var, lsc, mean, sd, invM, clip, g, kl);
    if (pass_ == 0) PPO_STAMP(19);
    f4 dZ[4];  // dZ2 = (W3^T g) * (1 - H2^2)
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int h = 16 * t + 4 * q + r;
        float dh = 0.0f;
#pragma unroll
        for (int j = 0; j < NOUT; ++j) dh = fmaf(w.w3(j, h), g[j], dh);
        dZ[t][r] = dh * (1.0f - H2[t][r] * H2[t][r]);
        sZ[h * kTS + rr] = dZ[t][r];
        sH[h * kTS + rr] = H1[t][r];
      }
    if (q == 0) {
#pragma unroll
      for (int j = 0; j < NOUT; ++j) sG[rr * kNA + j] = g[j];
    }
    __syncthreads();
    PPO_STAMP(2 + 4 * pass_);
    // ================================================================ B
    // dW2[16 wv + i][16 nt + c] += sum_rows dZ2 x H1 (k = row 4s + q; bf16: row 32s + 8q + j)
    if constexpr (PREC == kBF16) {
#pragma unroll
      for (int s = 0; s < kRP / 32; ++s) {
        const bf8 av = rows8(sZ + (16 * rb + l15) * kTS + 32 * s + 8 * q);
#pragma unroll
        for (int i = 0; i < NT2; ++i)
          acc2[i] = mma16(av, rows8(sH + (16 * (c2 + i) + l15) * kTS + 32 * s + 8 * q), acc2[i]);
      }
    } else {
#pragma unroll 4
      for (int s = 0; s < kRP / 4; ++s) {
        const float av = sZ[(16 * rb + l15) * kTS + 4 * s + q];
        float bv[NT2];
#pragma unroll
        for (int i = 0; i < NT2; ++i) bv[i] = sH[(16 * (c2 + i) + l15) * kTS + 4 * s + q];
#pragma unroll
        for (int i = 0; i < NT2; ++i) acc2[i] = mma(av, bv[i], acc2[i]);
      }
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) db2 += sZ[lane * kTS + 16 * wv + k];  // lane = hidden unit, own rows
    // dH1 = W2^T dZ2 (k = output unit o = 16t + 4q + r), dZ1 = dH1 * (1 - H1^2) in registers
    f4 dZ1[4];
    if constexpr (PREC == kBF16) {
      const bf8 bz[2] = {to_bf8(dZ[0], dZ[1]), to_bf8(dZ[2], dZ[3])};
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        f4 z = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          float v[8];
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) v[jj] = w.w2(32 * s + 16 * (jj >> 2) + 4 * q + (jj & 3), 16 * mt + l15);
          z = mma16(to_bf8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7])), bz[s], z);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) dZ1[mt][r] = z[r] * (1.0f - H1[mt][r] * H1[mt][r]);
      }
    } else {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        f4 z = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) z = mma(w.w2(16 * t + 4 * q + r, 16 * mt + l15), dZ[t][r], z);
#pragma unroll
        for (int r = 0; r < 4; ++r) dZ1[mt][r] = z[r] * (1.0f - H1[mt][r] * H1[mt][r]);
      }
    }
    __syncthreads();
    PPO_STAMP(3 + 4 * pass_);
    // ================================================================ C
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int h = 16 * t + 4 * q + r;
        sZ[h * kTS + rr] = dZ1[t][r];
        sH[h * kTS + rr] = H2[t][r];
      }
    __syncthreads();
    PPO_STAMP(4 + 4 * pass_);
    // ================================================================ D
    // dW1[16 wv + i][d] (+ db1 at d = D) += sum_rows dZ1 x [X | 1]
    if constexpr (PREC == kBF16) {
      constexpr int KS = KSPLIT ? kRP / 64 : kRP / 32;  // k-steps of 32 rows
      const int s0 = KSPLIT ? hh * KS : 0;
#pragma unroll
      for (int s = s0; s < s0 + KS; ++s) {
        const bf8 av = rows8(sZ + (16 * rb + l15) * kTS + 32 * s + 8 * q);
#pragma unroll
        for (int i = 0; i < NA1; ++i) {
          const int d = 16 * (c1 + i) + l15;
          float v[8];
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) v[jj] = d <= D ? sX[(32 * s + 8 * q + jj) * G::XS + d] : 0.0f;
          acc1[i] = mma16(av, to_bf8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7])),
                          acc1[i]);
        }
      }
    } else {
      constexpr int KS = KSPLIT ? kRP / 8 : kRP / 4;  // k-steps of 4 rows
      const int s0 = KSPLIT ? hh * KS : 0;
#pragma unroll 4
      for (int s = s0; s < s0 + KS; ++s) {
        const float av = sZ[(16 * rb + l15) * kTS + 4 * s + q];
        float bv[NA1];
#pragma unroll
        for (int i = 0; i < NA1; ++i) {
          const int d = 16 * (c1 + i) + l15;
          bv[i] = d <= D ? sX[(4 * s + q) * G::XS + d] : 0.0f;
        }
#pragma unroll
        for (int i = 0; i < NA1; ++i) acc1[i] = mma(av, bv[i], acc1[i]);
      }
    }
    // dW3 / db3 of own rows (lane = hidden unit / output)
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int row = 16 * wv + k;
      const float h2 = sH[lane * kTS + row];
#pragma unroll
      for (int j = 0; j < NOUT; ++j) dw3[j] = fmaf(sG[row * kNA + j], h2, dw3[j]);
      if (lane < NOUT) db3 += sG[row * kNA + lane];
    }
    __syncthreads();  // the next pass overwrites the transposes
    PPO_STAMP(5 + 4 * pass_);
    ++pass_;
    src = src_n;
    src_n = src_nn;
    cur = nxt;
  }
  // ---- tile accumulators -> the partial row (each wave owns its tiles)
  PPO_STAMP(14);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int o = 16 * rb + 4 * q + r;
#pragma unroll
    for (int i = 0; i < NT2; ++i) out[oW2 + o * kH + 16 * (c2 + i) + l15] = acc2[i][r];
  }
  float* xch = lds + S::SH;  // KSPLIT: the second half's dW1 tile, [row block][lane][4]
  if constexpr (KSPLIT) {
    if (hh == 1) *reinterpret_cast<float4*>(xch + (rb * 64 + lane) * 4) =
        make_float4(acc1[0][0], acc1[0][1], acc1[0][2], acc1[0][3]);
  }
  // ---- per-wave small sums, folded over the waves in a fixed order
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) kl += __shfl_xor(kl, o, 64);
  float* small = lds + S::SMALL + wv * S::SMALL_PER;
  small[lane] = db2;
#pragma unroll
  for (int j = 0; j < NOUT; ++j) small[64 + j * 64 + lane] = dw3[j];
  if (lane < NOUT) small[64 + kNA * 64 + lane] = db3;
  if (lane == 0) reinterpret_cast<double*>(small + 64 + kNA * 64 + kNA)[0] = kl;  // 8-aligned: SMALL_PER is even
  __syncthreads();
  PPO_STAMP(15);
  if (!KSPLIT || hh == 0) {
    if constexpr (KSPLIT) {  // rows of the pass's first half + its second half, in that order
      const float4 o2 = *reinterpret_cast<const float4*>(xch + (rb * 64 + lane) * 4);
      acc1[0][0] += o2.x, acc1[0][1] += o2.y, acc1[0][2] += o2.z, acc1[0][3] += o2.w;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int o = 16 * rb + 4 * q + r;
#pragma unroll
      for (int i = 0; i < NA1; ++i) {
        const int d = 16 * (c1 + i) + l15;
        if (d < D)
          out[oW1 + o * D + d] = acc1[i][r];
        else if (d == D)
          out[ob1 + o] = acc1[i][r];
      }
    }
  }
  if (wv != 0) return;
  const float* sm = lds + S::SMALL;
  constexpr int SP = S::SMALL_PER;
  auto fold = [&](int k) -> float {  // per-wave partials in a fixed order
    if constexpr (kGW == 4)
      return (sm[k] + sm[2 * SP + k]) + (sm[SP + k] + sm[3 * SP + k]);
    else
      return ((sm[k] + sm[4 * SP + k]) + (sm[2 * SP + k] + sm[6 * SP + k])) +
             ((sm[SP + k] + sm[5 * SP + k]) + (sm[3 * SP + k] + sm[7 * SP + k]));
  };
  for (int e = lane; e < 64 + NOUT * 64 + NOUT; e += 64) {
    const int k = e < 64 + NOUT * 64 ? e : 64 + kNA * 64 + (e - 64 - NOUT * 64);
    const float v = fold(k);
    if (e < 64)
      out[ob2 + e] = v;
    else if (e < 64 + NOUT * 64)
      out[oW3 + (e - 64)] = v;
    else
      out[ob3 + (e - 64 - NOUT * 64)] = v;
  }
  if (NET == 0 && lane == 0) {
    const double* kd = reinterpret_cast<const double*>(sm + 64 + kNA * 64 + kNA);
    const int st = S::SMALL_PER / 2;
    if constexpr (kGW == 4)
      a.kl_partial[blockIdx.x] = (kd[0] + kd[2 * st]) + (kd[st] + kd[3 * st]);
    else
      a.kl_partial[blockIdx.x] = ((kd[0] + kd[4 * st]) + (kd[2 * st] + kd[6 * st])) +
                                 ((kd[st] + kd[5 * st]) + (kd[3 * st] + kd[7 * st]));
  }
}

// ================================================================ bf16 k_ppo_grad
// The bf16 gradient (rx_ppo_batch.precision = RX_PREC_BF16) with
// every matrix operand in the form the 16x16x32 bf16 MFMA reads, so the pass is
// MFMAs, their LDS reads and the activation math -- no per-use conversions:
//  * weights: built ONCE per workgroup as bf16 MFMA fragments in LDS, one
//    ds_read_b128 each -- F1 (layer 1), F2 (layer 2), F3 (head) in the exact
//    operand order of mlp_forward's bf16 path (the forward is bit-identical to
//    k_policy_act / k_rollout's), FT2 = W2^T for dH1 = W2^T dZ2;
//  * the batch-row reductions dW = sum_rows dZ^T [H | X | 1]: the accumulator
//    tiles hold the row on the lane, so each lane stores its 4 registers of a
//    tile packed (v_cvt_pk_bf16_f32, one ds_write_b64) into a [row][unit] image
//    and the operand is read back transposed with ds_read_b64_tr_b16
//    (MI355X / cdna_hip_programming.md T10), rows 32s + 8g + 4h + (0..3) per
//    read: the batch row is the MFMA K dimension;
//  * bias gradients ride on ones columns: db2 as a fifth dW2 column tile (H
//    image column 64 = 1), db1 on the X image's column D (as the fp32 kernel),
//    dW3 | db3 as an MFMA over the g image (operand rows j < NOUT) against the
//    H2 image and its ones tile.
// Gradients are rounded to bf16 only where they are matrix operands, as the
// fp32-vs-bf16 contract of rx.h says; accumulation and everything else is f32.
// Same pass structure as the fp32 kernel (A forward + loss + images | B dW2, dH1
// | C images | D dW1, dW3), 47 KB of LDS: three 4-wave workgroups per CU.
//
// The images live in two regions of kRP rows x 96 bf16 (GradLdsB): A = dZ (cols
// 0..63: dZ2, then dZ1) | [X | 1] (cols 64..95); B = H (cols 0..63: H1, then H2) |
// its ones tile (64..79) | g (80..95).  The row stride is 48 dwords and every
// row is swizzled (sw_off: 16-column block b at b ^ ((r >> 3) & 1), 4-column
// chunk p at p ^ ((r >> 1) & 3)), which makes both of the kernel's LDS access
// shapes bank-conflict-free (MI355X_MICROARCH.md §LDS): a packed row-chunk store
// (ds_write_b64, groups of 16 lanes = 16 consecutive rows at one column, bank =
// dword mod 32: row bit 0 -> bank bit 4 through the stride, bit 3 -> bit 3 through
// the block swizzle, bits 1-2 -> bits 1-2 through the chunk swizzle) and the
// transposed operand read (ds_read_b64_tr_b16, halves of 32 lanes = rows
// {0..3, 8..11} + 32 s (+ 16) at one 16-column block, bank = dword mod 64: the
// stride spreads rows 0..3 over 16-dword steps, the block swizzle moves rows
// 8..11 by 8 dwords).  The plain [row][col] images of round 5 (strides 72 / 80 /
// 48 / 24 bf16) ran 2- to 4-way conflicts on both: 38.5 % of the LDS-active
// cycles (profiles/r05/pmc_ppo_bf16.json).  (Round 5's double-buffered image A/B,
// RX_PPO_BF_DB, measured no faster and is gone with the plain layout.)
constexpr int kIS = 96;  // image row stride (bf16): 48 dwords
template <int D>
struct GradLdsB {
  static constexpr int F1 = 0, F2 = F1 + 4 * 64 * 16, FT2 = F2 + 8 * 64 * 16, F3 = FT2 + 8 * 64 * 16,
                       B1 = F3 + 2 * 64 * 16, B2 = B1 + 64 * 4, W3 = B2 + 64 * 4, B3 = W3 + kNA * 64 * 4,
                       IA = B3 + 16, IB = IA + kRP * kIS * 2, KL = IB + kRP * kIS * 2, TOTAL = KL + 8 * kGW;
  static constexpr int XC = 64, ONES = 64, GC = 80;  // column of [X | 1] in A, of the ones tile and g in B
  static_assert(IA % 16 == 0 && IB % 16 == 0, "16-byte aligned images");
  static_assert(TOTAL <= 53 * 1024, "three workgroups per CU");
};

using bf4 = __bf16 __attribute__((ext_vector_type(4)));
using s4 = short __attribute__((ext_vector_type(4)));
// element offset of (row r, column c) in a swizzled image region (GradLdsB): the
// 16-column block b of row r at block b ^ ((r >> 3) & 1), its 4-column chunk p at
// chunk p ^ ((r >> 1) & 3); the 4 elements of a chunk stay contiguous (8 bytes)
__device__ __forceinline__ int sw_off(int r, int c) {
  return r * kIS + (((c >> 4) ^ ((r >> 3) & 1)) << 4) + ((((c >> 2) & 3) ^ ((r >> 1) & 3)) << 2) + (c & 3);
}
// 4 bf16 of one image row: the lane's 4 accumulator registers of a tile, at (row r, column c)
__device__ __forceinline__ void st_bf4(char* img, int r, int c, const f4& v) {
  bf4 b;
  b[0] = (__bf16)v[0], b[1] = (__bf16)v[1], b[2] = (__bf16)v[2], b[3] = (__bf16)v[3];
  *reinterpret_cast<bf4*>(img + 2 * sw_off(r, c)) = b;
}
// The 16x16x32 operand of k-step s over an image region:
// A[m = col c0 + lane & 15][k = row 32 s + 8 (lane >> 4) + j], two transposed reads
// of 4 rows each (T10: lane 4q + p of a 16-lane group addresses row q, columns 4p..4p+3).
// The lane's row is 32 s + 8 g + (i >> 2) (g = lane >> 4, i = lane & 15), so its
// swizzle terms are lane constants: block ^ (g & 1), chunk ^ ((i >> 3) & 1) (rows +4:
// chunk ^ (((i >> 3) & 1) + 2)).  tr_lane holds the lane's byte offsets for an
// even / odd block, low / high 4 rows; a read adds the compile-time 2 (32 s kIS + c0)
// (the ds_read offset field), so the swizzle costs no per-read VALU or registers.
struct tr_lane {
  int lo_e, lo_o, hi_e, hi_o;
};
__device__ __forceinline__ tr_lane tr_lane_of(int lane) {
  const int g = lane >> 4, i = lane & 15, j = i >> 2, g1 = g & 1, h = j >> 1;
  const int lo = 2 * ((8 * g + j) * kIS + 16 * g1 + 4 * ((i & 3) ^ h));
  const int hi = 2 * ((8 * g + j + 4) * kIS + 16 * g1 + 4 * ((i & 3) ^ (h + 2)));
  return tr_lane{lo, lo - 64 * g1, hi, hi - 64 * g1};
}
__device__ __forceinline__ bf8 tr_frag(const char* img, int s, int c0, const tr_lane& tl) {
  const int k = 2 * (32 * s * kIS + c0);  // c0: a multiple of 16
  const bool odd = (c0 >> 4) & 1;
  typedef short __attribute__((ext_vector_type(4))) v4s;
  const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) v4s*)(img + (odd ? tl.lo_o : tl.lo_e) + k));
  const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) v4s*)(img + (odd ? tl.hi_o : tl.hi_e) + k));
  bf8 r;
  const __bf16* pl = reinterpret_cast<const __bf16*>(&lo);
  const __bf16* ph = reinterpret_cast<const __bf16*>(&hi);
#pragma unroll
  for (int j = 0; j < 4; ++j) r[j] = pl[j], r[4 + j] = ph[j];
  return r;
}

template <int D, int NET>
__device__ __forceinline__ void ppo_grad_trunk_bf(const ppo_args& a, const float* __restrict__ W, char* lds,
                                                  float* __restrict__ out) {
  using L = Lay<D>;
  using G = Geo<D>;
  using S = GradLdsB<D>;
  constexpr int NOUT = NET ? 1 : kNA, NT1 = G::NT1;
  constexpr int oW1 = NET ? L::cW1 : L::aW1, ob1 = NET ? L::cb1 : L::ab1, oW2 = NET ? L::cW2 : L::aW2,
                ob2 = NET ? L::cb2 : L::ab2, oW3 = NET ? L::cW3 : L::aW3, ob3 = NET ? L::cb3 : L::ab3;
  static_assert(kGW == 4, "the bf16 trunk partitions its tiles over 4 waves");
  const rx_ppo_batch& b = a.b;
  const int t0 = threadIdx.x, lane = t0 & 63, l15 = lane & 15, q = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(t0 >> 6);
  const int rr = 16 * wv + l15;  // this lane's row within the pass
  const int64_t row0 = (int64_t)blockIdx.x * a.rows_per_wg;
  const int64_t row_end = min(row0 + (int64_t)a.rows_per_wg, (int64_t)b.mb);
  auto sgpr = [](float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); };
  auto sload = [](const float* p) { return *(const __attribute__((address_space(4))) float*)p; };
  const float mean = sload(b.adv_stats + 2 * a.m), sd = sload(b.adv_stats + 2 * a.m + 1);
  const float invM = 1.0f / (float)b.mb;
  const float clip = b.clip_coef;
  float var[kNA], lsc[kNA];
#pragma unroll
  for (int j = 0; j < kNA; ++j) {
    const float scale = expf(sload(b.log_std + j));
    var[j] = sgpr(scale * scale);
    lsc[j] = sgpr(logf(scale));
  }
  struct RowIn {
    float x[8], s0, s1, s2, s3;
  };
  auto src_of = [&](int64_t base) -> int64_t {
    const int64_t r_mb = base + rr;
    if (r_mb >= row_end) return -1;
    const int64_t v = b.perm[(int64_t)a.m * b.mb + r_mb];
    return (v >= 0 && v < b.n_rows) ? v : -1;
  };
  auto load_row = [&](int64_t src) -> RowIn {
    RowIn in;
    const bool ok = src >= 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int d = 8 * q + j;
      in.x[j] = (ok && d < D) ? b.obs[src * D + d] : 0.0f;
    }
    if (NET == 0) {
      in.s0 = ok ? b.actions[src * kNA] : 0.0f;
      in.s1 = ok ? b.actions[src * kNA + 1] : 0.0f;
      in.s2 = ok ? b.logprobs[src] : 0.0f;
      in.s3 = ok ? b.advantages[src] : 0.0f;
    } else {
      in.s0 = ok ? b.returns[src] : 0.0f;
      in.s1 = ok ? b.values[src] : 0.0f;
      in.s2 = in.s3 = 0.0f;
    }
    return in;
  };
  // ---- the trunk's weight fragments.  Coalesced f32 loads of W1 / W2 (the perm
  // indices before them, the first rows' gathers after) into an LDS scratch in
  // the image region, then every fragment is assembled from LDS: per-element
  // gathers from L2 (W1's 60-byte rows, W2's columns for FT2) cost ~400 cache-line
  // accesses per wave and made staging 35 % of the wave (profiles/r05/
  // ppo_stamps_bf16.json); coalesced, ~85.
  int64_t src = src_of(row0), src_n = src_of(row0 + kRP);
  constexpr int kW1N = (64 * D + kGT - 1) / kGT;  // W1 elements per thread
  constexpr int kS2 = 68;                         // W2 scratch row stride (f32, float4-aligned)
  float w1v[kW1N];
#pragma unroll
  for (int j = 0; j < kW1N; ++j) w1v[j] = t0 + kGT * j < 64 * D ? W[oW1 + t0 + kGT * j] : 0.0f;
  float4 w2v[4];  // W2 as 1,024 float4: thread t holds float4s t, t + 256, ...
#pragma unroll
  for (int j = 0; j < 4; ++j) w2v[j] = reinterpret_cast<const float4*>(W + oW2)[t0 + kGT * j];
  const float bv0 = t0 < 64 ? W[ob1 + t0] : (t0 < 128 ? W[ob2 + t0 - 64] : 0.0f);
  const float bv1 = t0 < NOUT * 64 ? W[oW3 + t0] : 0.0f;
  const float b3v = t0 < NOUT ? W[ob3 + t0] : 0.0f;
  RowIn cur = load_row(src);
  bf8* F1 = reinterpret_cast<bf8*>(lds + S::F1);
  bf8* F2 = reinterpret_cast<bf8*>(lds + S::F2);
  bf8* FT2 = reinterpret_cast<bf8*>(lds + S::FT2);
  bf8* F3 = reinterpret_cast<bf8*>(lds + S::F3);
  float* fB1 = reinterpret_cast<float*>(lds + S::B1);
  float* fB2 = reinterpret_cast<float*>(lds + S::B2);
  float* fW3 = reinterpret_cast<float*>(lds + S::W3);
  float* fB3 = reinterpret_cast<float*>(lds + S::B3);
  char* iA = lds + S::IA;  // dZ | [X | 1]
  char* iB = lds + S::IB;  // H | ones | g
  float* sW2 = reinterpret_cast<float*>(lds + S::IA);  // scratch: W2 [64][kS2], then W1 [64][D]
  float* sW1 = sW2 + 64 * kS2;
  static_assert(S::KL - S::IA >= (64 * kS2 + 64 * D) * 4, "the staging scratch fits in the image regions");
#pragma unroll
  for (int j = 0; j < kW1N; ++j)
    if (t0 + kGT * j < 64 * D) sW1[t0 + kGT * j] = w1v[j];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int e4 = t0 + kGT * j, o = e4 >> 4, i = 4 * (e4 & 15);
    *reinterpret_cast<float4*>(sW2 + o * kS2 + i) = w2v[j];
  }
  if (t0 < 64)
    fB1[t0] = bv0;
  else if (t0 < 128)
    fB2[t0 - 64] = bv0;
  if (t0 < NOUT * 64) fW3[t0] = bv1;
  if (t0 < NOUT) fB3[t0] = b3v;
  __syncthreads();
  {  // F1: slot t = (mt = t >> 6, lane): W1[16 mt + l15'][8 q' + j] (zero beyond D)
    const int ln = t0 & 63, o = 16 * (t0 >> 6) + (ln & 15), q1 = ln >> 4;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 8 * q1 + j < D ? sW1[o * D + 8 * q1 + j] : 0.0f;
    F1[t0] = to_bf8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]));
  }
  // F2 / FT2: slots t + 256 k = (mt, s, lane): F2 = W2[16 mt + l15'][h(s, q', j)],
  // FT2 = W2[h(s, q', j)][16 mt + l15'], h(s, q, j) = 32 s + 16 (j >> 2) + 4 q + (j & 3)
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int sl = t0 + 256 * k, mt = sl >> 7, s = (sl >> 6) & 1, ln = sl & 63, u = 16 * mt + (ln & 15),
              q1 = ln >> 4;
    F2[sl] = to_bf8(*reinterpret_cast<const float4*>(sW2 + u * kS2 + 32 * s + 4 * q1),
                    *reinterpret_cast<const float4*>(sW2 + u * kS2 + 32 * s + 16 + 4 * q1));
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = sW2[(32 * s + 16 * (j >> 2) + 4 * q1 + (j & 3)) * kS2 + u];
    FT2[sl] = to_bf8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]));
  }
  // F3: slot t < 128 = (s, lane): W3[l15'][h(s, q', j)] for l15' < NOUT, else 0
  if (t0 < 128) {
    const int s = t0 >> 6, ln = t0 & 63, q1 = ln >> 4;
    float4 lo = make_float4(0.0f, 0.0f, 0.0f, 0.0f), hi = lo;
    if ((ln & 15) < NOUT) {
      lo = *reinterpret_cast<const float4*>(fW3 + (ln & 15) * kH + 32 * s + 4 * q1);
      hi = *reinterpret_cast<const float4*>(fW3 + (ln & 15) * kH + 32 * s + 16 + 4 * q1);
    }
    F3[t0] = to_bf8(lo, hi);
  }
  __syncthreads();  // the scratch is dead: the images may be written
  // constant image columns: H's ones tile (column 64 = 1, 65..79 = 0), g's zero columns 4..15
  // (read only after the next pass's first barrier)
  {
    const int r = t0 >> 2, c = 4 * (t0 & 3);  // 64 rows x 4 chunks of 4 columns
    st_bf4(iB, r, S::ONES + c, c == 0 ? f4{1.0f, 0.0f, 0.0f, 0.0f} : f4{0.0f, 0.0f, 0.0f, 0.0f});
    if (c != 0) st_bf4(iB, r, S::GC + c, f4{0.0f, 0.0f, 0.0f, 0.0f});
  }
  PPO_STAMP(1);
  f4 acc2[5], acc1[NT1], acc3 = {0.0f, 0.0f, 0.0f, 0.0f}, acc3b = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int k = 0; k < 5; ++k) acc2[k] = f4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int k = 0; k < NT1; ++k) acc1[k] = f4{0.0f, 0.0f, 0.0f, 0.0f};
  double kl = 0.0;
  const float* b3 = fB3;
  const tr_lane tl = tr_lane_of(lane);
  int pass_ = 0;
  for (int64_t base = row0; base < row_end; base += kRP) {
    // ================================================================ A
    const int64_t src_nn = src_of(base + 2 * kRP);
    const RowIn nxt = load_row(src_n);
    const bool live = src >= 0;
    // [X | 1] row: d = 8q + j, the ones column d = D carries db1
    {
      float xv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) xv[j] = 8 * q + j == D ? 1.0f : cur.x[j];
      st_bf4(iA, rr, S::XC + 8 * q, f4{xv[0], xv[1], xv[2], xv[3]});
      st_bf4(iA, rr, S::XC + 8 * q + 4, f4{xv[4], xv[5], xv[6], xv[7]});
    }
    // forward: mlp_forward's bf16 arithmetic on the prebuilt fragments
    f4 H1[4], H2[4], y;
    mlp_forward_frag<NOUT>(F1, F2, F3, fB1, fB2, cur.x, H1, H2, y, lane, q);
    float g[NOUT];
    head_grad<NET>(b, cur.s0, cur.s1, cur.s2, cur.s3, live, y, b3, l15, q, var, lsc, mean, sd, invM, clip, g, kl);
    f4 dZ[4];  // dZ2 = (W3^T g) * (1 - H2^2)
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int h = 16 * t + 4 * q + r;
        float dh = 0.0f;
#pragma unroll
        for (int j = 0; j < NOUT; ++j) dh = fmaf(fW3[j * kH + h], g[j], dh);
        dZ[t][r] = dh * (1.0f - H2[t][r] * H2[t][r]);
      }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      st_bf4(iA, rr, 16 * t + 4 * q, dZ[t]);
      st_bf4(iB, rr, 16 * t + 4 * q, H1[t]);
    }
    if (q == 0) st_bf4(iB, rr, S::GC, f4{g[0], NOUT > 1 ? g[NOUT - 1] : 0.0f, 0.0f, 0.0f});
    __syncthreads();
    PPO_STAMP(2 + 4 * pass_);
    // ================================================================ B
    // dW2 rows [16 wv, +16) x column tiles 0..3, db2 on tile 4 (the ones column)
#pragma unroll
    for (int s = 0; s < kRP / 32; ++s) {
      const bf8 av = tr_frag(iA, s, 16 * wv, tl);
#pragma unroll
      for (int c = 0; c < 5; ++c) acc2[c] = mma16(av, tr_frag(iB, s, 16 * c, tl), acc2[c]);
    }
    // dH1 = W2^T dZ2 (B = dZ2 in registers, k = output unit), dZ1 = dH1 * (1 - H1^2)
    f4 dZ1[4];
    {
      const bf8 bz[2] = {to_bf8(dZ[0], dZ[1]), to_bf8(dZ[2], dZ[3])};
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        f4 z = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int s = 0; s < 2; ++s) z = mma16(FT2[(2 * mt + s) * 64 + lane], bz[s], z);
#pragma unroll
        for (int r = 0; r < 4; ++r) dZ1[mt][r] = z[r] * (1.0f - H1[mt][r] * H1[mt][r]);
      }
    }
    __syncthreads();  // C overwrites dZ2 and H1
    PPO_STAMP(3 + 4 * pass_);
    // ================================================================ C
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      st_bf4(iA, rr, 16 * t + 4 * q, dZ1[t]);
      st_bf4(iB, rr, 16 * t + 4 * q, H2[t]);
    }
    __syncthreads();
    PPO_STAMP(4 + 4 * pass_);
    // ================================================================ D
    // dW1 (+ db1 at d = D) rows [16 wv, +16); dW3 column tile wv, db3 (wave 0) on the ones tile
#pragma unroll
    for (int s = 0; s < kRP / 32; ++s) {
      const bf8 av = tr_frag(iA, s, 16 * wv, tl);
#pragma unroll
      for (int c = 0; c < NT1; ++c) acc1[c] = mma16(av, tr_frag(iA, s, S::XC + 16 * c, tl), acc1[c]);
      const bf8 gv = tr_frag(iB, s, S::GC, tl);
      acc3 = mma16(gv, tr_frag(iB, s, 16 * wv, tl), acc3);
      if (wv == 0) acc3b = mma16(gv, tr_frag(iB, s, S::ONES, tl), acc3b);
    }
    __syncthreads();  // the next pass overwrites the images
    PPO_STAMP(5 + 4 * pass_);
    ++pass_;
    src = src_n;
    src_n = src_nn;
    cur = nxt;
  }
  (void)pass_;  // (indexes the profiling build's stamps only)
  // ---- tile accumulators -> the partial row (each wave owns its tiles)
  PPO_STAMP(14);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int o = 16 * wv + 4 * q + r;
#pragma unroll
    for (int c = 0; c < 4; ++c) out[oW2 + o * kH + 16 * c + l15] = acc2[c][r];
    if (l15 == 0) out[ob2 + o] = acc2[4][r];
#pragma unroll
    for (int c = 0; c < NT1; ++c) {
      const int d = 16 * c + l15;
      if (d < D)
        out[oW1 + o * D + d] = acc1[c][r];
      else if (d == D)
        out[ob1 + o] = acc1[c][r];
    }
  }
  if (q == 0) {
#pragma unroll
    for (int j = 0; j < NOUT; ++j) out[oW3 + j * kH + 16 * wv + l15] = acc3[j];
    if (wv == 0 && l15 == 0) {
#pragma unroll
      for (int j = 0; j < NOUT; ++j) out[ob3 + j] = acc3b[j];
    }
  }
  if constexpr (NET == 0) {  // approx_kl partial: per wave, folded over the waves in a fixed order
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) kl += __shfl_xor(kl, o, 64);
    double* kd = reinterpret_cast<double*>(lds + S::KL);
    if (lane == 0) kd[wv] = kl;
    __syncthreads();
    if (t0 == 0) a.kl_partial[blockIdx.x] = (kd[0] + kd[2]) + (kd[1] + kd[3]);
  }
#ifdef RX_PPO_STAMPS
  __builtin_amdgcn_s_waitcnt(0);  // the partial-row stores landed (profiling build)
#endif
  PPO_STAMP(15);
}

// bf16 (RX_PPO_BF_FRAG = 1, the default): the fragment / transposed-image trunk
// above, three workgroups per CU (47 KB of LDS, <= 168 VGPRs); 0 = the bf16 path
// of ppo_grad_trunk (per-use conversions from the f32 LDS copy), kept for A/B.
#ifndef RX_PPO_BF_FRAG
#define RX_PPO_BF_FRAG 1
#endif
template <int D>
__global__ __launch_bounds__(kGT, 3) void k_ppo_grad_bf(ppo_args a, const float* __restrict__ W,
                                                        float* __restrict__ partial) {
  if (a.stop && *a.stop) return;  // KL early stop already hit: nothing to compute
  PPO_STAMP(0);
  __shared__ __attribute__((aligned(16))) char lds[GradLdsB<D>::TOTAL];
  float* out = partial + (size_t)blockIdx.x * Lay<D>::Pp;
  if (blockIdx.y == 0)
    ppo_grad_trunk_bf<D, 0>(a, W, lds, out);
  else
    ppo_grad_trunk_bf<D, 1>(a, W, lds, out);
}

// blockIdx.y = trunk (0 actor, 1 critic: their losses share no parameter, so
// they write disjoint ranges of the same partial row); blockIdx.x = row group.
template <int D, int PREC>
__global__ __launch_bounds__(kGT, RX_PPO_MINW) void k_ppo_grad(ppo_args a, const float* __restrict__ W,
                                                    float* __restrict__ partial) {
  if (a.stop && *a.stop) return;  // KL early stop already hit: nothing to compute
  PPO_STAMP(0);
  __shared__ __attribute__((aligned(16))) float lds[GradLds<D>::TOTAL];
  float* out = partial + (size_t)blockIdx.x * Lay<D>::Pp;
  if (blockIdx.y == 0)
    ppo_grad_trunk<D, 0, PREC>(a, W, lds, out);
  else
    ppo_grad_trunk<D, 1, PREC>(a, W, lds, out);
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
// With ``norm`` (the fused minibatch update, rx_ppo_minibatch_update) each
// workgroup also writes the per-tensor sums of squares of its 64 gradient
// entries to norm->ws[block][tensor] (clip_grad_norm_'s per-tensor norms, folded
// by k_adam_apply) and block 0 bumps the Adam step count unless it raises the
// early-stop flag: the optimizer launch that follows needs no norm pass.
struct norm_args {
  rx_adam_config cfg;
  float* ws;    // [gridDim.x][n_tensors], then Adam's 2 step scalars
  float* step;  // Adam step count
  const double* lr;
};

__global__ __launch_bounds__(1024) void k_ppo_reduce(const float* __restrict__ partial,
                                                     const double* __restrict__ klp, int n_wg, int P, int Pp, int mb,
                                                     float kl_target, float scale, float* grad, uint8_t* stop,
                                                     float* kl_at_stop, float* kl_out, const norm_args* norm_p,
                                                     norm_args norm) {
  // tested after the partial loads are issued (one round trip, not two), and made
  // block-uniform through LDS: block 0's wave 1 may raise *stop during this very
  // launch, so two waves of a later block could read different values
  const bool stopped = *stop;
  __shared__ float4 red[kRedSlices][kRedCols];
  __shared__ int s_stopped;
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
  if (threadIdx.x == 0) s_stopped = stopped;
  red[sl][c] = s;
  __syncthreads();
  if (s_stopped) return;  // block-uniform: KL early stop already hit
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
  float o4[4] = {};
  if (threadIdx.x < kRedCols) {  // (lanes past P take part in the norm tree with zeros)
    float4 t = red2[0][c];
    for (int k = 1; k < 8; ++k) {
      const float4 v = red2[k][c];
      t.x += v.x;
      t.y += v.y;
      t.z += v.z;
      t.w += v.w;
    }
    o4[0] = t.x, o4[1] = t.y, o4[2] = t.z, o4[3] = t.w;
    for (int q = 0; q < 4 && p4 + q < P; ++q) grad[p4 + q] = o4[q] * scale;
    if (norm_p) {  // per-tensor sums of squares of this block's 64 entries, lanes 0..15 in a fixed tree
      const int nt = norm.cfg.n_tensors;
      const int64_t b0 = (int64_t)blockIdx.x * 4 * kRedCols, b1 = b0 + 4 * kRedCols;
      for (int u = 0; u < nt; ++u) {
        const int64_t lo = norm.cfg.offsets[u], hi = norm.cfg.offsets[u + 1];
        float sq = 0.0f;
        if (!(hi <= b0 || lo >= b1)) {  // else: tensor outside this block (uniform over the 16 lanes)
          for (int k = 0; k < 4; ++k) {
            const float gk = o4[k] * scale;
            if (p4 + k < P && p4 + k >= lo && p4 + k < hi) sq = fmaf(gk, gk, sq);
          }
          for (int off = 1; off < kRedCols; off <<= 1) sq += __shfl_xor(sq, off, kRedCols);
        }
        if (threadIdx.x == 0) norm.ws[(size_t)blockIdx.x * nt + u] = sq;
      }
    }
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
    } else if (lane == 0 && norm_p) {
      const float st = *norm.step + 1.0f;  // the Adam step this minibatch takes
      *norm.step = st;
      rx_adam_scalars(norm.cfg, st, *norm.lr, norm.ws + (size_t)gridDim.x * norm.cfg.n_tensors);
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

constexpr int kAdvBatch = 16;  // k_adv_stats rows in flight per thread

__global__ __launch_bounds__(1024) void k_adv_stats(const float* __restrict__ adv, const int64_t* __restrict__ perm,
                                                    int mb, int64_t n_rows, float* stats, double* moments) {
  __shared__ double red[2][16];
  const int64_t base = (int64_t)blockIdx.x * mb;
  double s = 0.0, s2 = 0.0;
  // thread t adds rows t, t + 1024, ... in order; the perm indices and then the
  // gathered advantages of kAdvBatch rows are loaded before any is added, so a
  // batch costs two memory round trips instead of two per row
  for (int i0 = threadIdx.x; i0 < mb; i0 += 1024 * kAdvBatch) {
    int64_t k[kAdvBatch];
#pragma unroll
    for (int j = 0; j < kAdvBatch; ++j) {
      const int i = i0 + 1024 * j;
      k[j] = i < mb ? perm[base + i] : -1;
    }
    double x[kAdvBatch];
#pragma unroll
    for (int j = 0; j < kAdvBatch; ++j) x[j] = (k[j] >= 0 && k[j] < n_rows) ? adv[k[j]] : 0.0;
#pragma unroll
    for (int j = 0; j < kAdvBatch; ++j)
      if (i0 + 1024 * j < mb) {
        s += x[j];
        s2 += x[j] * x[j];
      }
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

// The same statistics spread over many workgroups (ABI v17, rx_ppo_adv_stats_ws):
// minibatch m is cut into chunks of kAdvChunk rows, one 256-thread workgroup
// each (thread t adds rows t, t + 256, ... of its chunk in order, every perm
// index and then every gathered advantage of its 8 rows in flight at once; a
// 64-lane xor tree, the 4 waves in order), which writes the chunk's (sum,
// square-sum) to ws[m][c]; k_adv_fold then adds a minibatch's chunks in chunk
// order.  n_mb * n_chunks workgroups gather instead of n_mb.
constexpr int kAdvChunk = 2048, kAdvT = 256, kAdvPer = kAdvChunk / kAdvT;

__global__ __launch_bounds__(kAdvT) void k_adv_chunk(const float* __restrict__ adv, const int64_t* __restrict__ perm,
                                                     int mb, int64_t n_rows, int n_chunks, double* __restrict__ ws) {
  __shared__ double red[2][kAdvT / 64];
  const int m = blockIdx.x / n_chunks, c = blockIdx.x - m * n_chunks;
  const int r0 = c * kAdvChunk, r1 = min(mb, r0 + kAdvChunk);
  const int64_t base = (int64_t)m * mb;
  int64_t k[kAdvPer];
#pragma unroll
  for (int j = 0; j < kAdvPer; ++j) {
    const int r = r0 + threadIdx.x + kAdvT * j;
    k[j] = r < r1 ? perm[base + r] : -1;
  }
  double x[kAdvPer];
#pragma unroll
  for (int j = 0; j < kAdvPer; ++j) x[j] = (k[j] >= 0 && k[j] < n_rows) ? (double)adv[k[j]] : 0.0;
  double s = 0.0, s2 = 0.0;
#pragma unroll
  for (int j = 0; j < kAdvPer; ++j) {
    s += x[j];
    s2 += x[j] * x[j];
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
    for (int w = 0; w < kAdvT / 64; ++w) {
      a += red[0][w];
      q += red[1][w];
    }
    ws[2 * (size_t)blockIdx.x] = a;
    ws[2 * (size_t)blockIdx.x + 1] = q;
  }
}

__global__ __launch_bounds__(64) void k_adv_fold(const double* __restrict__ ws, int n_mb, int n_chunks, int mb,
                                                 float* stats, double* moments) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n_mb) return;
  double a = 0.0, q = 0.0;
  for (int c = 0; c < n_chunks; ++c) {
    a += ws[2 * ((size_t)i * n_chunks + c)];
    q += ws[2 * ((size_t)i * n_chunks + c) + 1];
  }
  if (moments) {
    moments[2 * i] = a;
    moments[2 * i + 1] = q;
  } else {
    adv_write(a, q, (double)mb, stats, i);
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

extern "C" int rx_adv_chunks(int mb) { return (mb + kAdvChunk - 1) / kAdvChunk; }

extern "C" int rx_launch_adv_stats_ws(const rx_ppo_batch* b, int n_mb, double* ws, float* stats, double* moments,
                                      hipStream_t s) {
  const int nc = rx_adv_chunks(b->mb);
  hipLaunchKernelGGL(k_adv_chunk, dim3(n_mb * nc), dim3(kAdvT), 0, s, b->advantages, b->perm, b->mb, b->n_rows, nc,
                     ws);
  hipLaunchKernelGGL(k_adv_fold, dim3((n_mb + 63) / 64), dim3(64), 0, s, ws, n_mb, nc, b->mb, stats, moments);
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

#ifdef RX_PPO_STAMPS
// profiling build: copy the stamp array out ([kStampMaxWaves][kStampW] u64)
extern "C" int rx_ppo_stamps_read(unsigned long long* out, int n_waves) {
  const size_t n = (size_t)(n_waves < kStampMaxWaves ? n_waves : kStampMaxWaves) * kStampW;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ppo_stamps), n * sizeof(unsigned long long)) != hipSuccess) return -1;
  static unsigned long long zero[kStampMaxWaves * kStampW];
  return hipMemcpyToSymbol(HIP_SYMBOL(g_ppo_stamps), zero, sizeof zero) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int rx_ppo_reduce_blocks(int obs_dim) {
  const int Pp = obs_dim == 15 ? Lay<15>::Pp : Lay<19>::Pp;
  return (Pp + 4 * kRedCols - 1) / (4 * kRedCols);
}

extern "C" int rx_launch_ppo_grad(const rx_ppo_batch* b, int m, float scale, uint8_t* stop, float* kl_at_stop,
                                  float* kl_out, float* partial, double* klp, float* grad, hipStream_t s,
                                  const rx_adam_config* cfg, float* norm_ws, float* step, const double* lr) {
  const int rp = rows_per_wg(b->mb);
  const int n_wg = (b->mb + rp - 1) / rp;
  ppo_args a{*b, m, rp, stop, klp};
  int P, Pp;
  const bool bf = b->precision == kBF16;
  if (b->obs_dim == 15) {
    if (bf && RX_PPO_BF_FRAG)
      hipLaunchKernelGGL((k_ppo_grad_bf<15>), dim3(n_wg, 2), dim3(kGT), 0, s, a, b->params, partial);
    else if (bf)
      hipLaunchKernelGGL((k_ppo_grad<15, kBF16>), dim3(n_wg, 2), dim3(kGT), 0, s, a, b->params, partial);
    else
      hipLaunchKernelGGL((k_ppo_grad<15, kF32>), dim3(n_wg, 2), dim3(kGT), 0, s, a, b->params, partial);
    P = Lay<15>::P, Pp = Lay<15>::Pp;
  } else {
    if (bf && RX_PPO_BF_FRAG)
      hipLaunchKernelGGL((k_ppo_grad_bf<19>), dim3(n_wg, 2), dim3(kGT), 0, s, a, b->params, partial);
    else if (bf)
      hipLaunchKernelGGL((k_ppo_grad<19, kBF16>), dim3(n_wg, 2), dim3(kGT), 0, s, a, b->params, partial);
    else
      hipLaunchKernelGGL((k_ppo_grad<19, kF32>), dim3(n_wg, 2), dim3(kGT), 0, s, a, b->params, partial);
    P = Lay<19>::P, Pp = Lay<19>::Pp;
  }
  norm_args na{};
  const norm_args* np = nullptr;
  if (cfg) {
    na = norm_args{*cfg, norm_ws, step, lr};
    np = &na;  // only its non-nullness reaches the device: the struct travels by value
  }
  const int nb = rx_ppo_reduce_blocks(b->obs_dim);
  hipLaunchKernelGGL(k_ppo_reduce, dim3(nb), dim3(1024), 0, s, partial, klp, n_wg, P, Pp, b->mb, b->kl_target, scale,
                     grad, stop, kl_at_stop, kl_out, np, na);
  return (int)hipGetLastError();
}

extern "C" int rx_launch_selfplay_act(const rx_policy_io* ag, const rx_policy_io* op, float* obs_out,
                                      const float* rew_src, float* rew_out, int agent, hipStream_t s) {
  const int64_t blocks16 = (ag->n + 15) / 16;
  const int n_wg = (int)(3 * ((blocks16 + 3) / 4));
  const selfplay_copy cp{obs_out, rew_src, rew_out, agent};
  const bool ba = ag->precision == kBF16, bo = op->precision == kBF16;
  if (ba && bo)
    hipLaunchKernelGGL((k_selfplay_act<19, kBF16, kBF16>), dim3(n_wg), dim3(kT), 0, s, *ag, *op, cp);
  else if (ba)
    hipLaunchKernelGGL((k_selfplay_act<19, kBF16, kF32>), dim3(n_wg), dim3(kT), 0, s, *ag, *op, cp);
  else if (bo)
    hipLaunchKernelGGL((k_selfplay_act<19, kF32, kBF16>), dim3(n_wg), dim3(kT), 0, s, *ag, *op, cp);
  else
    hipLaunchKernelGGL((k_selfplay_act<19, kF32, kF32>), dim3(n_wg), dim3(kT), 0, s, *ag, *op, cp);
  return (int)hipGetLastError();
}

extern "C" int rx_launch_policy_act(const rx_policy_io* io, hipStream_t s, const void* frag) {
  // one wave per 16 rows and trunk, 4 waves (one trunk) per workgroup
  const int64_t blocks16 = (io->n + 15) / 16;
  const int n_wg = (int)(2 * ((blocks16 + 3) / 4));
  const bool bf = io->precision == kBF16;
  const bf8* fr = static_cast<const bf8*>(frag);
  if (io->obs_dim == 15) {
    if (bf && fr)
      hipLaunchKernelGGL((k_policy_act<15, kBF16, true>), dim3(n_wg), dim3(kT), 0, s, *io, io->params, fr);
    else if (bf)
      hipLaunchKernelGGL((k_policy_act<15, kBF16>), dim3(n_wg), dim3(kT), 0, s, *io, io->params, fr);
    else
      hipLaunchKernelGGL((k_policy_act<15, kF32>), dim3(n_wg), dim3(kT), 0, s, *io, io->params, fr);
  } else {
    if (bf && fr)
      hipLaunchKernelGGL((k_policy_act<19, kBF16, true>), dim3(n_wg), dim3(kT), 0, s, *io, io->params, fr);
    else if (bf)
      hipLaunchKernelGGL((k_policy_act<19, kBF16>), dim3(n_wg), dim3(kT), 0, s, *io, io->params, fr);
    else
      hipLaunchKernelGGL((k_policy_act<19, kF32>), dim3(n_wg), dim3(kT), 0, s, *io, io->params, fr);
  }
  return (int)hipGetLastError();
}

extern "C" size_t rx_policy_frag_bytes() { return 2 * (size_t)kFragTrunk * sizeof(bf8); }

extern "C" int rx_launch_policy_frag(int obs_dim, const float* params, void* img, hipStream_t s) {
  if (obs_dim == 15)
    hipLaunchKernelGGL(k_policy_frag<15>, dim3(2), dim3(256), 0, s, params, static_cast<bf8*>(img));
  else
    hipLaunchKernelGGL(k_policy_frag<19>, dim3(2), dim3(256), 0, s, params, static_cast<bf8*>(img));
  return (int)hipGetLastError();
}
