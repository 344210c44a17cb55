// rx_sort.hip -- the spatial re-sort of the env order (every sort_interval
// dynamics launches), which also MOVES the engine's working state: the env
// state lives in wave order (position p holds env perm[p]), so the kernels'
// state reads and writes are coalesced, and a re-sort permutes it.
// Scheduling only: no result depends on the order (test_culling_and_sort_are_exact).
//
// The key the REWARD half writes per perm position is a BIN: the slot's bin
// base (bases ascend with the slot id) + (closest waypoint >> shift), so bins
// of one slot are contiguous, slot groups keep their place in the perm, and
// the whole key space is <= RX_SORT_MAX_BINS (rx_assign picks the shift).  A
// counting sort over that small key space, four launches:
//   k_sort_hist     per wave: lanes grouped by bin (ballot), the group leaders'
//                   counts added in one vector atomic whose return values give
//                   every env its rank within its bin (rx_bin_count; the
//                   single-agent split step's REWARD half does this itself)
//   k_sort_scan     one workgroup: exclusive scan of the histogram -> cursors,
//                   histogram cleared for the next sort
//   k_sort_scatter  new position = cursor[bin] + rank (no atomics); the env id
//                   and its whole state row move there (into the shadow copy)
//   k_state_copy    shadow -> working copy (coalesced), so every launch keeps
//                   reading the same buffers (HIP-graph replay safe)
// The envs of a wave are track neighbours (the previous sort), so a wave sees
// only a handful of bins.  Order inside a bin follows the atomic order of the
// waves (not fixed run to run; nothing depends on it).
//
// rx_state_sync: the caller's bound arrays (env order) <-> the working copy.
#include <hip/hip_runtime.h>

#include "rx_internal.h"

namespace {

constexpr int kBlock = 256;
constexpr int kScanThreads = 1024;

__global__ __launch_bounds__(kBlock) void k_sort_hist(const uint32_t* __restrict__ keys, int n,
                                                       uint32_t* __restrict__ hist, uint32_t* __restrict__ off) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  off[i] = rx_bin_count(hist, keys[i]);
}

__global__ __launch_bounds__(kScanThreads) void k_sort_scan(uint32_t* __restrict__ hist,
                                                             uint32_t* __restrict__ cursor, int nbins) {
  __shared__ uint32_t part[kScanThreads];
  const int t = threadIdx.x;
  const int per = (nbins + kScanThreads - 1) / kScanThreads;
  const int b0 = t * per, b1 = min(nbins, b0 + per);
  uint32_t s = 0;
  for (int b = b0; b < b1; ++b) s += hist[b];
  part[t] = s;
  __syncthreads();
  for (int off = 1; off < kScanThreads; off <<= 1) {  // Hillis-Steele inclusive scan of the thread sums
    const uint32_t x = t >= off ? part[t - off] : 0u;
    __syncthreads();
    part[t] += x;
    __syncthreads();
  }
  uint32_t run = part[t] - s;  // exclusive
  for (int b = b0; b < b1; ++b) {
    const uint32_t c = hist[b];
    cursor[b] = run;
    run += c;
    hist[b] = 0u;
  }
}

// one env's state row (position i of a working copy), held in registers
template <int A>
struct Row {
  double f[A][8];
  int32_t fs[A];
  uint8_t fl[A];
  int32_t steps, epl;
  uint8_t ef;
  double epr;
  __device__ __forceinline__ void load(const rx_state& src, int i) {
#pragma unroll
    for (int q = 0; q < A; ++q) {
      const int si = A * i + q;
      f[q][0] = src.x[si];
      f[q][1] = src.y[si];
      f[q][2] = src.angle[si];
      f[q][3] = src.vx[si];
      f[q][4] = src.vy[si];
      f[q][5] = src.progress[si];
      f[q][6] = src.last_progress[si];
      f[q][7] = src.last_steering[si];
      fl[q] = src.flags[si];
      fs[q] = src.finished_step ? src.finished_step[si] : 0;
    }
    steps = src.steps[i];
    ef = src.env_flags[i];
    epr = src.ep_return[i];
    epl = src.ep_length[i];
  }
  __device__ __forceinline__ void store(const rx_state& dst, int j) const {
#pragma unroll
    for (int q = 0; q < A; ++q) {
      const int di = A * j + q;
      dst.x[di] = f[q][0];
      dst.y[di] = f[q][1];
      dst.angle[di] = f[q][2];
      dst.vx[di] = f[q][3];
      dst.vy[di] = f[q][4];
      dst.progress[di] = f[q][5];
      dst.last_progress[di] = f[q][6];
      dst.last_steering[di] = f[q][7];
      dst.flags[di] = fl[q];
      if (dst.finished_step) dst.finished_step[di] = fs[q];
    }
    dst.steps[j] = steps;
    dst.env_flags[j] = ef;
    dst.ep_return[j] = epr;
    dst.ep_length[j] = epl;
  }
};

// one env's state row: working-state element i (position) -> j
template <int A>
__device__ __forceinline__ void move_row(const rx_state& src, int i, const rx_state& dst, int j) {
  Row<A> r;
  r.load(src, i);
  r.store(dst, j);
}

template <int A>
__global__ __launch_bounds__(kBlock) void k_sort_scatter(const uint32_t* __restrict__ keys,
                                                          const uint32_t* __restrict__ off, int n,
                                                          const uint32_t* __restrict__ cursor,
                                                          const int32_t* __restrict__ perm,
                                                          int32_t* __restrict__ perm_tmp, rx_state work,
                                                          rx_state tmp) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint32_t dst = cursor[keys[i]] + off[i];
  perm_tmp[dst] = perm[i];
  move_row<A>(work, i, tmp, (int)dst);
}

// Up to kFusedBins bins the scan runs inside the scatter: every workgroup
// scans the whole histogram in LDS (at most 32 KB, read from L2) and takes its
// cursors from there -- one launch and its kernel boundary fewer per re-sort;
// k_state_copy then clears the histogram (every scatter workgroup has read it).
constexpr int kFusedBins = 8192;

template <int A>
__global__ __launch_bounds__(kBlock) void k_sort_scatter_scan(const uint32_t* __restrict__ keys,
                                                               const uint32_t* __restrict__ off, int n,
                                                               const uint32_t* __restrict__ hist, int nbins,
                                                               const int32_t* __restrict__ perm,
                                                               int32_t* __restrict__ perm_tmp, rx_state work,
                                                               rx_state tmp) {
  __shared__ uint32_t cur[kFusedBins];
  __shared__ uint32_t wtot[kBlock / 64];
  const int t = threadIdx.x, i = blockIdx.x * kBlock + t;
  const bool v = i < n;
  // the env's key, rank, id and state row are loaded first: their latency overlaps the scan
  uint32_t key = 0, rk = 0;
  int32_t id = 0;
  Row<A> r;
  if (v) {
    key = keys[i];
    rk = off[i];
    id = perm[i];
    r.load(work, i);
  }
  for (int b = t; b < nbins; b += kBlock) cur[b] = hist[b];
  __syncthreads();
  const int per = (nbins + kBlock - 1) / kBlock;
  const int b0 = min(nbins, t * per), b1 = min(nbins, b0 + per);
  uint32_t s = 0;
  for (int b = b0; b < b1; ++b) s += cur[b];
  const int lane = t & 63, w = t >> 6;
  uint32_t inc = s;  // inclusive scan of the thread sums within the wave, then over the wave totals
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  if (lane == 63) wtot[w] = inc;
  __syncthreads();
  uint32_t run = inc - s;
  for (int k = 0; k < w; ++k) run += wtot[k];
  for (int b = b0; b < b1; ++b) {  // this thread's chunk of bins -> exclusive cursors
    const uint32_t c = cur[b];
    cur[b] = run;
    run += c;
  }
  __syncthreads();
  if (!v) return;
  const uint32_t dst = cur[key] + rk;
  perm_tmp[dst] = id;
  r.store(tmp, (int)dst);
}

// shadow -> working copy; with hist, also clears the histogram (fused-scan re-sort)
template <int A>
__global__ __launch_bounds__(kBlock) void k_state_copy(int n, const int32_t* __restrict__ perm_tmp,
                                                        int32_t* __restrict__ perm, rx_state tmp, rx_state work,
                                                        uint32_t* __restrict__ hist, int nbins) {
  const int j = blockIdx.x * kBlock + threadIdx.x;
  for (int b = j; b < nbins; b += (int)gridDim.x * kBlock) hist[b] = 0u;
  if (j >= n) return;
  perm[j] = perm_tmp[j];
  move_row<A>(tmp, j, work, j);
}

// to_user: working row p -> the caller's row perm[p]; else the reverse
template <int A>
__global__ __launch_bounds__(kBlock) void k_state_sync(int n, const int32_t* __restrict__ perm, rx_state work,
                                                        rx_state user, int to_user) {
  const int p = blockIdx.x * kBlock + threadIdx.x;
  if (p >= n) return;
  const int e = perm[p];
  if (to_user)
    move_row<A>(work, p, user, e);
  else
    move_row<A>(user, e, work, p);
}

// rx_random_permutation: a pseudo-random permutation of [0, n) in one
// launch (the device minibatch shuffle, config["shuffle"] = "device").  A
// 4-round UNBALANCED Feistel network on bits = ceil(log2 n) bits (halves of
// a = bits / 2 and b = bits - a bits; round k maps the current right half
// through F into the width of the left one, then the halves swap, so after the
// even number of rounds the widths are back) is a bijection of [0, 2^bits);
// cycle-walking (apply it again while the value is >= n) turns it into a
// bijection of [0, n), fewer than 2 walks on average since 2^bits < 2n, none
// when n is a power of two (configs[1]: n = 2^19).  Round 6: the balanced
// network of rounds 3-5 ran on 2 ceil(bits / 2) bits (2^20 for 2^19 rows, two
// walks on average and a wave waiting for its longest lane's chain).
// Round function: the splitmix64 finalizer of (half ^ round key).
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__global__ __launch_bounds__(kBlock) void k_feistel_perm(int64_t n, int bits, uint64_t seed,
                                                          int64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const int a = bits >> 1, b = bits - a;  // left / right widths of the input
  uint64_t key[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) key[k] = mix64(seed + 0x9e3779b97f4a7c15ull * (uint64_t)(k + 1));
  uint64_t x = (uint64_t)i;
  do {
    int wl = a, wr = b;
    uint64_t l = x >> wr, r = x & ((1ull << wr) - 1ull);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint64_t t = l ^ (mix64(r ^ key[k]) & ((1ull << wl) - 1ull));
      l = r;
      r = t;
      const int w = wl;
      wl = wr;
      wr = w;
    }
    x = (l << wr) | r;
  } while (x >= (uint64_t)n);
  out[i] = (int64_t)x;
}

}  // namespace

extern "C" int rx_sort_envs(const uint32_t* keys, uint32_t* off, int n, int A, uint32_t* hist, uint32_t* cursor, int nbins,
                            int32_t* perm, int32_t* perm_tmp, const rx_state* work, const rx_state* tmp,
                            hipStream_t s, int hist_done) {
  if (n <= 0) return 0;
  if (nbins <= 0 || nbins > RX_SORT_MAX_BINS || (A != 1 && A != 2)) return (int)hipErrorInvalidValue;
  const int grid = (n + kBlock - 1) / kBlock;
  // hist_done: the step's REWARD half counted the bins while writing the keys
  if (!hist_done) hipLaunchKernelGGL(k_sort_hist, dim3(grid), dim3(kBlock), 0, s, keys, n, hist, off);
  if (nbins <= kFusedBins) {
    if (A == 1) {
      hipLaunchKernelGGL(k_sort_scatter_scan<1>, dim3(grid), dim3(kBlock), 0, s, keys, off, n, hist, nbins, perm,
                         perm_tmp, *work, *tmp);
      hipLaunchKernelGGL(k_state_copy<1>, dim3(grid), dim3(kBlock), 0, s, n, perm_tmp, perm, *tmp, *work, hist, nbins);
    } else {
      hipLaunchKernelGGL(k_sort_scatter_scan<2>, dim3(grid), dim3(kBlock), 0, s, keys, off, n, hist, nbins, perm,
                         perm_tmp, *work, *tmp);
      hipLaunchKernelGGL(k_state_copy<2>, dim3(grid), dim3(kBlock), 0, s, n, perm_tmp, perm, *tmp, *work, hist, nbins);
    }
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(k_sort_scan, dim3(1), dim3(kScanThreads), 0, s, hist, cursor, nbins);
  if (A == 1) {
    hipLaunchKernelGGL(k_sort_scatter<1>, dim3(grid), dim3(kBlock), 0, s, keys, off, n, cursor, perm, perm_tmp, *work,
                       *tmp);
    hipLaunchKernelGGL(k_state_copy<1>, dim3(grid), dim3(kBlock), 0, s, n, perm_tmp, perm, *tmp, *work, nullptr, 0);
  } else {
    hipLaunchKernelGGL(k_sort_scatter<2>, dim3(grid), dim3(kBlock), 0, s, keys, off, n, cursor, perm, perm_tmp, *work,
                       *tmp);
    hipLaunchKernelGGL(k_state_copy<2>, dim3(grid), dim3(kBlock), 0, s, n, perm_tmp, perm, *tmp, *work, nullptr, 0);
  }
  return (int)hipGetLastError();
}

extern "C" int rx_state_sync(const rx_state* work, const rx_state* user, const int32_t* perm, int n, int A,
                             int to_user, hipStream_t s) {
  if (n <= 0) return 0;
  if (A != 1 && A != 2) return (int)hipErrorInvalidValue;
  const int grid = (n + kBlock - 1) / kBlock;
  if (A == 1)
    hipLaunchKernelGGL(k_state_sync<1>, dim3(grid), dim3(kBlock), 0, s, n, perm, *work, *user, to_user);
  else
    hipLaunchKernelGGL(k_state_sync<2>, dim3(grid), dim3(kBlock), 0, s, n, perm, *work, *user, to_user);
  return (int)hipGetLastError();
}

extern "C" int rx_launch_permutation(int64_t n, uint64_t seed, int64_t* out, hipStream_t s) {
  if (n <= 0) return 0;
  int bits = 1;
  while (bits < 62 && (1ll << bits) < n) ++bits;  // 2^bits >= n and < 2n (cycle-walk length)
  const int64_t grid = (n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(k_feistel_perm, dim3((unsigned)grid), dim3(kBlock), 0, s, n, bits, seed, out);
  return (int)hipGetLastError();
}
