// rx_kernels.hip -- batched racing-env step + GAE kernels for gfx950 (MI355X).
//
// Design:
//  * Envs are grouped by track slot on the host (rx_assign); every wavefront
//    works on ONE slot, so the track's waypoints/segments are wave-uniform and
//    are read with scalar loads (s_load) into SGPRs: no LDS staging, no bank
//    conflicts, and the VALU ops take the segment coordinates as SGPR
//    operands.  The wave tables (WaveEntry) are built once per assignment.
//  * k_dyn: one lane per env.  Car dynamics, progress/collision argmins over the
//    waypoints (all 5 query points -- centre + 4 corners -- in ONE pass over
//    the wave-uniform waypoint stream), reward, done, autoreset, episode stats,
//    and the non-ray observation columns.
//  * k_rays: one lane per (env, agent, ray): 11x more lanes than envs, so even
//    65,536 envs give ~11 waves per SIMD for latency hiding.  Exact,
//    division-free hit test per segment (derivation in DESIGN.md §Raycast);
//    one f64 division per HIT segment only.
//  * Arithmetic: binary64, the reference's operation order, compiled with
//    -ffp-contract=off; explicit FMAs only where the reference calls np.dot.
//    sin/cos = rx_sincos (correctly rounded), pow(x,2) = x*x (rx_math.h).
//  * k_gae / k_gae_scan: agent/ppo.py:134-154 in float32.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>
#include <stdint.h>

#include "rx.h"
#include "rx_internal.h"
#include "rx_math.h"
#include "rx_policy.h"

#define RX_TWO_PI 6.283185307179586  // 2*np.pi, environment/car.py:54
#define RX_MAX_SPEED 30.0
#define RX_DT 0.05
#define RX_MAX_RANGE 50.0

namespace {

struct Car {
  double x, y, angle, vx, vy, progress;
  bool crashed;
};

__device__ __forceinline__ int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }
// a wave-uniform double into an SGPR pair (a value loaded from a uniform address
// the compiler cannot prove unclobbered otherwise occupies two VGPRs)
__device__ __forceinline__ double uniform_d(double v) {
  const unsigned long long u = __double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)u);
  const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(u >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

__device__ __forceinline__ unsigned long long uniform64(unsigned long long v) {
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v), hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return ((unsigned long long)hi << 32) | lo;
}

// State accesses of the env device functions (plain loads and stores).
template <class T>
__device__ __forceinline__ T ldc(const T* p) {
  return *p;
}
template <class T, class U>
__device__ __forceinline__ void stc(T* p, U v) {
  *p = (T)v;
}

// f32 np.clip with Python-float bounds (stays float32 under NEP 50)
// Load of track-table data at a wave-uniform address through the constant
// address space: the tables are never written by a kernel, and the cast lets
// the compiler issue s_load (scalar cache, SGPR operands) even after the
// kernel's first global store -- a generic pointer loses that proof at the
// first store (the REWARD half's) and falls back to vector loads.
#ifdef RX_NO_LDU  // A/B knob: plain generic loads
typedef const double* rx_cdp;
typedef const float* rx_cfp;
#else
typedef const __attribute__((address_space(4))) double* rx_cdp;
typedef const __attribute__((address_space(4))) float* rx_cfp;
#endif
__device__ __forceinline__ double ldu(const double* p) { return *(rx_cdp)p; }
__device__ __forceinline__ double2 ldu(const double2* p) {
  const rx_cdp q = (rx_cdp)(const double*)p;
  return make_double2(q[0], q[1]);
}
__device__ __forceinline__ double4 ldu(const double4* p) {
  const rx_cdp q = (rx_cdp)(const double*)p;
  return make_double4(q[0], q[1], q[2], q[3]);
}
__device__ __forceinline__ float4 ldu(const float4* p) {
  const rx_cfp q = (rx_cfp)(const float*)p;
  return make_float4(q[0], q[1], q[2], q[3]);
}

// Lane-varying track slots (rx_config.lane_tracks, DESIGN.md §3 "Lane-varying
// track slots"): with LV the lanes of a wave may belong to different slots, so a
// track-table read is a per-lane vector load and every culling decision is the
// lane's own; without it the wave's slot is uniform -- scalar loads (ldu), wave
// votes, SGPR indices.  The arithmetic is the same either way, and no result
// depends on which boxes a lane skips (the culling is exact), so both forms give
// bit-identical outputs.
template <bool LV, class T>
__device__ __forceinline__ T ldt(const T* p) {
  if constexpr (LV)
    return *p;
  else
    return ldu(p);
}
template <bool LV>
__device__ __forceinline__ int uni(int v) {
  if constexpr (LV)
    return v;
  else
    return uniform(v);
}
template <bool LV>
__device__ __forceinline__ bool vote(bool b) {
  if constexpr (LV)
    return b;
  else
    return __any(b);
}

__device__ __forceinline__ float clipf(float a, float lo, float hi) {
  float y = a < lo ? lo : a;
  return y > hi ? hi : y;
}

// Car.get_corners -- environment/car.py:26-43, given cos/sin of the angle
__device__ __forceinline__ void corners(double x, double y, double c, double s, double cx[4], double cy[4]) {
  // local (2,1), (2,-1), (-2,-1), (-2,1): products by +-2 / +-1 are exact
  cx[0] = (c * 2.0 + (-s) * 1.0) + x;
  cy[0] = (s * 2.0 + c * 1.0) + y;
  cx[1] = (c * 2.0 + (-s) * -1.0) + x;
  cy[1] = (s * 2.0 + c * -1.0) + y;
  cx[2] = (c * -2.0 + (-s) * -1.0) + x;
  cy[2] = (s * -2.0 + c * -1.0) + y;
  cx[3] = (c * -2.0 + (-s) * 1.0) + x;
  cy[3] = (s * -2.0 + c * 1.0) + y;
}

// Argmin over a wave-uniform waypoint stream for NP query points per lane
// (Track.closest_waypoint_idx, environment/track.py:150-152: array `**2` is a
// square, first index on ties).  act[p] masks points whose car is frozen.
template <int NP>
__device__ __forceinline__ void argmin_pts(const double2* __restrict__ wp, int W, const double px[NP],
                                           const double py[NP], int idx[NP]) {
  double best[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    best[p] = __builtin_inf();
    idx[p] = 0;
  }
#pragma unroll 2
  for (int i = 0; i < W; ++i) {
    const double2 w = ldu(wp + i);  // uniform address -> s_load_dwordx4
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      double dx = w.x - px[p], dy = w.y - py[p];
      double d = dx * dx + dy * dy;
      bool lt = d < best[p];
      best[p] = lt ? d : best[p];
      idx[p] = lt ? i : idx[p];
    }
  }
}

// Closest waypoint of the car's previous position (progress = idx / W exactly).
__device__ __forceinline__ int prev_waypoint(double progress, int W) {
  int i = (int)(progress * (double)W + 0.5);
  return i < 0 ? 0 : (i >= W ? W - 1 : i);
}

// Order-independent argmin update: smaller distance, or equal distance and a
// smaller index -- the same result as the reference's first-index argmin
// whatever order the waypoints are visited in.
__device__ __forceinline__ void argmin_take(double d, int i, double& best, int& idx) {
  const bool take = (d < best) | ((d == best) & (i < idx));
  best = take ? d : best;
  idx = take ? i : idx;
}

// May a waypoint box hold a waypoint at squared distance <= best[p] from some
// point p of the lane?  Tested once per car, from the car centre: every point p
// of car q lies within RX_CAR_RADIUS of the car centre c_q, so
// dist(p, box) >= dist(c_q, box) - RX_CAR_RADIUS, and a box with
// dist(c_q, box)^2 > T_q = (RX_CAR_RADIUS + sqrt(max_p best_p))^2 (inflated by
// 2^-40 relative + 1e-12) can hold no waypoint at distance <= any of the car's
// bests.  One distance bound per car instead of one per point.
#define RX_CAR_RADIUS 2.23607  // >= |corner - centre| = sqrt(2^2 + 1^2) = 2.2360680 (car.py:26-43)
template <int NC, bool LV = false>
__device__ __forceinline__ bool box_may_hold_c(const double* __restrict__ b, const double cxs[NC], const double cys[NC],
                                               const double T[NC]) {
  double x0, y0, x1, y1;
  if constexpr (LV) {  // one 32-byte box: two dwordx4 vector loads
    const double4 v = *reinterpret_cast<const double4*>(b);
    x0 = v.x, y0 = v.y, x1 = v.z, y1 = v.w;
  } else {
    x0 = ldu(b), y0 = ldu(b + 1), x1 = ldu(b + 2), y1 = ldu(b + 3);
  }
  bool need = false;
#pragma unroll
  for (int q = 0; q < NC; ++q) {
    const double gx = __builtin_fmax(__builtin_fmax(x0 - cxs[q], cxs[q] - x1), 0.0);
    const double gy = __builtin_fmax(__builtin_fmax(y0 - cys[q], cys[q] - y1), 0.0);
    need = need | !(gx * gx + gy * gy > T[q]);
  }
  return need;
}

template <int NP, int NC>
__device__ __forceinline__ void car_thresholds(const double best[NP], double T[NC], bool active = true) {
  constexpr int PPC = NP / NC;
#pragma unroll
  for (int q = 0; q < NC; ++q) {
    double m = best[q * PPC];
#pragma unroll
    for (int p = q * PPC + 1; p < (q + 1) * PPC; ++p) m = __builtin_fmax(m, best[p]);
    const double r = RX_CAR_RADIUS + __builtin_sqrt(m);
    T[q] = active ? (r * r) * (1.0 + 0x1p-40) + 1e-12 : -1.0;  // -1: needs no box (result unused)
  }
}

// The same argmin with culling (exact).  Phase 1: every lane scans a window
// of 2H+1 waypoints around ITS car's previous closest waypoint (per-lane
// gathers; the car moved <= 1.5 units, so the window nearly always holds the
// answer).  Phase 2: the slot's waypoint chunks are visited wave-uniformly;
// a chunk is scanned (scalar loads) only if for some lane and point the
// box's squared distance lower bound does not exceed that point's best.
// The bound is shrunk by 2^-46 relative, far beyond the few-ulp rounding of
// both the bound and the per-waypoint distances, so a skipped chunk can
// neither beat nor tie the best (ties are broken by index, argmin_take).
template <int NP, int NC, bool LV = false>
__device__ __forceinline__ void argmin_culled(const double2* __restrict__ wp, const double* __restrict__ wbox,
                                              const double* __restrict__ wsbox, int W,
                                              const double px[NP], const double py[NP], const int prev[NC],
                                              const double cxs[NC], const double cys[NC], int H, int idx[NP],
                                              unsigned long long* counters, unsigned long long* stamps = nullptr,
                                              bool active = true) {
  constexpr int PPC = NP / NC;  // points per car (the lane's points of each car)
  double best[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    best[p] = __builtin_inf();
    idx[p] = 0x7fffffff;
  }
#pragma unroll
  for (int q = 0; q < NC; ++q) {
    for (int j = -H; j <= H; ++j) {
      int i = prev[q] + j;
      i = i < 0 ? i + W : (i >= W ? i - W : i);
      const double2 w = wp[i];  // per-lane gather (L1/L2 resident)
#pragma unroll
      for (int p = q * PPC; p < (q + 1) * PPC; ++p) {
        const double dx = w.x - px[p], dy = w.y - py[p];
        argmin_take(dx * dx + dy * dy, i, best[p], idx[p]);
      }
    }
  }
  // two levels: super-chunks of RX_WP_SUPER leaves of RX_WP_CHUNK waypoints.
  // The super-chunk tests use the window's bests (an upper bound of the final
  // ones, so the set is conservative) and are branch-free, so their scalar
  // loads are all in flight together -- one latency instead of one per super.
  // Needed super-chunks are then visited outward from the wave's first car and
  // their leaves tested against the running bests.
#ifdef RX_DYN_STAMPS
  if (stamps) {
    __builtin_amdgcn_s_waitcnt(0);
    stamps[0] = __builtin_amdgcn_s_memtime();
  }
#endif
  const int nwc = (W + RX_WP_CHUNK - 1) / RX_WP_CHUNK;
  const int nws = (nwc + RX_WP_SUPER - 1) / RX_WP_SUPER;  // <= 64 (W <= 64 * RX_WP_CHUNK * RX_WP_SUPER)
  unsigned long long smask = 0;
  double T[NC];
  car_thresholds<NP, NC>(best, T, active);
#pragma unroll 4
  for (int u = 0; u < nws; ++u)
    smask |= (unsigned long long)(vote<LV>(box_may_hold_c<NC, LV>(wsbox + 4 * u, cxs, cys, T)) ? 1 : 0) << u;
  if constexpr (!LV) smask = uniform64(smask);
#ifdef RX_DYN_STAMPS
  if (stamps) {
    __builtin_amdgcn_s_waitcnt(0);
    stamps[1] = __builtin_amdgcn_s_memtime();
  }
#endif
  const int u0 = uni<LV>(prev[0] / (RX_WP_CHUNK * RX_WP_SUPER));
  int scanned = 0, tested = nws;
  for (int s = 0; s < nws; ++s) {
    const int off = (s + 1) >> 1;
    const bool back = (s & 1) != 0;
    int u = back ? u0 - off : u0 + off;
    u = u < 0 ? u + nws : (u >= nws ? u - nws : u);
    if (!((smask >> u) & 1ull)) continue;
    const int l0 = u * RX_WP_SUPER, nl = min(nwc, l0 + RX_WP_SUPER) - l0;
    for (int q = 0; q < nl; ++q) {
      const int c = l0 + (back ? nl - 1 - q : q);
      ++tested;  // T is current: the bests change only inside a leaf scan, which refreshes it
      if (!vote<LV>(box_may_hold_c<NC, LV>(wbox + 4 * c, cxs, cys, T))) continue;
      ++scanned;
      const int i1 = min(W, (c + 1) * RX_WP_CHUNK);
      int i = c * RX_WP_CHUNK;
      for (; i + 4 <= i1; i += 4) {  // four waypoints per batch of scalar loads
        const double2 w[4] = {ldt<LV>(wp + i), ldt<LV>(wp + i + 1), ldt<LV>(wp + i + 2), ldt<LV>(wp + i + 3)};
#pragma unroll
        for (int v = 0; v < 4; ++v) {
#pragma unroll
          for (int p = 0; p < NP; ++p) {
            const double dx = w[v].x - px[p], dy = w[v].y - py[p];
            argmin_take(dx * dx + dy * dy, i + v, best[p], idx[p]);
          }
        }
      }
      for (; i < i1; ++i) {
        const double2 w = ldt<LV>(wp + i);
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          const double dx = w.x - px[p], dy = w.y - py[p];
          argmin_take(dx * dx + dy * dy, i, best[p], idx[p]);
        }
      }
      car_thresholds<NP, NC>(best, T, active);
    }
  }
#ifndef RX_DYN_STAMPS  // the stamp build reuses io.counters for its stamps: no culling counts there
  if (counters && (LV || (threadIdx.x & 63) == (__builtin_amdgcn_readfirstlane(threadIdx.x) & 63))) {
    atomicAdd(&counters[2], (unsigned long long)tested);  // LV: every lane its own tests
    atomicAdd(&counters[3], (unsigned long long)scanned);
  }
#endif
}

// Wide closest-waypoint argmin (one env per wave, dyn_lpe 64, small N): for
// each of the car's 5 points the 64 lanes split the slot's waypoints (lane l
// takes i = l, l + 64, ...; coalesced gathers) and combine (distance, index)
// in a lexicographic wave minimum: the reference's first-index argmin
// (track.py:150-152) whatever the split.  All 64 lanes must be active; lane
// P < 5 keeps point P's index.
__device__ __forceinline__ void argmin_wave_take(const double2 w, int i, const double px[5], const double py[5],
                                                 double best[5], int bi[5]) {
#pragma unroll
  for (int p = 0; p < 5; ++p) {
    const double dx = w.x - px[p], dy = w.y - py[p];
    const double d = dx * dx + dy * dy;
    if (d < best[p]) {  // ascending i per lane: strict < keeps the first index
      best[p] = d;
      bi[p] = i;
    }
  }
}

__device__ __forceinline__ int argmin_wave(const double2* __restrict__ wp, int W, const double px[5],
                                           const double py[5], int P) {
  const int l = threadIdx.x & 63;
  double best[5];
  int bi[5];
#pragma unroll
  for (int p = 0; p < 5; ++p) {
    best[p] = __builtin_inf();
    bi[p] = 0x7fffffff;
  }
  // every waypoint is loaded once for the 5 points, four loads in flight at a time
  int i = l;
  for (; i + 192 < W; i += 256) {
    const double2 w0 = wp[i], w1 = wp[i + 64], w2 = wp[i + 128], w3 = wp[i + 192];
    argmin_wave_take(w0, i, px, py, best, bi);
    argmin_wave_take(w1, i + 64, px, py, best, bi);
    argmin_wave_take(w2, i + 128, px, py, best, bi);
    argmin_wave_take(w3, i + 192, px, py, best, bi);
  }
  for (; i < W; i += 64) argmin_wave_take(wp[i], i, px, py, best, bi);
  int mine = 0;
#pragma unroll
  for (int p = 0; p < 5; ++p) {
    double bp = best[p];
    int ip = bi[p];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double ob = __shfl_xor(bp, o, 64);
      const int oi = __shfl_xor(ip, o, 64);
      const bool take = (ob < bp) | ((ob == bp) & (oi < ip));
      bp = take ? ob : bp;
      ip = take ? oi : ip;
    }
    if (p == P) mine = ip;
  }
  return mine;
}

// Car.update -- environment/car.py:45-80, minus the argmins (done by the
// caller for all cars of the lane in one pass).  Returns cos/sin of the new
// angle and the 4 corners.
__device__ __forceinline__ void car_kinematics(Car& c, double steering, double throttle, double cs[2],
                                               double cx[4], double cy[4]) {
  double angular_velocity = steering * 3.0;
  double ang = c.angle + (angular_velocity * RX_DT);
  ang = rx_pymod(ang, RX_TWO_PI);
  double s, co;
  rx_sincos(ang, &s, &co);
  double vf = c.vx * co + c.vy * s;
  double vl = c.vx * (-s) + c.vy * co;
  double accel_forward = throttle * 10.0;
  vf = (vf + (accel_forward * RX_DT)) * 0.985;
  vl = (vl * 0.85) * 0.9;
  double vx = vf * co - vl * s;
  double vy = vf * s + vl * co;
  double speed = __builtin_sqrt(rx_sq(vx) + rx_sq(vy));
  if (speed > RX_MAX_SPEED) {
    double scale = RX_MAX_SPEED / speed;
    vx *= scale;
    vy *= scale;
  }
  c.angle = ang;
  c.vx = vx;
  c.vy = vy;
  c.x = c.x + (vx * RX_DT);
  c.y = c.y + (vy * RX_DT);
  cs[0] = co;
  cs[1] = s;
  corners(c.x, c.y, co, s, cx, cy);
}

// Track.check_collision for one corner given its argmin -- track.py:163-171
__device__ __forceinline__ bool corner_out(const double2* __restrict__ wp, const double2* __restrict__ nrm, int idx,
                                           double cx, double cy, double width) {
  double2 w = wp[idx];
  double2 n = nrm[idx];
  double px = cx - w.x, py = cy - w.y;
  double dist = __builtin_fabs(rx_dot2_np(px, py, n.x, n.y));
  return dist > width;
}

__device__ __forceinline__ double speed_of(double vx, double vy) { return __builtin_sqrt(rx_sq(vx) + rx_sq(vy)); }

// Spatial-coherence key for the next wave assignment: the sort bin of (slot,
// waypoint of the car).  Sorting by it (rx_sort_envs) keeps slot groups in
// place and puts cars that are near each other on the track into the same
// wavefronts, which is what makes k_rays' per-wave chunk culling effective.
// Pure scheduling: results never depend on the order.
__device__ __forceinline__ void write_sort_key(const rx_kargs& a, int pos, int k, double progress, int W) {
  if (!a.sort_keys) return;
  int w = (int)(progress * (double)W + 0.5);
  w = w < 0 ? 0 : (w > W ? W : w);
  const uint32_t key = (uint32_t)(a.sort_base[k] + (w >> a.sort_shift));
  a.sort_keys[pos] = key;
  if (a.sort_hist)  // the re-sort's histogram and each env's rank in its bin (k_sort_hist's work)
    a.sort_off[pos] = rx_bin_count(a.sort_hist, key);
}

// ray_order 2: the (agent, ray) tasks of a dynamics wave's envs (64 track
// neighbours after the spatial sort) are ordered by the absolute direction
// of the ray (64 sectors) before k_rays runs, so each of the block's ray waves
// holds nearly parallel rays from nearby origins, whichever env they belong to.
// A per-wave counting sort in LDS: ds_add_rtn ranks every task in its sector,
// a 64-lane scan turns the sector counts into offsets, and the task ids are
// written to tasks_out[perm_start*A*R ..] as (A*p + q)*R + r with p the
// env's position.  Runs every step with all 64 lanes of the wave (env lanes
// have p >= 0).  The direction is the car's new angle
// (the one k_rays casts from).  Scheduling only: no result depends on it.
#define RX_IO_ROW(a, pos) ((a).perm[(pos)])
constexpr int kTaskSectors = 64;
template <int A>
__device__ __forceinline__ int sort_block_tasks_lds(const rx_kargs& a, int p, const double* ang, int32_t* cnt,
                                                    int32_t* stage) {
  constexpr int kMaxT = 16 * A;  // rx_assign enforces n_sensors <= 16 for ray_order 2
  const int R = a.n_sensors, AR = A * R;
  const int lane = threadIdx.x & 63;
  const float inv = (float)kTaskSectors * 0.15915494309189535f;  // sectors per radian
  int pk[kMaxT];  // (rank << 6) | sector per task
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if (p >= 0) {
#pragma unroll
    for (int t = 0; t < kMaxT; ++t)
      if (t < AR) {
        const int q = t / R, r = t - (t / R) * R;
        const float th = (float)(ang[q] + a.rel_angles[r]);
        const int sec = (int)__builtin_floorf(th * inv) & (kTaskSectors - 1);
        pk[t] = (atomicAdd(&cnt[sec], 1) << 6) | sec;
      }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
#ifdef RX_DYN_STAMPS  // profiling build: the sort's own phases (ranks | scan + scatter | row copy)
  __builtin_amdgcn_s_waitcnt(0);
  const unsigned long long ts1 = __builtin_amdgcn_s_memtime();
#endif
  const int c0 = cnt[lane];
  int c = c0;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(c, o, 64);
    if (lane >= o) c += v;
  }
  cnt[lane] = c - c0;  // exclusive offset of sector `lane`
  const int total = __shfl(c, 63, 64);  // the block's tasks (AR per env lane)
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
  // scatter the task ids into the wave's LDS staging row, then store the row
  // coalesced (each of them was a scattered 4-byte global store: 704 per wave)
  if (p >= 0) {
#pragma unroll
    for (int t = 0; t < kMaxT; ++t)
      if (t < AR) stage[cnt[pk[t] & 63] + (pk[t] >> 6)] = A * p * R + t;  // task id (A*p + q)*R + r
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
#ifdef RX_DYN_STAMPS
  __builtin_amdgcn_s_waitcnt(0);
  const unsigned long long ts2 = __builtin_amdgcn_s_memtime();
  if (a.io.counters && lane == 0 && blockDim.x == 64) {  // k_kin1: one wave per workgroup
    a.io.counters[16 + 12 * (int)blockIdx.x + 10] = ts1;
    a.io.counters[16 + 12 * (int)blockIdx.x + 11] = ts2;
  }
#endif
  return total;
}

// the block's sorted task ids from the LDS row to tasks_out[perm_start*A*R ..],
// 64-lane contiguous stores (k_kin1 / k_dyn)
template <int A>
__device__ __forceinline__ void sort_block_tasks(const rx_kargs& a, int perm_start, int p, const double* ang,
                                                 int32_t* cnt, int32_t* stage) {
  const int total = sort_block_tasks_lds<A>(a, p, ang, cnt, stage);
  const int lane = threadIdx.x & 63;
  int32_t* out = a.tasks_out + (size_t)perm_start * (A * a.n_sensors);
  for (int i = lane; i < total; i += 64) stc(out + i, stage[i]);
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// ============================================================ k_dyn, A == 1
// RacingEnv.step / reset (environment/racing_env.py:86-167), plus
// RecordEpisodeStatistics and SyncVectorEnv autoreset.  LPE lanes per
// env: every lane of an env evaluates the (cheap) dynamics, the five argmins
// (centre + 4 corners) are split over the lanes, the progress index and the
// crash flag are combined with lane shuffles, and lane 0 of the env does the
// rest.  4x the waves of one-env-per-lane: the argmin's scalar-load chains are
// latency-bound, and more waves per SIMD hide them.
__device__ __forceinline__ double pick5(const double v[5], int P) {
  return P == 0 ? v[0] : P == 1 ? v[1] : P == 2 ? v[2] : P == 3 ? v[3] : v[4];
}

// Profiling build only (-DRX_DYN_STAMPS, tools/dyn_stamps.py): per-wave
// s_memtime stamps at phase boundaries of k_dyn1, each after a full
// s_waitcnt so a phase includes the memory latency it waited for, written to
// io.counters[16 + 8 * wave + j].
#ifdef RX_DYN_STAMPS
#define RX_STAMP(j)                                            \
  do {                                                         \
    __builtin_amdgcn_s_waitcnt(0);                             \
    stamp[j] = __builtin_amdgcn_s_memtime();                   \
  } while (0)
#else
#define RX_STAMP(j) \
  do {              \
  } while (0)
#endif

// Which part of RacingEnv.step a dyn1_env instance runs.  FULL: everything
// (k_dyn1).  The split step (k_kin1 then k_step2; rx_api.cpp)
// lets the raycast run concurrently with the expensive half: KIN = resets,
// actions, Car.update's kinematics, the non-ray obs columns and the ray-task
// sort -- all the raycast needs -- and REWARD = the closest-waypoint argmins,
// wall collision, progress, reward, done and episode statistics of the envs
// KIN stepped (KIN marks the envs it reset with RX_EF_RESET_NOW; REWARD skips
// and clears them).  The arithmetic is the same code either way.
#define RX_PART_FULL 0
#define RX_PART_KIN 1
#define RX_PART_REWARD 2
#define RX_EF_RESET_NOW 2u

// The persistent rollout stages its env's slot (waypoints, normals, boundary
// segments) in LDS once and hands the kernels' device functions these
// pointers instead of the table in HBM (nullptr: the table).
struct rx_slot_lds {
  const double2* wp;
  const double2* nrm;
  const double4* seg;
};

template <int LPE, int PART, bool LV = false>
__device__ __forceinline__ void dyn1_env(const rx_kargs& a, int wave, double* ang_out, int& e_out, double ep_out[3],
                                         int sub_block = 0, const rx_slot_lds* sl = nullptr) {
  static_assert(!LV || LPE == 1, "lane-varying slots: one lane per env");
  constexpr bool FULL = PART == RX_PART_FULL, KIN = PART == RX_PART_KIN, REW = PART == RX_PART_REWARD;
#ifdef RX_DYN_STAMPS
  unsigned long long stamp[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  stamp[0] = __builtin_amdgcn_s_memtime();
#endif
  constexpr int NPL = (5 + LPE - 1) / LPE;  // argmin points per lane
  if (wave >= a.n_dyn_waves) return;
  const rx_wave we = a.dyn_waves[wave];
  // env slot in the dynamics wave's 64-env group (a wave at LPE lanes per env
  // covers 64 / LPE of them; sub_block picks which when the group's dynamics
  // wave was built for one lane per env: the REWARD half at LPE = 2)
  const int lane = (threadIdx.x & 63) / LPE + sub_block * (64 / LPE);
  const int sub = threadIdx.x & (LPE - 1);
  // LV: the lane's own slot (the wave's 64 positions may hold 64 slots)
  const int k = LV ? (lane < we.count ? a.pos_slot[we.perm_start + lane] : 0) : uniform(we.track);
  const rx_slot_hdr* __restrict__ hd = a.tr.hdr + k;  // LV: every per-slot scalar from one line
  const int wp0 = LV ? hd->wp0 : uniform(a.tr.wp_off[k]);
  const int W = LV ? hd->W : uniform(a.tr.wp_off[k + 1]) - wp0;
  const double2* __restrict__ wp = sl ? sl->wp : reinterpret_cast<const double2*>(a.tr.wp) + wp0;
  const double2* __restrict__ nrm = sl ? sl->nrm : reinterpret_cast<const double2*>(a.tr.nrm) + wp0;
  const double* __restrict__ meta = LV ? hd->meta : a.tr.meta + 8 * k;
  const double width = meta[3];
  if (lane >= we.count) return;
  // p = the env's position in the wave order: the engine's working state is
  // stored in that order (coalesced); e = the env id, the row of every io buffer
  int p = we.perm_start + lane;
  int e = REW ? -1 : RX_IO_ROW(a, p);  // REWARD: loaded after the argmins

  const rx_state& S = a.st;
  uint8_t ef = ldc(S.env_flags + p);
  uint8_t fl = ldc(S.flags + p);
  // every per-env load up front, so their latencies overlap (not one round
  // trip per use) -- except in the REWARD half, which runs under the raycast
  // at the raycast's 64-VGPR budget: its values not needed by the argmins
  // (velocity, last progress, episode counters, steps) load after them, so
  // they are not live across the argmin loops (fewer spills)
  Car c{ldc(S.x + p), ldc(S.y + p), REW ? 0.0 : ldc(S.angle + p), REW ? 0.0 : ldc(S.vx + p), REW ? 0.0 : ldc(S.vy + p), ldc(S.progress + p),
        (fl & RX_F_CRASHED) != 0};
  double last_steering = REW ? 0.0 : ldc(S.last_steering + p);
  const bool step_mode = a.mode == RX_MODE_STEP;  // wave-uniform
  const float2 act =
      (step_mode && !REW) ? reinterpret_cast<const float2*>(a.io.actions)[e] : make_float2(0.0f, 0.0f);
  double last_progress = (KIN || REW) ? 0.0 : ldc(S.last_progress + p);
  double ep_ret0 = (KIN || REW) ? 0.0 : ldc(S.ep_return + p);
  int ep_len0 = (KIN || REW) ? 0 : ldc(S.ep_length + p);
  double speed_w = (KIN || REW) ? 0.0 : (S.speed_weight ? S.speed_weight[e] : a.speed_weight);  // caller's, env order
  int steps = REW ? 0 : ldc(S.steps + p);  // REWARD: already advanced by KIN
  double cs[2] = {0.0, 0.0};
  if (REW) {
    cs[0] = ldc(a.cs_scratch + 2 * p);
    cs[1] = ldc(a.cs_scratch + 2 * p + 1);
  }
  RX_STAMP(1);
  bool do_reset;
  if (REW)
    do_reset = (ef & RX_EF_RESET_NOW) != 0;
  else if (a.mode == RX_MODE_RESET)
    do_reset = (a.reset_mask == nullptr) || a.reset_mask[e];
  else
    do_reset = (a.autoreset == RX_AUTORESET_NEXT_STEP) && (ef & RX_EF_PENDING_RESET);
  const bool stepping = step_mode && !do_reset;

  double reward = 0.0, pd = 0.0;
  bool term = false, trunc = false;
  // ---------------------------------------------------------------- step
  // Lanes that step run the argmin loop together; reset lanes are masked.
  bool moving = stepping && !c.crashed;
  double cx[4], cy[4];
  if (!REW && stepping) {
    const double steering = (double)clipf(act.x, -1.0f, 1.0f);  // racing_env.py:106
    const double throttle = (double)clipf(act.y, 0.0f, 1.0f);
    last_steering = steering;
    if (moving) car_kinematics(c, steering, throttle, cs, cx, cy);
  }
  if (REW && moving) corners(c.x, c.y, cs[0], cs[1], cx, cy);  // car.py:26-43 of the stepped state
  RX_STAMP(2);
  if (!KIN && moving) {
    const double px[5] = {c.x, cx[0], cx[1], cx[2], cx[3]};
    const double py[5] = {c.y, cy[0], cy[1], cy[2], cy[3]};
    // this lane's points: P = sub + LPE*j (point 0 = centre, 1..4 = corners);
    // slots past point 4 repeat the lane's first point and are ignored
    double qx[NPL], qy[NPL];
    int idx[NPL];
#pragma unroll
    for (int j = 0; j < NPL; ++j) {
      const int P = sub + LPE * j < 5 ? sub + LPE * j : sub;
      qx[j] = pick5(px, P);
      qy[j] = pick5(py, P);
    }
    if constexpr (LPE == 64) {
      idx[0] = argmin_wave(wp, W, px, py, sub < 5 ? sub : -1);
    } else if (a.cull_chunk > 0) {
      const int prev[1] = {prev_waypoint(c.progress, W)};
      const double ccx[1] = {c.x}, ccy[1] = {c.y};
      argmin_culled<NPL, 1, LV>(wp, a.tr.wchunk_box + 4 * (size_t)(LV ? hd->wchunk_off : uniform(a.tr.wchunk_off[k])),
                            a.tr.wsuper_box + 4 * (size_t)(LV ? hd->wsuper_off : uniform(a.tr.wsuper_off[k])), W, qx,
                            qy, prev, ccx, ccy,
                            a.argmin_window, idx, a.io.counters
#ifdef RX_DYN_STAMPS
                            , stamp + 3
#endif
      );
    } else {
      argmin_pts<NPL>(wp, W, qx, qy, idx);
    }
    RX_STAMP(5);
    int out = 0;  // Track.check_collision: any corner outside (track.py:163-171)
#pragma unroll
    for (int j = 0; j < NPL; ++j) {
      const int P = sub + LPE * j;
      if (P >= 1 && P < 5) out |= corner_out(wp, nrm, idx[j], qx[j], qy[j], width) ? 1 : 0;
    }
#pragma unroll
    for (int o = 1; o < LPE; o <<= 1) out |= __shfl_xor(out, o, 64);
    const int i0 = __shfl(idx[0], (int)(threadIdx.x & 63) - sub, 64);  // centre argmin lives on sub 0
    c.progress = (double)i0 / (double)W;  // track.py:159-161
    c.crashed = out != 0;
  }
  RX_STAMP(6);
  if (sub != 0) return;  // one lane per env from here on
  // REWARD: p passes through an empty asm, so the addresses of the late loads and
  // of the stores below are recomputed from it (2 VALU each) instead of being kept
  // live as 64-bit pointers across the argmins (they were spilled to scratch)
  if constexpr (REW) __asm__ volatile("" : "+v"(p));
  if (REW) {  // the REWARD half's late loads (see above)
    e = RX_IO_ROW(a, p);
    c.vx = ldc(S.vx + p);
    c.vy = ldc(S.vy + p);
    last_progress = ldc(S.last_progress + p);
    ep_ret0 = ldc(S.ep_return + p);
    ep_len0 = ldc(S.ep_length + p);
    speed_w = S.speed_weight ? S.speed_weight[e] : a.speed_weight;
    steps = ldc(S.steps + p);
  }
  bool ended = false;
  double epr = 0.0, epl_d = 0.0;
  if (!REW && stepping) steps += 1;
  if (!KIN && stepping) {
    const double pg = c.progress;
    pd = pg - last_progress;  // racing_env.py:112-116
    if (last_progress > 0.9 && pg < 0.1)
      pd = (1.0 - last_progress) + pg;
    else if (last_progress < 0.1 && pg > 0.9)
      pd = -((1.0 - pg) + last_progress);
    double r = pd * 200;
    if (!(fl & RX_F_CP25) && 0.25 <= pg && pg < 0.35) { fl |= RX_F_CP25; r += 20; }
    if ((fl & RX_F_CP25) && !(fl & RX_F_CP50) && 0.50 <= pg && pg < 0.60) { fl |= RX_F_CP50; r += 20; }
    if ((fl & RX_F_CP50) && !(fl & RX_F_CP75) && 0.75 <= pg && pg < 0.85) { fl |= RX_F_CP75; r += 20; }
    if (!c.crashed && pd > 0) {  // :137-140
      double ratio = rx_clip(speed_of(c.vx, c.vy) / RX_MAX_SPEED, 0.0, 1.0);
      r += ratio * speed_w;
    }
    if (c.crashed) r -= 60;
    const uint8_t all_cp = RX_F_CP25 | RX_F_CP50 | RX_F_CP75;
    if ((fl & all_cp) == all_cp && last_progress > 0.9 && pg < 0.1 && pd > 0) {  // :145-150
      fl |= RX_F_FINISHED;
      r += 100;
      double tb = 200 - ((double)steps / 10);
      if (tb > 0) r += tb;
    }
    fl = (uint8_t)((fl & ~RX_F_CRASHED) | (c.crashed ? RX_F_CRASHED : 0));
    reward = r;
    term = c.crashed || (fl & RX_F_FINISHED);
    trunc = steps >= a.max_steps;
    // RecordEpisodeStatistics.step
    epr = ep_ret0 + r;
    const int epl = ep_len0 + 1;
    epl_d = (double)epl;
    stc(S.ep_return + p, epr);
    stc(S.ep_length + p, epl);
    ended = term || trunc;
    if (a.io.ep_done) a.io.ep_done[e] = ended;
    if (ended && a.autoreset == RX_AUTORESET_NEXT_STEP) ef |= RX_EF_PENDING_RESET;
    if (FULL && ended && a.autoreset == RX_AUTORESET_SAME_STEP) do_reset = true;  // reset AFTER the outputs
  } else if (!REW && !stepping && a.io.ep_done) {
    a.io.ep_done[e] = 0;
  }
  // info of the stepped state (racing_env.py:77-84,156-159)
  if ((FULL || (REW && stepping)) && a.io.info) {
    double* inf = a.io.info + (size_t)e * RX_INFO_W;
    inf[RX_INFO_SPEED] = speed_of(c.vx, c.vy);
    inf[RX_INFO_PROGRESS] = (fl & RX_F_FINISHED) ? 1.0 : c.progress;
    inf[RX_INFO_PROGRESS_DELTA] = pd;
    inf[RX_INFO_PLACEMENT] = 0.0;
  }
  // ---------------------------------------------------------------- reset
  if (!REW && do_reset) {  // RacingEnv.reset + Car.reset, racing_env.py:86-102, car.py:17-24
    c.x = meta[0];
    c.y = meta[1];
    c.angle = meta[2];
    c.vx = 0.0;
    c.vy = 0.0;
    c.progress = 0.0;
    c.crashed = false;
    fl = 0;
    steps = 0;
    last_steering = 0.0;
    ef &= (uint8_t)~RX_EF_PENDING_RESET;
    if (KIN) ef |= RX_EF_RESET_NOW;
    stc(S.ep_return + p, 0.0);
    stc(S.ep_length + p, 0);
    if (a.io.info && (a.mode == RX_MODE_RESET || a.autoreset == RX_AUTORESET_NEXT_STEP)) {
      double* inf = a.io.info + (size_t)e * RX_INFO_W;
      inf[RX_INFO_SPEED] = 0.0;
      inf[RX_INFO_PROGRESS] = 0.0;
      inf[RX_INFO_PROGRESS_DELTA] = 0.0;
      if (KIN) inf[RX_INFO_PLACEMENT] = 0.0;
    }
  }
  if (REW && do_reset) ef &= (uint8_t)~RX_EF_RESET_NOW;
  if (FULL && (stepping || do_reset)) {
    stc(S.x + p, c.x);
    stc(S.y + p, c.y);
    stc(S.angle + p, c.angle);
    stc(S.vx + p, c.vx);
    stc(S.vy + p, c.vy);
    stc(S.progress + p, c.progress);
    stc(S.last_progress + p, c.progress);  // racing_env.py:165 (0.0 after reset)
    stc(S.last_steering + p, last_steering);
    stc(S.steps + p, steps);
    stc(S.flags + p, fl);
    stc(S.env_flags + p, ef);
  }
  if (KIN && (stepping || do_reset)) {
    stc(S.x + p, c.x);
    stc(S.y + p, c.y);
    stc(S.angle + p, c.angle);
    stc(S.vx + p, c.vx);
    stc(S.vy + p, c.vy);
    stc(S.last_steering + p, last_steering);
    stc(S.steps + p, steps);
    if (moving) {
      reinterpret_cast<double2*>(a.cs_scratch)[p] = make_double2(cs[0], cs[1]);
    }
    if (do_reset) {
      stc(S.progress + p, 0.0);
      stc(S.last_progress + p, 0.0);
      stc(S.flags + p, fl);
      stc(S.env_flags + p, ef);
    }
  }
  if (REW && (stepping || do_reset)) {
    if (stepping) {
      stc(S.progress + p, c.progress);
      stc(S.last_progress + p, c.progress);  // racing_env.py:165
      stc(S.flags + p, fl);
    }
    stc(S.env_flags + p, ef);
  }
  RX_STAMP(7);
  // ---------------------------------------------------------------- outputs
  // reset-by-NEXT_STEP / explicit reset: reward 0, term = trunc = False
  if (FULL || (REW && stepping) || (KIN && do_reset)) {
    const bool wrote_step = stepping;
    const float rf = wrote_step ? (float)reward : 0.0f;
    if (a.io.reward) a.io.reward[e] = rf;
    if (a.io.reward64) a.io.reward64[e] = wrote_step ? reward : 0.0;
    const bool t_out = wrote_step && term, u_out = wrote_step && trunc;
    if (a.io.terminated) a.io.terminated[e] = t_out;
    if (a.io.truncated) a.io.truncated[e] = u_out;
    if (a.io.done_f32) a.io.done_f32[e] = (t_out || u_out) ? 1.0f : 0.0f;
  }
  // non-ray observation columns of the CURRENT state (racing_env.py:58-75)
  if (!REW) {
    double s, co;
    if (moving && !do_reset) {  // car_kinematics already evaluated sin/cos of this angle
      co = cs[0];
      s = cs[1];
    } else {
      rx_sincos(c.angle, &s, &co);
    }
    double vf = c.vx * co + c.vy * s;
    double vl = (-c.vx) * s + c.vy * co;
    float* o = a.io.obs + (size_t)e * a.D + a.n_sensors;
    o[0] = (float)rx_clip(vf / RX_MAX_SPEED, -1.0, 1.0);
    o[1] = (float)rx_clip(vl / RX_MAX_SPEED, -1.0, 1.0);
    o[2] = (float)rx_clip(0.0 / 3.0, -1.0, 1.0);  // angular_velocity is always 0
    o[3] = (float)last_steering;
  }
  if (!KIN) write_sort_key(a, p, k, c.progress, W);
  if (!REW) {
    ang_out[0] = c.angle;
    e_out = p;  // the ray tasks name the position (k_rays reads the state there, writes obs row perm[p])
  }
  if (ended) {  // RecordEpisodeStatistics: summed per wave by the caller
    ep_out[0] = epr;
    ep_out[1] = epl_d;
    ep_out[2] = 1.0;
  }
#ifdef RX_DYN_STAMPS
  RX_STAMP(8);
#ifdef RX_DYN_STAMPS_NO_REWARD  // the split step's KIN phases (tools/dyn_stamps.py kin): REWARD keeps out
  if constexpr (!REW)
#endif
    if (a.io.counters && (threadIdx.x & 63) == (__builtin_amdgcn_readfirstlane(threadIdx.x) & 63))
      for (int j = 0; j < 9; ++j) a.io.counters[16 + 12 * wave + j] = stamp[j];
#endif
}

// Episode statistics of the envs that ended this step, summed over the wave
// (all 64 lanes present) and added with ONE atomic per counter per wave into
// one of RX_EP_SHARDS accumulator rows: per-env device-scope atomics on the
// same three addresses serialised the launch, and even one per wave on three
// shared addresses cost ~1.5 % of the step (RX_NO_EPSTATS A/B).
__device__ __forceinline__ void add_episode_stats(const rx_kargs& a, const double v[3]) {
  if (!a.io.ep_stats || !__any(v[2] != 0.0)) return;
  double s0 = v[0], s1 = v[1], s2 = v[2];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s0 += __shfl_xor(s0, o, 64);
    s1 += __shfl_xor(s1, o, 64);
    s2 += __shfl_xor(s2, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {  // RX_EP_SHARDS rows of 4 (3 used): the reader sums them
    double* st = a.io.ep_stats + 4 * ((blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) & (RX_EP_SHARDS - 1));
    atomicAdd(&st[0], s0);
    atomicAdd(&st[1], s1);
    atomicAdd(&st[2], s2);
  }
}

// rx_profile: each wave stores the 100 MHz device wall clock (s_memrealtime,
// one chip-wide counter) when it starts and ends, at its wave index (plain
// stores: no contention).  The host takes min(start) .. max(end) as the
// launch's duration -- the kernel's execution span, as rocprofv3 measures it,
// without the dispatch / cache-flush time that stream events around a launch
// include.
// Both stamps are stored at the END of the wave: a global store at the start
// would precede every table load in program order and cost the compiler its
// proof that those loads see unclobbered memory (vector instead of scalar loads).
__device__ __forceinline__ unsigned long long prof_start(const rx_kargs& a) {
  return a.prof_ts ? wall_clock64() : 0ull;
}
__device__ __forceinline__ void prof_end(const rx_kargs& a, int wave, unsigned long long t0) {
  if (!a.prof_ts || (threadIdx.x & 63) != 0 || wave >= a.prof_stride) return;
  a.prof_ts[wave] = t0;
  a.prof_ts[a.prof_stride + wave] = wall_clock64();
}

// k_dyn1 (PART = FULL) and k_kin1 (PART = KIN): 4 waves per workgroup.
template <int LPE, int PART, bool LV = false>
__global__ __launch_bounds__(256) void k_dyn1(rx_kargs a) {
  const int wave = uniform(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  if (wave >= a.n_dyn_waves) return;
  // ray-task sort: per wave 64 sector counters and a staging row of its <= 64 x 16 task ids
  // (k_kin1 runs one wave per workgroup, k_dyn1 four)
  // dynamic LDS, task_sort_lds_bytes: sized only when the launch sorts (the
  // static rows cost occupancy on the resets / same-step launches, which never sort)
  constexpr int NW = PART == RX_PART_KIN ? 1 : 4;
  extern __shared__ int32_t task_lds[];
  const int wl = NW == 1 ? 0 : (int)(threadIdx.x >> 6);
  int32_t* cnt = task_lds + wl * (kTaskSectors + 64 * 16);
  int32_t* stage = cnt + kTaskSectors;
  const bool sorting = a.tasks_out != nullptr;
  if (sorting) cnt[threadIdx.x & 63] = 0;
  const unsigned long long prof_t0 = prof_start(a);
  double ang[1], ep[3] = {0.0, 0.0, 0.0};
  int e = -1;  // set on the lane that finishes an env (sub 0)
  dyn1_env<LPE, PART, LV>(a, wave, ang, e, ep);
  if (PART == RX_PART_FULL) add_episode_stats(a, ep);
  if (sorting) sort_block_tasks<1>(a, uniform(a.dyn_waves[wave].perm_start), e, ang, cnt, stage);
  prof_end(a, wave, prof_t0);
#ifdef RX_DYN_STAMPS
  __builtin_amdgcn_s_waitcnt(0);
  const unsigned long long t7 = __builtin_amdgcn_s_memtime();
  if (a.io.counters && (threadIdx.x & 63) == 0) a.io.counters[16 + 12 * wave + 9] = t7;
#endif
}

// ============================================================ k_dyn, A == 2
// MultiRacingEnv.step / reset (environment/multi_racing_env.py:118-269), one
// env (both cars) per lane.
__device__ double multi_reward(Car& c, uint8_t& fl, int32_t& finished_step, double last_progress, int steps) {
  // MultiRacingEnv.calc_reward -- multi_racing_env.py:155-196
  double p = c.progress;
  double pd = p - last_progress;
  if (last_progress > 0.9 && p < 0.1)
    pd = (1.0 - last_progress) + p;
  else if (last_progress < 0.1 && p > 0.9)
    pd = -((1.0 - p) + last_progress);
  double r = 0.0;
  r += pd * 200;
  if (!c.crashed && pd > 0) {
    double ratio = rx_clip(speed_of(c.vx, c.vy) / RX_MAX_SPEED, 0.0, 1.0);
    r += ratio * 18;
  }
  if (!(fl & RX_F_CP25) && 0.25 <= p && p < 0.35) { fl |= RX_F_CP25; r += 25; }
  if ((fl & RX_F_CP25) && !(fl & RX_F_CP50) && 0.50 <= p && p < 0.60) { fl |= RX_F_CP50; r += 25; }
  if ((fl & RX_F_CP50) && !(fl & RX_F_CP75) && 0.75 <= p && p < 0.85) { fl |= RX_F_CP75; r += 25; }
  const uint8_t all_cp = RX_F_CP25 | RX_F_CP50 | RX_F_CP75;
  if ((fl & all_cp) == all_cp && last_progress > 0.9 && p < 0.1 && pd > 0) {
    fl |= RX_F_FINISHED;
    finished_step = steps;
    double tb = 300 - ((double)steps / 15);
    r += 100 + (tb > 0 ? tb : 0.0);
  }
  if (c.crashed && !(fl & RX_F_HAS_CRASHED)) {
    r -= 160;
    fl |= RX_F_HAS_CRASHED;
  }
  return r;
}

// MultiCar.rectangles_intersect -- environment/multi_car.py:16-43
__device__ __forceinline__ bool rect_intersect(const double ax[4], const double ay[4], const double bx[4],
                                               const double by[4]) {
  double axx[4], axy[4];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    axx[i] = -(ay[i + 1] - ay[i]);
    axy[i] = ax[i + 1] - ax[i];
    axx[2 + i] = -(by[i + 1] - by[i]);
    axy[2 + i] = bx[i + 1] - bx[i];
  }
  bool sep = false;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    double amax = -__builtin_inf(), amin = __builtin_inf(), bmax = -__builtin_inf(), bmin = __builtin_inf();
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      double pa = rx_dot2_np(ax[c], ay[c], axx[q], axy[q]);
      double pb = rx_dot2_np(bx[c], by[c], axx[q], axy[q]);
      amax = pa > amax ? pa : amax;
      amin = pa < amin ? pa : amin;
      bmax = pb > bmax ? pb : bmax;
      bmin = pb < bmin ? pb : bmin;
    }
    sep = sep || (amax < bmin || bmax < amin);
  }
  return !sep;
}

// PART as for dyn1_env: FULL = the whole step (k_dyn2); the split two-car step
// runs KIN (resets, kinematics, car-car contact, non-ray obs, ray-task sort:
// everything the raycast reads) in k_kin2, then REWARD (argmins, wall
// collision, rewards, placement, done, episode statistics) beside the raycast
// in k_step2<2>.  Contact only needs the kinematic poses, so it moves to KIN;
// KIN passes "the cars touched" to REWARD in env_flags (RX_EF_TOUCH) and the
// stepped cos / sin of each moving car in cs_scratch[2e + q].
#define RX_EF_TOUCH 4u
// RLPE (REWARD only): lanes per env.  2 = a lane pair per env, lane `sub` runs
// car `sub`'s closest-waypoint pass (the REWARD chain's two sequential passes
// become one), the pair exchanges progress / crash flag, and lane 0 of the pair
// does the rest; sub_block picks which 32 of the dynamics wave's 64 envs.
template <int PART, int RLPE = 1>
__device__ __forceinline__ void dyn2_env(const rx_kargs& a, int wave, double* ang_out, int& e_out, double ep_out[3],
                                         int sub_block = 0) {
  constexpr bool FULL = PART == RX_PART_FULL, KIN = PART == RX_PART_KIN, REW = PART == RX_PART_REWARD;
  static_assert(RLPE == 1 || (RLPE == 2 && REW), "two lanes per env: the REWARD part only");
  if (wave >= a.n_dyn_waves) return;
  const rx_wave we = a.dyn_waves[wave];
  const int lane = (int)(threadIdx.x & 63) / RLPE + sub_block * (64 / RLPE);
  const int sub = (int)threadIdx.x & (RLPE - 1);
  const int k = uniform(we.track);
  const int wp0 = uniform(a.tr.wp_off[k]);
  const int W = uniform(a.tr.wp_off[k + 1]) - wp0;
  const double2* __restrict__ wp = reinterpret_cast<const double2*>(a.tr.wp) + wp0;
  const double2* __restrict__ nrm = reinterpret_cast<const double2*>(a.tr.nrm) + wp0;
  const double* __restrict__ meta = a.tr.meta + 8 * k;
  const double width = uniform_d(meta[3]);
  const double maxd = uniform_d(meta[4]);
  if (lane >= we.count) return;
  const int p = we.perm_start + lane;  // working-state position (see dyn1_env)
  const int e = a.perm[p];             // env id: io rows, the start-slot draw
  const rx_state& S = a.st;

  uint8_t ef = S.env_flags[p];
  Car c[2];
  uint8_t fl[2];
  double last_steering[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int i = 2 * p + q;
    fl[q] = S.flags[i];
    // REWARD needs no angle, and loads the velocity only after the argmins
    // (fewer live registers through them: k_step2<2> runs at 80 VGPRs)
    c[q] = REW ? Car{S.x[i], S.y[i], 0.0, 0.0, 0.0, S.progress[i], (fl[q] & RX_F_CRASHED) != 0}
               : Car{S.x[i], S.y[i], S.angle[i], S.vx[i], S.vy[i], S.progress[i], (fl[q] & RX_F_CRASHED) != 0};
    last_steering[q] = REW ? 0.0 : S.last_steering[i];
  }
  bool do_reset;
  if (REW)
    do_reset = (ef & RX_EF_RESET_NOW) != 0;
  else if (a.mode == RX_MODE_RESET)
    do_reset = (a.reset_mask == nullptr) || a.reset_mask[e];
  else
    do_reset = (a.autoreset == RX_AUTORESET_NEXT_STEP) && (ef & RX_EF_PENDING_RESET);
  const bool stepping = (a.mode == RX_MODE_STEP) && !do_reset;
  int steps = S.steps[p];  // REWARD: already advanced by KIN
  double rw[2] = {0.0, 0.0};
  int place[2] = {0, 0};
  bool term = false, trunc = false;
  // sin/cos of each car's CURRENT angle, evaluated at most once per step
  // (kinematics, car-car contact and the observation all need them)
  double sn[2], cn[2];
  bool have_sc[2] = {false, false};
  if (stepping) {
    float av[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (!REW) {
      const float4 act = reinterpret_cast<const float4*>(a.io.actions)[e];
      av[0] = act.x;
      av[1] = act.y;
      av[2] = act.z;
      av[3] = act.w;
    }
    double cx[2][4], cy[2][4], cs[2][2];
    bool mv[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {  // multi_racing_env.py:215-220
      mv[q] = !c[q].crashed;
      if (REW) continue;  // REWARD: corners per car in its argmin pass below
      {
        last_steering[q] = (double)clipf(av[2 * q], -1.0f, 1.0f);
        const float thr = clipf((av[2 * q + 1] + 1.0f) / 2.0f, 0.0f, 1.0f);
        if (mv[q]) {
          car_kinematics(c[q], last_steering[q], (double)thr, cs[q], cx[q], cy[q]);
          cn[q] = cs[q][0];
          sn[q] = cs[q][1];
          have_sc[q] = true;
          if (KIN) reinterpret_cast<double2*>(a.cs_scratch)[2 * p + q] = make_double2(cs[q][0], cs[q][1]);
        }
      }
    }
    if (REW && RLPE == 2) {
      // lane `sub` = car `sub`: ONE pass per wave over both cars' points (the
      // argmin is per lane, culling over the wave's union), then the pair swaps
      const bool mvq = sub ? mv[1] : mv[0];
      Car cq = sub ? c[1] : c[0];
      if (__any(mvq)) {
        const double2 sc = reinterpret_cast<const double2*>(a.cs_scratch)[2 * p + sub];
        double px[5], py[5];
        px[0] = cq.x;
        py[0] = cq.y;
        corners(cq.x, cq.y, sc.x, sc.y, px + 1, py + 1);
        int idx[5];
        if (a.cull_chunk > 0) {
          const int prev[1] = {prev_waypoint(cq.progress, W)};
          const double ccx[1] = {cq.x}, ccy[1] = {cq.y};
          argmin_culled<5, 1>(wp, a.tr.wchunk_box + 4 * (size_t)uniform(a.tr.wchunk_off[k]),
                              a.tr.wsuper_box + 4 * (size_t)uniform(a.tr.wsuper_off[k]), W, px, py, prev, ccx, ccy,
                              a.argmin_window, idx, a.io.counters, nullptr, mvq);
        } else {
          argmin_pts<5>(wp, W, px, py, idx);
        }
        if (mvq) {
          cq.progress = (double)idx[0] / (double)W;
          bool out = false;
#pragma unroll
          for (int j = 0; j < 4; ++j) out = out || corner_out(wp, nrm, idx[1 + j], px[1 + j], py[1 + j], width);
          cq.crashed = out;
        }
      }
      const double po = __shfl_xor(cq.progress, 1, 64);
      const int co = __shfl_xor(cq.crashed ? 1 : 0, 1, 64);
      c[0].progress = sub ? po : cq.progress;
      c[0].crashed = sub ? (co != 0) : cq.crashed;
      c[1].progress = sub ? cq.progress : po;
      c[1].crashed = sub ? cq.crashed : (co != 0);
    } else if (REW && (mv[0] || mv[1])) {
      // one pass per car (as FULL's culled passes below): corners of the stepped
      // pose (car.py:26-43, KIN's cos / sin), the 5 closest waypoints, wall
      // collision; only this car's corners are live during its pass
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        if (!__any(mv[q])) continue;
        const double2 sc = reinterpret_cast<const double2*>(a.cs_scratch)[2 * p + q];
        double px[5], py[5];
        px[0] = c[q].x;
        py[0] = c[q].y;
        corners(c[q].x, c[q].y, sc.x, sc.y, px + 1, py + 1);
        int idx[5];
        if (a.cull_chunk > 0) {
          const int prev[1] = {prev_waypoint(c[q].progress, W)};
          const double ccx[1] = {c[q].x}, ccy[1] = {c[q].y};
          argmin_culled<5, 1>(wp, a.tr.wchunk_box + 4 * (size_t)uniform(a.tr.wchunk_off[k]),
                              a.tr.wsuper_box + 4 * (size_t)uniform(a.tr.wsuper_off[k]), W, px, py, prev, ccx, ccy,
                              a.argmin_window, idx, a.io.counters, nullptr, mv[q]);
        } else {
          argmin_pts<5>(wp, W, px, py, idx);
        }
        if (mv[q]) {
          c[q].progress = (double)idx[0] / (double)W;
          bool out = false;
#pragma unroll
          for (int j = 0; j < 4; ++j) out = out || corner_out(wp, nrm, idx[1 + j], px[1 + j], py[1 + j], width);
          c[q].crashed = out;
        }
      }
    }
    if (REW && RLPE == 2 && sub != 0) return;  // one lane per env from here on
    if (REW) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        c[q].vx = S.vx[2 * p + q];
        c[q].vy = S.vy[2 * p + q];
      }
    }
    if (FULL && (mv[0] || mv[1])) {
      double px[10], py[10];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        px[5 * q] = c[q].x;
        py[5 * q] = c[q].y;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          px[5 * q + 1 + j] = cx[q][j];
          py[5 * q + 1 + j] = cy[q][j];
        }
      }
      int idx[10];
      if (a.cull_chunk > 0) {
        // one culled pass per car: the envs of a wave are sorted by car 0's
        // position, so car 1s are scattered once the cars separate -- a joint
        // pass scanned the union of both (nearly every leaf), and every scanned
        // leaf evaluated all 10 points.  A car that does not move (crashed) is
        // left out of its pass (its result is not used).
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          if (!__any(mv[q])) continue;
          const int prev[1] = {prev_waypoint(c[q].progress, W)};
          const double ccx[1] = {c[q].x}, ccy[1] = {c[q].y};
          argmin_culled<5, 1>(wp, a.tr.wchunk_box + 4 * (size_t)uniform(a.tr.wchunk_off[k]),
                              a.tr.wsuper_box + 4 * (size_t)uniform(a.tr.wsuper_off[k]), W, px + 5 * q, py + 5 * q,
                              prev, ccx, ccy, a.argmin_window, idx + 5 * q, a.io.counters, nullptr, mv[q]);
        }
      } else {
        argmin_pts<10>(wp, W, px, py, idx);
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        if (!mv[q]) continue;
        c[q].progress = (double)idx[5 * q] / (double)W;
        bool out = false;
#pragma unroll
        for (int j = 0; j < 4; ++j) out = out || corner_out(wp, nrm, idx[5 * q + 1 + j], cx[q][j], cy[q][j], width);
        c[q].crashed = out;
      }
    }
    // car-car contact, multi_racing_env.py:222-231 (corners of the current state)
    if (!REW) {
      double ax[4], ay[4], bx[4], by[4];
#pragma unroll
      for (int q = 0; q < 2; ++q)
        if (!have_sc[q]) {
          rx_sincos(c[q].angle, &sn[q], &cn[q]);
          have_sc[q] = true;
        }
      corners(c[0].x, c[0].y, cn[0], sn[0], ax, ay);
      corners(c[1].x, c[1].y, cn[1], sn[1], bx, by);
      ef &= (uint8_t)~RX_EF_TOUCH;
      if (rect_intersect(ax, ay, bx, by)) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          c[q].vx *= 0.92;
          c[q].vy *= 0.92;
          rw[q] = -5.0;
        }
        if (KIN) ef |= RX_EF_TOUCH;
      }
    } else if (ef & RX_EF_TOUCH) {  // touching_penalties from KIN's contact test
      rw[0] = rw[1] = -5.0;
      ef &= (uint8_t)~RX_EF_TOUCH;
    }
    if (!REW) steps += 1;
  }
  if (REW && RLPE == 2 && sub != 0) return;  // (not stepping: the pass above did not run)
  if (!KIN && stepping) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int i = 2 * p + q;
      fl[q] = (uint8_t)((fl[q] & ~RX_F_CRASHED) | (c[q].crashed ? RX_F_CRASHED : 0));
      int32_t fs = S.finished_step[i];
      double r = multi_reward(c[q], fl[q], fs, S.last_progress[i], steps);
      S.finished_step[i] = fs;
      rw[q] = r + rw[q];  // calc_reward(i) + touching_penalties[i]
    }
    const bool any_fin = (fl[0] & RX_F_FINISHED) || (fl[1] & RX_F_FINISHED);
    const bool all_crash = c[0].crashed && c[1].crashed;
    term = any_fin || all_crash;
    trunc = steps >= a.max_steps;
    if (term || trunc) {  // place(), multi_racing_env.py:198-211,252-259
      double sc[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int fs = S.finished_step[2 * p + q];
        double v = (double)((fl[q] & RX_F_FINISHED) ? 10000 : 0) + c[q].progress * 100;
        v = v + (double)(c[q].crashed ? 0 : 10);
        v = v + 1.0 / (double)(fs > 0 ? fs : 10000);
        sc[q] = v;
      }
      const int first = (sc[1] >= sc[0]) ? 1 : 0;  // sort(reverse=True): ties -> larger idx first
      place[first] = 1;
      place[1 - first] = 2;
      rw[first] += 250;
    }
    double epr = S.ep_return[p] + rw[0];
    int epl = S.ep_length[p] + 1;
    S.ep_return[p] = epr;
    S.ep_length[p] = epl;
    const bool ended = term || trunc;
    if (a.io.ep_done) a.io.ep_done[e] = ended;
    if (ended) {  // RecordEpisodeStatistics: summed per wave by the caller
      ep_out[0] = epr;
      ep_out[1] = (double)epl;
      ep_out[2] = 1.0;
    }
    if (ended && a.autoreset == RX_AUTORESET_NEXT_STEP) ef |= RX_EF_PENDING_RESET;
    if (FULL && ended && a.autoreset == RX_AUTORESET_SAME_STEP) do_reset = true;
  } else if (!REW && !stepping && a.io.ep_done) {
    a.io.ep_done[e] = 0;
  }
  // split: KIN writes the zero info of the envs it resets, REWARD that of the stepped ones
  if (a.io.info && (FULL || (REW && stepping) || (KIN && !stepping))) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      double* inf = a.io.info + (size_t)(2 * e + q) * RX_INFO_W;
      const bool keep = stepping;
      inf[RX_INFO_SPEED] = keep ? speed_of(c[q].vx, c[q].vy) : 0.0;
      inf[RX_INFO_PROGRESS] = keep ? ((fl[q] & RX_F_FINISHED) ? 1.0 : c[q].progress) : 0.0;
      inf[RX_INFO_PROGRESS_DELTA] = 0.0;
      inf[RX_INFO_PLACEMENT] = keep ? (double)place[q] : 0.0;
    }
  }
  if (!REW && do_reset) {  // multi_racing_env.py:118-153; start slot from the device RNG
    have_sc[0] = have_sc[1] = false;  // angles are reset below
    const uint64_t h = splitmix64(a.seed ^ splitmix64(((uint64_t)a.reset_count[e]++ << 32) ^ (uint64_t)e));
    // agent_order[0] after np.random.shuffle([0, 1]) (multi_racing_env.py:127-128): with
    // rx_set_start_draws the shuffle's own draw -- one MT19937 output u, j = u & 1,
    // swap when j == 0 -- of the env's turn in the reference's env-order reset
    // sequence; otherwise the device hash
    int first = (int)(h & 1ull);
    if (a.draws) {
      const int64_t j = *a.draw_base + a.reset_rank[e];
      first = (j < a.n_draws && (a.draws[j] & 1u)) ? 0 : 1;
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const double offset = ((double)((first == q) ? 0 : 1) - 0.5) * 3.5;
      c[q].x = meta[0] + meta[5] * offset;
      c[q].y = meta[1] + meta[6] * offset;
      c[q].angle = meta[2];
      c[q].vx = c[q].vy = 0.0;
      c[q].progress = 0.0;
      c[q].crashed = false;
      fl[q] = 0;
      last_steering[q] = 0.0;
      S.finished_step[2 * p + q] = -1;
    }
    steps = 0;
    ef &= (uint8_t)~(RX_EF_PENDING_RESET | RX_EF_TOUCH);
    if (KIN) ef |= RX_EF_RESET_NOW;
    S.ep_return[p] = 0.0;
    S.ep_length[p] = 0;
  }
  if (REW && do_reset) ef &= (uint8_t)~RX_EF_RESET_NOW;
  if (FULL && (stepping || do_reset)) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int i = 2 * p + q;
      S.x[i] = c[q].x;
      S.y[i] = c[q].y;
      S.angle[i] = c[q].angle;
      S.vx[i] = c[q].vx;
      S.vy[i] = c[q].vy;
      S.progress[i] = c[q].progress;
      S.last_progress[i] = c[q].progress;
      S.last_steering[i] = last_steering[q];
      S.flags[i] = fl[q];
    }
    S.steps[p] = steps;
    S.env_flags[p] = ef;
  }
  if (KIN && (stepping || do_reset)) {  // the pose the raycast and REWARD read
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int i = 2 * p + q;
      S.x[i] = c[q].x;
      S.y[i] = c[q].y;
      S.angle[i] = c[q].angle;
      S.vx[i] = c[q].vx;
      S.vy[i] = c[q].vy;
      S.last_steering[i] = last_steering[q];
      if (do_reset) {
        S.progress[i] = 0.0;
        S.last_progress[i] = 0.0;
        S.flags[i] = fl[q];
      }
    }
    S.steps[p] = steps;
    S.env_flags[p] = ef;
  }
  if (REW && (stepping || do_reset)) {
    if (stepping) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int i = 2 * p + q;
        S.progress[i] = c[q].progress;
        S.last_progress[i] = c[q].progress;
        S.flags[i] = fl[q];
      }
    }
    S.env_flags[p] = ef;
  }
  // outputs: reset-by-NEXT_STEP / explicit reset gives reward 0, term = trunc = False
  if (FULL || (REW && stepping) || (KIN && !stepping)) {
    const bool wrote_step = stepping;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      if (a.io.reward) a.io.reward[2 * e + q] = wrote_step ? (float)rw[q] : 0.0f;
      if (a.io.reward64) a.io.reward64[2 * e + q] = wrote_step ? rw[q] : 0.0;
    }
    const bool t_out = wrote_step && term, u_out = wrote_step && trunc;
    if (a.io.terminated) a.io.terminated[e] = t_out;
    if (a.io.truncated) a.io.truncated[e] = u_out;
    if (a.io.done_f32) a.io.done_f32[e] = (t_out || u_out) ? 1.0f : 0.0f;
  }
  // non-ray observation columns, multi_racing_env.py:226-271
#pragma unroll
  for (int q = 0; q < 2 && !REW; ++q) {
    const Car& me = c[q];
    const Car& o = c[1 - q];
    double s, co;
    if (have_sc[q]) {
      s = sn[q];
      co = cn[q];
    } else {
      rx_sincos(me.angle, &s, &co);
    }
    double vf = me.vx * co + me.vy * s;
    double vl = (-me.vx) * s + me.vy * co;
    double rx_ = o.x - me.x, ry_ = o.y - me.y;
    double lrx = rx_ * co + ry_ * s;
    double lry = (-rx_) * s + ry_ * co;
    double rvx = o.vx - me.vx, rvy = o.vy - me.vy;
    double lvx = rvx * co + rvy * s;
    double lvy = (-rvx) * s + rvy * co;
    float* ob = a.io.obs + (size_t)(2 * e + q) * a.D + a.n_sensors;
    ob[0] = (float)rx_clip(vf / RX_MAX_SPEED, -1.0, 1.0);
    ob[1] = (float)rx_clip(vl / RX_MAX_SPEED, -1.0, 1.0);
    ob[2] = (float)rx_clip(0.0 / 3.0, -1.0, 1.0);
    ob[3] = (float)last_steering[q];
    ob[4] = (float)rx_clip(lrx / maxd, -1.0, 1.0);
    ob[5] = (float)rx_clip(lry / maxd, -1.0, 1.0);
    ob[6] = (float)rx_clip(lvx / RX_MAX_SPEED, -1.0, 1.0);
    ob[7] = (float)rx_clip(lvy / RX_MAX_SPEED, -1.0, 1.0);
  }
  if (!KIN) write_sort_key(a, p, k, c[0].progress, W);
  if (!REW) {
    ang_out[0] = c[0].angle;
    ang_out[1] = c[1].angle;
    e_out = p;
  }
}

// k_dyn2 (PART = FULL) and k_kin2 (PART = KIN, one wave per workgroup so that
// block b's wave lands on the XCD of block b's REWARD and raycast waves).
template <int PART>
__global__ __launch_bounds__(256) void k_dyn2(rx_kargs a) {
  const int wave = uniform(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  if (wave >= a.n_dyn_waves) return;
  constexpr int NW = PART == RX_PART_KIN ? 1 : 4;  // k_kin2: one wave per workgroup
  extern __shared__ int32_t task_lds[];  // task_sort_lds_bytes (as k_dyn1)
  const int wl = NW == 1 ? 0 : (int)(threadIdx.x >> 6);
  int32_t* cnt = task_lds + wl * (kTaskSectors + 64 * 32);
  int32_t* stage = cnt + kTaskSectors;
  const bool sorting = a.tasks_out != nullptr;
  if (sorting) cnt[threadIdx.x & 63] = 0;
  const unsigned long long prof_t0 = prof_start(a);
  double ang[2], ep[3] = {0.0, 0.0, 0.0};
  int e = -1;
  dyn2_env<PART>(a, wave, ang, e, ep);
  if (PART == RX_PART_FULL) add_episode_stats(a, ep);
  if (sorting) sort_block_tasks<2>(a, uniform(a.dyn_waves[wave].perm_start), e, ang, cnt, stage);
  prof_end(a, wave, prof_t0);
}

// ============================================================ k_rays
// Track.raycast (environment/track.py:173-199) -- and for A == 2
// MultiTrack.raycast_with_cars (multi_track.py:5-44) -- one lane per
// (env, agent, ray).
//
// Exact division-free hit test.  With D = |dotp|, C = sgn(dotp)*cross,
// N = sgn(dotp)*dot (sign flips are exact, and IEEE division is sign-symmetric,
// so t = cross/dotp = C/D and s = dot/dotp = N/D bit for bit):
//   valid  <=> D > 1e-10
//   t >= 0 <=> C >= 0          (no underflow: |C| >= 1e-32 when nonzero here)
//   s >= 0 <=> N >= 0
//   s <= 1 <=> round(N/D) <= 1 <=> N <= D
// (both are doubles and D > 1e-10 is normal: N > D means N >= D + ulp(D) >
// D (1 + 2^-53), so N/D lies strictly above the rounding midpoint 1 + 2^-53 and
// rounds up to 1 + 2^-52; N <= D gives N/D <= 1 exactly.  Round 6: one compare
// where rounds 1-5 tested fl(N - D) <= D 2^-53, the same predicate in 3 VALU;
// tests/test_prefilter_cpu.py checks the equivalence on 4 M adversarial pairs).
// Only hit segments divide.
// The sign flips are one XOR of dotp's sign bit into the high words (not a
// compare + two selects): they differ from `dotp < 0 ? -x : x` only for dotp =
// -0.0 or NaN, where D > 1e-10 is false and no hit is reported either way.
// bestf (the float32 bound of best the box tests read) is refreshed by the
// callers once per scanned leaf, not per hit.
// Smallest float32 >= x (x >= 0): the f32 box tests compare against it.
__device__ __forceinline__ float f32_up(double x) {
  float f = (float)x;
  if ((double)f < x) f = __int_as_float(__float_as_int(f) + 1);
  return f;
}

__device__ __forceinline__ void seg_test(const double4 g, double ox, double oy, double v3x, double v3y, double& best) {
  const double v1x = ox - g.x, v1y = oy - g.y;
  const double dotp = g.z * v3x + g.w * v3y;
  const double cross = g.z * v1y - g.w * v1x;
  const double dot = v1x * v3x + v1y * v3y;
  const double D = __builtin_fabs(dotp);
  const long long sgn = __double_as_longlong(dotp) & (long long)0x8000000000000000ull;
  const double C = __longlong_as_double(__double_as_longlong(cross) ^ sgn);
  const double N = __longlong_as_double(__double_as_longlong(dot) ^ sgn);
  const bool hit = (D > 1e-10) & (C >= 0.0) & (N >= 0.0) & (N <= D);
  if (hit) {
    const double t = C / D;
    best = t < best ? t : best;
  }
}

typedef float rx_f2 __attribute__((ext_vector_type(2)));

// Segment pre-filter (float32, one lane's ray).  With a = (o - start) . v3
// (the reference's `dot`) and p = v2 . v3 (`dotp`), s = a / p lies in [0, 1]
// iff a and a - p do not share a strict sign, i.e. iff
// |2a - p| - |p| <= 0.  Computed in float32 from the float32 segment table as
// a = c0 - sx v3x - sy v3y with the lane's c0 = o . v3 (two fmas on the
// wave-uniform segment words, no packed operand copies) and p = sz v3x + sw v3y,
// the left side is within 2^-22 (5.5 M1 + 3 L) of its value on the f64
// operands (M1 = |ox| + |oy| + |sx| + |sy|, L = the slot's longest segment:
// input roundings 3 * 2^-24 M1, c0 2 * 2^-24 M1, the two fmas 2 * 2^-24 M1, p
// 4 * 2^-24 L, then 2a - p and the subtraction), and those differ from the
// exact one by ~2^-50 (M1 + L).  So a segment this test rejects, with
// e2 = 2^-17 (M1 + L + 1) >= 5.8x that bound, has a and a - p of one strict
// sign by a margin >= 2^-18 (M1 + L): the f64 test then sees N < 0 or
// N > D and reports no hit.  Rejecting it changes nothing; the
// wave runs the exact test on a segment iff some lane may hit it.
struct seg_pref {
  const float4* __restrict__ segf;  // the slot's float32 segments
  rx_f2 v3f;                        // (-sin, cos) in float32
  float c0;                         // of . v3f: the float32 origin projected on v3
  float e2;                         // 2^-17 (|ox| + |oy| + max(|sx| + |sy|) + L + 1)
#ifdef RX_RAY_STAMPS
  int* cnt;  // profiling build: [0] segments pre-filtered, [1] exact tests run, [2] of them with a lane's hit
#endif
};
__device__ __forceinline__ bool seg_may_hit(const float4 f, const seg_pref& pf) {
  const float aa = __builtin_fmaf(-f.y, pf.v3f.y, __builtin_fmaf(-f.x, pf.v3f.x, pf.c0));
  const float dp = __builtin_fmaf(f.w, pf.v3f.y, f.z * pf.v3f.x);
  return !(__builtin_fabsf(__builtin_fmaf(2.0f, aa, -dp)) - __builtin_fabsf(dp) > pf.e2);
}
// |x| - |y| as ONE v_sub_f32 with abs modifiers (the packed VALU has none)
__device__ __forceinline__ float abs_sub(float x, float y) {
  float d;
  asm("v_sub_f32_e64 %0, |%1|, |%2|" : "=v"(d) : "v"(x), "v"(y));
  return d;
}
// seg_may_hit for two segments at once, the same float32 operations: a, p and
// 2a - p of both in packed fmas (v_pk_fma_f32: 2.5 VALU per segment), then
// one abs-subtract each (left to itself the compiler pairs the abs-subtracts too,
// as 4 v_and + 1 v_pk_add, or packs nothing).  Same roundings: same decisions.
__device__ __forceinline__ void seg_may_hit2(const float4 f0, const float4 f1, const seg_pref& pf, bool& h0,
                                             bool& h1) {
  const rx_f2 vx = {pf.v3f.x, pf.v3f.x}, vy = {pf.v3f.y, pf.v3f.y}, c0 = {pf.c0, pf.c0};
  const rx_f2 aa = __builtin_elementwise_fma(-rx_f2{f0.y, f1.y}, vy, __builtin_elementwise_fma(-rx_f2{f0.x, f1.x}, vx, c0));
  const rx_f2 dp = __builtin_elementwise_fma(rx_f2{f0.w, f1.w}, vy, rx_f2{f0.z, f1.z} * vx);
  const rx_f2 u = __builtin_elementwise_fma(rx_f2{2.0f, 2.0f}, aa, -dp);
  h0 = !(abs_sub(u.x, dp.x) > pf.e2);
  h1 = !(abs_sub(u.y, dp.y) > pf.e2);
}

// Segments [j0, j1) of a wave-uniform slot, four scalar loads in flight at a
// time (each test ends in a divergent branch, so a plain loop would wait for
// every s_load on its own).  FILT: the exact test of a segment runs only if
// the float32 pre-filter passes for some lane.
template <bool FILT, bool LV = false>
__device__ __forceinline__ void ray_segments(const double4* __restrict__ seg, int j0, int j1, double ox, double oy,
                                             double v3x, double v3y, double& best, float& bestf, const seg_pref& pf) {
  int j = j0;
  if constexpr (FILT) {
    for (; j + 4 <= j1; j += 4) {
      const float4 f0 = ldt<LV>(pf.segf + j), f1 = ldt<LV>(pf.segf + j + 1), f2 = ldt<LV>(pf.segf + j + 2),
                   f3 = ldt<LV>(pf.segf + j + 3);
      bool m0, m1, m2, m3;
      seg_may_hit2(f0, f1, pf, m0, m1);
      seg_may_hit2(f2, f3, pf, m2, m3);
      const bool h0 = vote<LV>(m0), h1 = vote<LV>(m1), h2 = vote<LV>(m2), h3 = vote<LV>(m3);
#ifdef RX_RAY_STAMPS
      pf.cnt[0] += 4;
      const bool hh[4] = {h0, h1, h2, h3};
      for (int u = 0; u < 4; ++u) {
        if (!hh[u]) continue;
        const double b0 = best;
        seg_test(ldu(seg + j + u), ox, oy, v3x, v3y, best);
        pf.cnt[1] += 1;
        pf.cnt[2] += __any(best != b0) ? 1 : 0;
      }
      continue;
#endif
      if (h0) seg_test(ldt<LV>(seg + j), ox, oy, v3x, v3y, best);
      if (h1) seg_test(ldt<LV>(seg + j + 1), ox, oy, v3x, v3y, best);
      if (h2) seg_test(ldt<LV>(seg + j + 2), ox, oy, v3x, v3y, best);
      if (h3) seg_test(ldt<LV>(seg + j + 3), ox, oy, v3x, v3y, best);
    }
    for (; j < j1; ++j)
      if (vote<LV>(seg_may_hit(ldt<LV>(pf.segf + j), pf))) seg_test(ldt<LV>(seg + j), ox, oy, v3x, v3y, best);
    bestf = f32_up(best);
    return;
  }
  for (; j + 4 <= j1; j += 4) {
    const double4 g0 = ldt<LV>(seg + j), g1 = ldt<LV>(seg + j + 1), g2 = ldt<LV>(seg + j + 2), g3 = ldt<LV>(seg + j + 3);
    seg_test(g0, ox, oy, v3x, v3y, best);
    seg_test(g1, ox, oy, v3x, v3y, best);
    seg_test(g2, ox, oy, v3x, v3y, best);
    seg_test(g3, ox, oy, v3x, v3y, best);
  }
  for (; j < j1; ++j) seg_test(ldt<LV>(seg + j), ox, oy, v3x, v3y, best);
  bestf = f32_up(best);
}

// The four lanes of a quad (lanes 4i .. 4i+3) exchange a double: DPP
// quad_perm [1,0,3,2] / [2,3,0,1] (every lane of the wave active).
template <int CTRL>
__device__ __forceinline__ double quad_dpp(double v) {
  const unsigned long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp((int)(unsigned)u, (int)(unsigned)u, CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(unsigned)(u >> 32), (int)(unsigned)(u >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

#ifndef RX_LPR_PREFETCH
#define RX_LPR_PREFETCH 1
#endif
// One scanned leaf's segments [j0, j1) for the lanes of a wave.  LPR = 1: each
// lane tests all of them for its ray (ray_segments).  LPR = 2 or 4 (few envs:
// the raycast is a latency chain, rx_assign): LPR adjacent lanes of a quad
// hold the SAME ray and split the leaf (lane sub tests j0 + sub, j0 + sub +
// LPR, ...), then take the minimum of their bests, so every lane goes on with
// the ray's best -- the minimum over the leaf's exact hits, whoever tested
// which segment.
template <bool FILT, int LPR, bool LV = false, bool PF = false>
__device__ __forceinline__ void leaf_segments(const double4* __restrict__ seg, int j0, int j1, double ox, double oy,
                                              double v3x, double v3y, double& best, float& bestf, const seg_pref& pf) {
  if constexpr (LPR == 1) {
    ray_segments<FILT, LV>(seg, j0, j1, ox, oy, v3x, v3y, best, bestf, pf);
  } else {
    static_assert(!LV, "lane-varying slots: one lane per ray");
    static_assert(LPR == 2 || LPR == 4, "2 or 4 lanes per ray");
    const int sub = threadIdx.x & (LPR - 1);
    constexpr int PER = 8 / LPR;  // a lane's segments of a leaf of <= 8
    // PF: kernels scheduled at LPR lanes per ray (not the 1-lane kernels' tail split,
    // whose register budget the extra live loads would blow)
    if (PF && RX_LPR_PREFETCH && j1 - j0 <= 8) {
      // every segment of the lane's share loaded before the first test (one memory
      // round trip per leaf, not one per segment: the test's divergent branch kept
      // the compiler from hoisting the next load)
      double4 g[PER];
      float4 f[PER];
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int j = j0 + sub + LPR * k < j1 ? j0 + sub + LPR * k : j0;
        g[k] = seg[j];
        if constexpr (FILT) f[k] = pf.segf[j];
      }
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        bool may = j0 + sub + LPR * k < j1;
        if constexpr (FILT) may = may && seg_may_hit(f[k], pf);
        if (may) seg_test(g[k], ox, oy, v3x, v3y, best);
      }
    } else {
      for (int jb = j0; jb < j1; jb += LPR) {
        const int j = jb + sub < j1 ? jb + sub : j0;
        const double4 g = seg[j];
        bool may = jb + sub < j1;
        if constexpr (FILT) may = may && seg_may_hit(pf.segf[j], pf);
        if (may) seg_test(g, ox, oy, v3x, v3y, best);
      }
    }
    best = __builtin_fmin(best, quad_dpp<0xB1>(best));
    if constexpr (LPR == 4) best = __builtin_fmin(best, quad_dpp<0x4E>(best));
    bestf = f32_up(best);
  }
}

// Chunk culling (exact; derivation in DESIGN.md §3).  The 2W boundary
// segments of a slot are cut into chunks of G consecutive segments with
// axis-aligned boxes of their end points.  A computed hit on segment j means
// the exact line intersection P = o + t*.d lies within eps_s|v2| of the
// segment and the computed t_j >= t* - eps_t, where (|D| > 1e-10, |v1| <= R,
// t* <= T, |v2| <= L, u = 2^-53)
//   eps_t  <= u*L*(4R + 2T)/1e-10 + u*T,    eps_s|v2| <= u*(3R + 2L)*L/1e-10.
// So with the box grown by mb >= eps_s|v2| and the slab entry distance
// t_in <= t*, every hit of a chunk has t_j >= t_in - mt; if that is >= the
// lane's best t found so far, no segment of the chunk can lower the minimum
// and the chunk is skipped.  A wave skips a chunk only if all its lanes may.
// Chunks are visited outward from the wave's first car, so best tightens
// early; envs are kept spatially sorted (write_sort_key) so a wave's cars
// are neighbours.
// The slab test runs in packed float32 on outward-rounded f32 boxes: a slab
// plane's t = (b + n) / d is ONE v_pk_fma_f32 per box corner, b * id + c with
// the lane's c = n * id (n = the margin-grown origin offset, id = 1 / d)
// computed once per ray.  Conservative by construction: the
// per-lane box margin mbf adds 3(|ox|+|oy|+1)2^-24 for the f32 rounding of the
// origin and 2^-22(|ox|+|oy|+mbf) for the rounding of c (an absolute error of
// at most 2^-24 |n| in position units, covered 4x); the remaining roundings
// scale a slab endpoint by at most 1 +- 6*2^-24, and the slack k = 2^-20 >
// 2 * 6*2^-24 on both the empty-interval test and the entry distance absorbs
// them; bestf >= best.  |b * id| stays far below f32 overflow: no double lies
// within 2^-64 of an odd multiple of pi/2 at the angles a car reaches, so a
// nonzero cos / sin rounds to |d| > 2^-65 and |id| < 2^65.  An f32
// direction component of 0 makes id and c infinite: b * inf + c is +-inf or
// NaN, and fmin / fmax drop a NaN, leaving the axis unconstrained -- more
// boxes kept, never fewer.
// The box decision from the slab interval [lo, hi] (entry clamped at -mtf):
// x = lo - |lo| k and y = hi + |hi| k bound the exact entry from below and
// the exit from above (k = 2^-20 covers the <= 6 * 2^-24 relative roundings
// of lo and hi, and the 2 * 2^-24 of x and y themselves); the ray misses the
// box if x - y > 1e-6, and no segment in it can lower the lane's minimum if
// x >= bm = bestf + mtf (the caller's per-leaf sum: its rounding, 2^-24 of a
// value that x exceeds, is inside x's 2^-20 slack).  9 VALU per box test with
// the two packed fmas, max3 and min.
// (x and y as single v_fma_f32 with abs modifiers: left to itself the SLP
// vectorizer pairs them into a v_pk_fma_f32 plus a v_or and a v_and for the
// abs the packed form lacks.)
__device__ __forceinline__ bool slab_keep(float lo, float hi, float bm) {
  const float k = 0x1p-20f;
  float x, y;
  asm("v_fma_f32 %0, -|%1|, %2, %1" : "=v"(x) : "v"(lo), "s"(k));
  asm("v_fma_f32 %0, |%1|, %2, %1" : "=v"(y) : "v"(hi), "s"(k));
  return !(x - y > 1e-6f) && x < bm;
}
template <bool LV = false>
__device__ __forceinline__ bool chunk_needed_f(const float* __restrict__ box, rx_f2 clo, rx_f2 chi, rx_f2 id2,
                                               float mtf, float bm) {
  const float4 b = ldt<LV>(reinterpret_cast<const float4*>(box));
  const rx_f2 t1 = __builtin_elementwise_fma(rx_f2{b.x, b.y}, id2, clo);
  const rx_f2 t2 = __builtin_elementwise_fma(rx_f2{b.z, b.w}, id2, chi);
  const float lo = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(t1.x, t2.x), __builtin_fminf(t1.y, t2.y)), -mtf);
  const float hi = __builtin_fminf(__builtin_fmaxf(t1.x, t2.x), __builtin_fmaxf(t1.y, t2.y));
  return slab_keep(lo, hi, bm);
}

template <int A>
__device__ __forceinline__ void ray_finish(const rx_kargs& a, int pos, int q, int ray, double ox, double oy,
                                           double v3x, double v3y, double best);

// chunk_needed_f for a wave whose lanes all cast into one direction quadrant:
// the box comes quadrant-ordered as (near.x, near.y, far.x, far.y) and nn / nf
// are the matching origin offsets (times id), so each axis' entry / exit distance needs no
// min / max (4 fewer VALU).  Same decision as chunk_needed_f: with the axis'
// direction sign fixed, rounding is monotone, so min(t1, t2) IS the near
// plane's t and max(t1, t2) the far one's; only where chunk_needed_f meets a
// NaN (0 * inf: origin on a slab plane, f32 direction component 0) does this
// test drop the NaN and keep the box -- more conservative, never less.
template <bool LV = false>
__device__ __forceinline__ bool chunk_needed_q(const float* __restrict__ box, rx_f2 cn, rx_f2 cf, rx_f2 id2,
                                               float mtf, float bm) {
  const float4 b = ldt<LV>(reinterpret_cast<const float4*>(box));
  const rx_f2 tn = __builtin_elementwise_fma(rx_f2{b.x, b.y}, id2, cn);
  const rx_f2 tf = __builtin_elementwise_fma(rx_f2{b.z, b.w}, id2, cf);
  const float lo = __builtin_fmaxf(__builtin_fmaxf(tn.x, tn.y), -mtf);
  const float hi = __builtin_fminf(tf.x, tf.y);
  return slab_keep(lo, hi, bm);
}

// Lane-varying slots (RX_LEAF_BATCH): a kept super's 8 leaf boxes are tested as
// one batch against the bound of now -- the 8 per-lane box loads in flight
// together, one wait, instead of a load -> test -> branch chain per leaf.  The
// bound only falls (after a scan), so a leaf the batch rejects for every lane is
// rejected at its turn too; a candidate is re-tested exactly once a scan has
// lowered the bound since the batch.  The leaves scanned, their order, and so
// every result, are those of the one-at-a-time loop.  Stress pool, 65,536 envs:
// k_step2 196.9 -> 148.3 us.  Slot-uniform waves keep the one-at-a-time loop:
// their scalar loads hit the scalar cache, and the re-tests and the batch's SGPRs
// cost more than the chain (seed-1 pool 56.8 -> 60.7 us, 4,096 envs 20.3 ->
// 22.2 us); batching both sides' super boxes as well was slower (156 us).
// profiles/r06/j_*, k_*.
#ifndef RX_LEAF_BATCH
#define RX_LEAF_BATCH 1
#endif
// The culled scan of one lane's ray over slot k's chunks (cull_chunk G > 0),
// visiting them outward from chunk c0.  FAST: quadrant-ordered box block
// `block` (1..4) with chunk_needed_q and offsets (n1, n2) = (near, far) * id;
// otherwise block 0 with chunk_needed_f and (n1, n2) = (nlo, nhi) * id.
template <bool FAST, bool FILT, int LPR, bool LV = false, bool PF = false>
__device__ __forceinline__ void cull_scan(const rx_kargs& a, int k, int W, int nch, const double4* __restrict__ seg,
                                          int c0, int block, rx_f2 n1, rx_f2 n2, rx_f2 id2, float mtf, double ox,
                                          double oy, double v3x, double v3y, double& best, float& bestf, int& tested,
                                          int& scanned, const seg_pref& pf) {
  const int G = a.cull_chunk;
  const float* __restrict__ fboxes =
      a.tr.chunk_box_f +
      4 * ((size_t)block * a.tr.n_chunk_boxes + (size_t)(LV ? a.tr.hdr[k].chunk_off : uniform(a.tr.chunk_off[k])));
  float bm = bestf + mtf;  // refreshed with bestf after every leaf scan
  auto needed = [&](const float* box) {
    return FAST ? chunk_needed_q<LV>(box, n1, n2, id2, mtf, bm) : chunk_needed_f<LV>(box, n1, n2, id2, mtf, bm);
  };
  const int SG = a.cull_super;
  if (SG <= 0) {
    for (int s = 0; s < nch; ++s) {
      const int off = (s + 1) >> 1;
      int c = (s & 1) ? c0 - off : c0 + off;
      c = c < 0 ? c + nch : (c >= nch ? c - nch : c);
#pragma unroll
      for (int side = 0; side < 2; ++side) {
        ++tested;
        if (vote<LV>(needed(fboxes + 4 * (side * nch + c)))) {
          ++scanned;
          leaf_segments<FILT, LPR, LV, PF>(seg, side * W + c * G, side * W + min(W, (c + 1) * G), ox, oy, v3x, v3y,
                                       best, bestf, pf);
          bm = bestf + mtf;
        }
      }
    }
    return;
  }
  // two levels: a super-chunk box (union of SG chunk boxes) first; its
  // chunks are tested only if some lane may need it.  A chunk inside a
  // skipped super-chunk is skipped by the same bound, so the result is
  // unchanged (exactness argument of chunk_needed applies to any box that
  // contains the segments).
  const int nsup = (nch + SG - 1) / SG;
  const float* __restrict__ sboxes =
      a.tr.super_box_f +
      4 * ((size_t)block * a.tr.n_super_boxes + (size_t)(LV ? a.tr.hdr[k].super_off : uniform(a.tr.super_off[k])));
  const int u0 = uni<LV>(c0 / SG);
  constexpr bool BATCH = LV && RX_LEAF_BATCH;
  for (int s = 0; s < nsup; ++s) {
    const int off = (s + 1) >> 1;
    const bool back = (s & 1) != 0;
    int u = back ? u0 - off : u0 + off;
    u = u < 0 ? u + nsup : (u >= nsup ? u - nsup : u);
    const int l0 = u * SG, nl = min(nch, l0 + SG) - l0;
#pragma unroll
    for (int side = 0; side < 2; ++side) {
      ++tested;
      if (!vote<LV>(needed(sboxes + 4 * (side * nsup + u)))) continue;
      if (BATCH && SG == 8) {
        unsigned m = 0;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int qq = q < nl ? q : nl - 1;
          const int c = l0 + (back ? nl - 1 - qq : qq);
          if (vote<LV>(needed(fboxes + 4 * (side * nch + c))) && q < nl) m |= 1u << q;
        }
        tested += nl;
        bool dirty = false;  // a scan has lowered bm since the batch
        while (m) {
          const int q = __builtin_ctz(m);
          m &= m - 1;
          const int c = l0 + (back ? nl - 1 - q : q);
          if (dirty) {
            ++tested;
            if (!vote<LV>(needed(fboxes + 4 * (side * nch + c)))) continue;
          }
          ++scanned;
          leaf_segments<FILT, LPR, LV, PF>(seg, side * W + c * G, side * W + min(W, (c + 1) * G), ox, oy, v3x, v3y,
                                       best, bestf, pf);
          bm = bestf + mtf;
          dirty = true;
        }
        continue;
      }
      for (int q = 0; q < nl; ++q) {
        const int c = l0 + (back ? nl - 1 - q : q);  // forward supers ascending, backward ones descending
        ++tested;
        if (vote<LV>(needed(fboxes + 4 * (side * nch + c)))) {
          ++scanned;
          leaf_segments<FILT, LPR, LV, PF>(seg, side * W + c * G, side * W + min(W, (c + 1) * G), ox, oy, v3x, v3y,
                                       best, bestf, pf);
          bm = bestf + mtf;
        }
      }
    }
  }
}

// Profiling build only (-DRX_RAY_STAMPS, tools/ray_stamps.py): per ray wave,
// s_memtime after a full s_waitcnt at phase boundaries (0 entry, 1 task + state
// loads, 2 sincos, 3 culling setup, 4 traversal, 5 obs store), the wall clock
// at entry / exit (6, 7) and the wave's box tests / leaf scans (8, 9), written
// to io.counters[16 + 12 * wave + j].  The product library has no stamps.
#ifdef RX_RAY_STAMPS
#define RAY_STAMP(j)                                 \
  do {                                               \
    __builtin_amdgcn_s_waitcnt(0);                   \
    rstamp[j] = __builtin_amdgcn_s_memtime();        \
  } while (0)
#else
#define RAY_STAMP(j) \
  do {               \
  } while (0)
#endif

// One ray wave: the wave record `we` (slot, tasks [task_start, task_start + count)
// of `tasks`: the ray-wave table's record and the global task buffer in k_step2 /
// k_rays).  `wave` only indexes the profiling stamps.
// LV (lane-varying slots): the wave's tasks are the (env, agent, ray) tasks of its
// 64-env block in env-major order -- 11 rays of ~6 envs, so lanes of one env share
// their slot's cache lines -- and every lane reads its own env's slot.
template <int A, int LPR, bool LV = false, bool PF = false>
__device__ __forceinline__ void rays_wave(const rx_kargs& a, const rx_wave we, const int32_t* tasks, int wave) {
  static_assert(!LV || LPR == 1, "lane-varying slots: one lane per ray");
#ifdef RX_RAY_STAMPS
  unsigned long long rstamp[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  rstamp[6] = wall_clock64();
  RAY_STAMP(0);
#endif
  const int lane = threadIdx.x & 63;
  const int kw = LV ? 0 : uniform(we.track);
  int wp0 = 0, W = 0;
  if constexpr (!LV) {
    wp0 = uniform(a.tr.wp_off[kw]);
    W = uniform(a.tr.wp_off[kw + 1]) - wp0;
  }
  const int count = uniform(we.count);  // tasks of this wave (64 / LPR at most)
  if (count <= 0) return;
  // LPR lanes per task; lanes past the wave's tasks repeat its last one (their
  // values equal that task's at every point, so no wave vote or minimum
  // changes and every lane stays active for the quad exchanges); only the
  // first lane of an own task writes
  const int tl = lane / LPR;
  const bool own = tl < count;
  const int R = a.n_sensors;
  const int task = we.task_start + (own ? tl : count - 1);
  int env_local = 0, q, ray, pos;
  if (LV || a.ray_order == 0) {  // (env, agent, ray): 11 rays of ~6 envs per wave
    env_local = task / (A * R);
    const int rem = task - env_local * (A * R);
    q = rem / R;
    ray = rem - q * R;
  } else if (a.ray_order == 2) {  // sorted (agent, ray) tasks: direction- and position-binned waves
    const int t = ldc(tasks + task);
    const int iq = t / R;
    ray = t - iq * R;
    pos = iq / A;
    q = iq - pos * A;
  } else {  // ray-major: one (agent, ray) over consecutive (position-sorted) envs
    const int ng = uniform(a.slot_nenv[kw]);
    const int qr = task / ng;
    env_local = task - qr * ng;
    q = qr / R;
    ray = qr - q * R;
  }
  if (LV || a.ray_order != 2) pos = we.perm_start + env_local;
  int k = kw;
  if constexpr (LV) {  // the lane's env's slot
    k = a.pos_slot[pos];
    wp0 = a.tr.hdr[k].wp0;
    W = a.tr.hdr[k].W;
  }
  const int S_ = 2 * W;
  const double4* __restrict__ seg = reinterpret_cast<const double4*>(a.tr.seg) + 2 * wp0;
  const int i = A * pos + q;  // working state (position order); the obs row is A * perm[pos] + q
  const double ox = ldc(a.st.x + i), oy = ldc(a.st.y + i);
  const double theta = ldc(a.st.angle + i) + a.rel_angles[ray];  // racing_env.py:50
  RAY_STAMP(1);
  double sn, cs;
  rx_sincos(theta, &sn, &cs);
  const double v3x = -sn, v3y = cs;
  RAY_STAMP(2);
  double best = __builtin_inf();
  float bestf = __builtin_inff();
  const int G = a.cull_chunk;
  if (G <= 0) {
    ray_segments<false, LV>(seg, 0, S_, ox, oy, v3x, v3y, best, bestf, seg_pref{});
  } else {
    const int nch = (W + G - 1) / G;  // chunks per side
    const double* __restrict__ sg = LV ? a.tr.hdr[k].geo : a.tr.slot_geo + 4 * k;
    const double cx = sg[0], cy = sg[1], rad = sg[2], L = sg[3];
    const double ddx = ox - cx, ddy = oy - cy;
    const double Rr = __builtin_sqrt(ddx * ddx + ddy * ddy) + rad;  // >= |o - p| for every boundary point p
    const double T = Rr + L;
    const double u2 = 0x1p-52;  // 2u: factor-2 safety on both bounds
    const double mt = u2 * L * (4.0 * Rr + 2.0 * T) * 1e10 + u2 * T + 1e-9;
    const double mb = u2 * (3.0 * Rr + 2.0 * L) * L * 1e10 + 1e-9;
    // float32 box-test operands (chunk_needed_f): origin, margins, inverse direction d = (cos, sin)
    const float oxf = (float)ox, oyf = (float)oy;
    const float mbf0 = (float)mb * (1.0f + 0x1p-20f) +
                       3.0f * (__builtin_fabsf(oxf) + __builtin_fabsf(oyf) + 1.0f) * 0x1p-24f;
    const float mbf = mbf0 + (__builtin_fabsf(oxf) + __builtin_fabsf(oyf) + mbf0) * 0x1p-22f;  // + c's rounding
    const float mtf = (float)mt * (1.0f + 0x1p-20f) + 1e-6f;
    const rx_f2 nlo = {-(oxf + mbf), -(oyf + mbf)}, nhi = {mbf - oxf, mbf - oyf};
    const float csf = (float)cs, snf = (float)sn;
    const rx_f2 id2 = {1.0f / csf, 1.0f / snf};
    // visit chunks outward from the wave's first car
    int w0 = (int)(ldc(a.st.progress + i) * (double)W + 0.5);
    w0 = w0 < 0 ? 0 : (w0 >= W ? W - 1 : w0);
    const int c0 = uni<LV>(w0 / G);
    // direction quadrant (sign bits of the f32 direction, as id2's signs): a
    // wave whose lanes all share it takes the quadrant-ordered box tables
    const int quad = (int)(__float_as_uint(csf) >> 31) | (int)((__float_as_uint(snf) >> 31) << 1);
    const int quad0 = uniform(quad);
    int scanned = 0, tested = 0;
    // segment pre-filter operands (seg_may_hit): |sx| + |sy| <= |cx| + |cy| + 2 rad for every boundary point
#ifdef RX_RAY_STAMPS
    int cnt[3] = {0, 0, 0};
#endif
    const seg_pref pf{reinterpret_cast<const float4*>(a.tr.seg_f) + 2 * wp0, rx_f2{-snf, csf},
                      __builtin_fmaf(oyf, csf, oxf * -snf),
                      (float)((__builtin_fabs(ox) + __builtin_fabs(oy) + __builtin_fabs(cx) + __builtin_fabs(cy) +
                               2.0 * rad + L + 1.0) * 0x1p-17)
#ifdef RX_RAY_STAMPS
                      , cnt
#endif
    };
    RAY_STAMP(3);
    auto scan = [&](auto filt) {
      constexpr bool F = decltype(filt)::value;
      // LV: the plain box table (block 0) -- the lanes of an env then share its box lines
      // whatever their quadrants (fewer lines per wave: stress pool 213 -> 200 us)
      if (!LV && a.box_quadrants && __all(quad == quad0)) {
        const rx_f2 nn = {(quad0 & 1) ? nhi.x : nlo.x, (quad0 & 2) ? nhi.y : nlo.y};
        const rx_f2 nf = {(quad0 & 1) ? nlo.x : nhi.x, (quad0 & 2) ? nlo.y : nhi.y};
        cull_scan<true, F, LPR, LV, PF>(a, k, W, nch, seg, c0, quad0 + 1, nn * id2, nf * id2, id2, mtf, ox, oy, v3x,
                                    v3y, best, bestf, tested, scanned, pf);
      } else {
        cull_scan<false, F, LPR, LV, PF>(a, k, W, nch, seg, c0, 0, nlo * id2, nhi * id2, id2, mtf, ox, oy, v3x, v3y,
                                     best, bestf, tested, scanned, pf);
      }
    };
    // LV: no float32 pre-filter -- with per-lane segment loads the filter's extra
    // 16-byte load per segment costs more than the f64 tests it saves (stress pool,
    // 65,536 envs: k_step2 247 -> 216 us, profiles/r06/d_lv_ab.jsonl), and leaving
    // it out of the lane-varying kernels frees registers for a sixth wave per SIMD
    if (!LV && a.seg_filter && a.tr.seg_f)
      scan(std::true_type{});
    else
      scan(std::false_type{});
    RAY_STAMP(4);
#ifdef RX_RAY_STAMPS
    rstamp[8] = (unsigned long long)tested;
    rstamp[9] = (unsigned long long)scanned;
    rstamp[10] = (unsigned long long)cnt[1] | ((unsigned long long)cnt[2] << 32);  // exact tests | that lowered a best
    rstamp[11] = (unsigned long long)cnt[0];                                       // segments pre-filtered
#else
    if (a.io.counters && (LV || lane == (__builtin_amdgcn_readfirstlane(threadIdx.x) & 63))) {
      atomicAdd(&a.io.counters[0], (unsigned long long)tested);  // LV: every lane its own tests
      atomicAdd(&a.io.counters[1], (unsigned long long)scanned);
    }
#endif
  }
  if (own && (lane & (LPR - 1)) == 0) ray_finish<A>(a, pos, q, ray, ox, oy, v3x, v3y, best);
#ifdef RX_RAY_STAMPS
  RAY_STAMP(5);
  rstamp[7] = wall_clock64();
  if (a.io.counters && lane == (__builtin_amdgcn_readfirstlane(threadIdx.x) & 63))
    for (int j = 0; j < 12; ++j) a.io.counters[16 + 12 * wave + j] = rstamp[j];
#endif
}

// The observation of one ray from the wall minimum `best` (inf = no hit):
// Track.raycast's max_dist for no hit (track.py:199, uncapped otherwise),
// the other car's edges for A = 2 (MultiTrack.raycast_with_cars,
// multi_track.py:5-44), float32 division by 50 (racing_env.py:46,51,53).
template <int A>
__device__ __forceinline__ void ray_finish(const rx_kargs& a, int pos, int q, int ray, double ox, double oy,
                                           double v3x, double v3y, double best) {
  double dist = (best == __builtin_inf()) ? RX_MAX_RANGE : best;
  if (A == 2) {
    const int o = A * pos + (1 - q);  // the other car (working state)
    const double ocx = a.st.x[o], ocy = a.st.y[o];
    const double dx = ocx - ox, dy = ocy - oy;
    double min_car = RX_MAX_RANGE;
    if (!(__builtin_sqrt(rx_dot2_np(dx, dy, dx, dy)) < 0.5)) {  // multi_track.py:12-14
      double os, oc, qx[4], qy[4];
      rx_sincos(a.st.angle[o], &os, &oc);
      corners(ocx, ocy, oc, os, qx, qy);
#pragma unroll
      for (int m = 0; m < 4; ++m) {  // ray_seg_intersection, multi_track.py:28-44
        const double sx = qx[m], sy = qy[m], ex = qx[(m + 1) & 3], ey = qy[(m + 1) & 3];
        const double v1x = ox - sx, v1y = oy - sy;
        const double v2x = ex - sx, v2y = ey - sy;
        const double dotp = rx_dot2_np(v2x, v2y, v3x, v3y);
        if (!(__builtin_fabs(dotp) < 1e-10)) {
          const double t = (v2x * v1y - v2y * v1x) / dotp;
          const double s = rx_dot2_np(v1x, v1y, v3x, v3y) / dotp;
          if (t >= 0 && 0 <= s && s <= 1 && t < min_car) min_car = t;
        }
      }
    }
    dist = (min_car < dist) ? min_car : dist;
  }
  const int e = RX_IO_ROW(a, pos);
  a.io.obs[(size_t)(A * e + q) * a.D + ray] = (float)dist / 50.0f;  // racing_env.py:46,51,53
}

template <int A, int LPR, bool LV = false, bool PF = false>
__device__ __forceinline__ void rays_body(const rx_kargs& a, int wave) {
  if (wave >= a.n_ray_waves) return;
  rays_wave<A, LPR, LV, PF>(a, a.ray_waves[wave], a.tasks, wave);
}

// A ray wave of the table: at the schedule's LPR lanes per ray, or -- for the
// dispatch tail (rx_config.ray_tail: the waves at and after a.ray_tail_from,
// 64 / ray_tail_lpr tasks each, rx_assign) -- at ray_tail_lpr lanes per ray.
// Only one-lane-per-ray schedules have a tail.
// Single-agent envs: the ray waves dispatched in the last (100 - RX_RAY_PRIO_FROM) %
// of the table (the centre classes, whose chains end the launch) take issue
// priority RX_RAY_PRIO over the waves sharing their SIMD.  Scheduling only.
// Same-session A/B (profiles/r04/ab_ray_prio_{1,2}.txt, ab_ray_prio_sizes.txt):
// 65,536 envs 827.6-830.0 -> 837.4-844.7 M env-steps/s (k_step2 67.5 -> 65.3-66.7 us),
// 4,096 envs +2.8 %, 16,384 +2 %; from 50 / 60 % of the table -5 / -4 %, priority 2-3
// no better than 1; two-car envs -5.5 % at 8,192 (off there)
#ifndef RX_RAY_PRIO
#define RX_RAY_PRIO 1
#endif
#ifndef RX_RAY_PRIO_FROM
#define RX_RAY_PRIO_FROM 70
#endif
template <int A, int LPR, bool LV = false, bool PF = false>
__device__ __forceinline__ void rays_dispatch(const rx_kargs& a, int wave) {
  if constexpr (LV) {  // no tail split, no dispatch-order priority (rx_assign: group-octet-major)
    rays_body<A, 1, true>(a, wave);
    return;
  }
  if constexpr (A == 1 && RX_RAY_PRIO > 0) {
    if (wave * 100 >= a.n_ray_waves * RX_RAY_PRIO_FROM) __builtin_amdgcn_s_setprio(RX_RAY_PRIO);
  }
  if constexpr (LPR == 1) {
    if (a.ray_tail_from >= 0 && wave >= a.ray_tail_from) {
      if (a.ray_tail_lpr == 4)
        rays_body<A, 4, false, false>(a, wave);
      else
        rays_body<A, 2, false, false>(a, wave);
      return;
    }
  }
  rays_body<A, LPR, false, PF>(a, wave);
}

template <int A, bool LV = false>
__global__ __launch_bounds__(256) void k_rays(rx_kargs a) {
  const int wave = uniform(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  const unsigned long long prof_t0 = prof_start(a);
  if (LV)
    rays_dispatch<A, 1, LV>(a, wave);
  else if (a.ray_lpr == 4)
    rays_body<A, 4>(a, wave);
  else if (a.ray_lpr == 2)
    rays_body<A, 2>(a, wave);
  else
    rays_dispatch<A, 1>(a, wave);
  prof_end(a, wave, prof_t0);
}

// Small-N raycast (a.wide: few envs, latency-bound): one WAVE per (env,
// agent, ray) task in env order; the 64 lanes split the slot's 2W boundary
// segments (lane l tests j = l, l + 64, ...; coalesced loads), then a wave
// minimum.  Brute force, so no culling argument is involved; the min over the
// exact t of hits is order-independent, hence bit-identical to k_rays.
template <int A>
__device__ __forceinline__ void ray_wide(const rx_kargs& a, int iq, int ray, const double4* seg_lds = nullptr) {
  const int pos = iq / A, q = iq - pos * A;  // iq = A * position + agent (working state)
  const int k = uniform(a.st.track[a.perm[pos]]);
  const int wp0 = uniform(a.tr.wp_off[k]);
  const int S_ = 2 * (uniform(a.tr.wp_off[k + 1]) - wp0);
  const double4* __restrict__ seg = seg_lds ? seg_lds : reinterpret_cast<const double4*>(a.tr.seg) + 2 * wp0;
  const double ox = a.st.x[iq], oy = a.st.y[iq];
  double sn, cs;
  rx_sincos(a.st.angle[iq] + a.rel_angles[ray], &sn, &cs);  // racing_env.py:50
  const double v3x = -sn, v3y = cs;
  double best = __builtin_inf();
  int j = threadIdx.x & 63;
  for (; j + 192 < S_; j += 256) {  // four coalesced loads in flight before the (divergent) tests
    const double4 g0 = seg[j], g1 = seg[j + 64], g2 = seg[j + 128], g3 = seg[j + 192];
    seg_test(g0, ox, oy, v3x, v3y, best);
    seg_test(g1, ox, oy, v3x, v3y, best);
    seg_test(g2, ox, oy, v3x, v3y, best);
    seg_test(g3, ox, oy, v3x, v3y, best);
  }
  for (; j < S_; j += 64) seg_test(seg[j], ox, oy, v3x, v3y, best);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) best = __builtin_fmin(best, __shfl_xor(best, o, 64));
  if ((threadIdx.x & 63) == 0) ray_finish<A>(a, pos, q, ray, ox, oy, v3x, v3y, best);
}

template <int A>
__global__ __launch_bounds__(256) void k_rays_wide(rx_kargs a) {
  const int wave = uniform(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  const unsigned long long prof_t0 = prof_start(a);
  const int R = a.n_sensors;
  if (wave < a.n_wide_tasks) {
    const int iq = wave / R;
    ray_wide<A>(a, iq, wave - iq * R);
  }
  prof_end(a, wave, prof_t0);
}

// Second kernel of the split step (A = 1, rx_api.cpp): one wave per
// workgroup; workgroups [0, n_rw) run the REWARD part of RacingEnv.step for
// dynamics wave blockIdx (n_rw = n_dyn_waves rounded up to 8, so the raycast
// waves keep their XCD placement), the rest cast rays for ray wave
// blockIdx - n_rw.  The two halves share no data they write (REWARD reads the
// stepped positions k_kin1 wrote; the raycast reads them and, as an ordering
// hint only, progress), so they run side by side: the latency-bound argmin
// hides under the VALU-bound raycast.
#ifndef RX_REWARD_PRIO
#define RX_REWARD_PRIO 0
#endif
#ifndef RX_STEP2_MINW
#define RX_STEP2_MINW 8  // min waves per SIMD: caps VGPRs at 64 so the raycast half keeps full occupancy (some spills in the REWARD half)
#endif
#ifndef RX_STEP2_MINW_LV
// lane-varying slots (k_step2<1, 1, 1, true>): 6 waves per SIMD (80 VGPRs, 22 spilled) -- stress pool,
// 65,536 envs, k_step2 216 / 213 / 227 us at 5 / 6 / 7 waves, 200 us at 6 with the plain box tables
// (profiles/r06/e_lv_nf.jsonl)
#define RX_STEP2_MINW_LV 6
#endif
#ifndef RX_STEP2_MINW_2
#define RX_STEP2_MINW_2 6  // two-car k_step2<2>: 80 VGPRs (fewer REWARD spills; 8 -> 6 waves: +9 % at 8,192 envs, +1 % at 65,536)
#endif
// One instantiation per (REWARD lanes per env, lanes per ray) schedule: with
// the three schedules of each half inlined into ONE kernel, its register
// allocation was the maximum over all of them, and the REWARD half spilled at
// the raycast's 64-VGPR cap (k_step2<1>: 36 B/lane of scratch) whichever
// schedule ran.  For A = 2, RLPE 2 gives each car of an env its own lane in the
// REWARD half (dyn2_env<REWARD, 2>).
template <int A, int RLPE, int LPR, bool LV = false>
__global__ __launch_bounds__(64, A == 1 ? (LV ? RX_STEP2_MINW_LV : RX_STEP2_MINW) : RX_STEP2_MINW_2) void k_step2(
    rx_kargs a, int n_rw) {
  const int b = uniform((int)blockIdx.x);
  const unsigned long long prof_t0 = prof_start(a);
  if (b < n_rw) {
#if RX_REWARD_PRIO > 0
    // issue priority over the raycast waves sharing the SIMD: the REWARD
    // waves are long latency chains that would otherwise finish last
    __builtin_amdgcn_s_setprio(RX_REWARD_PRIO);
#endif
    double ang[A], ep[3] = {0.0, 0.0, 0.0};
    int e = -1;
    if constexpr (A == 1) {
      // RLPE lanes per env (fewer argmin points per lane; few envs):
      // block b = sub-block * n1 + dynamics wave, so a REWARD wave keeps the
      // XCD (b % 8) of its k_kin1 wave (n1 = n_dyn_waves rounded up to 8)
      const int n1 = n_rw / RLPE, w = b % n1, sb = b / n1;
      dyn1_env<RLPE, RX_PART_REWARD, LV>(a, w, ang, e, ep, RLPE == 1 ? 0 : sb);
    } else if constexpr (RLPE == 2) {
      const int n1 = n_rw / 2, w = b % n1, sb = b / n1;  // as the single-agent REWARD half at 2 lanes
      dyn2_env<RX_PART_REWARD, 2>(a, w, ang, e, ep, sb);
    } else {
      dyn2_env<RX_PART_REWARD>(a, b, ang, e, ep);
    }
    add_episode_stats(a, ep);
  } else {
    rays_dispatch<A, LPR, LV, LPR == 4>(a, b - n_rw);  // PF: prefetched leaf scans at 4 lanes per ray
  }
  prof_end(a, b, prof_t0);
}

// ============================================================ k_rollout
// PPO.collect_rollout (agent/ppo.py:97-132) for few single-agent envs as ONE
// persistent launch (rx_rollout): workgroup b = the env of dynamics wave b
// (small N: one env per wave), and per step t
//   policy   : waves 0 / 1 = actor / critic trunk on obs[t], lane = hidden
//              unit, weights staged once in LDS (transposed: lane reads are
//              conflict-free).  Every output is the fmaf chain, in the same
//              order, that k_policy_act's MFMAs compute (rx_ppo.hip: inputs in
//              order, hidden units in the order t, r, q), so actions,
//              log-probs and values equal rx_policy_act's with the same eps
//              bit for bit;
//   dynamics : wave 0 runs RacingEnv.step (dyn1_env<64, FULL>, as k_dyn1<64>);
//   raycast  : wave w casts rays w, w + kRollWaves, ... (ray_wide, as
//              k_rays_wide) into obs[t+1].
// An env's actions depend only on its own observations, so workgroups never
// wait for each other: the T steps run back to back inside the workgroup with
// three barriers per step and no kernel launch between them.
#ifndef RX_ROLL_WAVES
#define RX_ROLL_WAVES 12
#endif
constexpr int kRollWaves = RX_ROLL_WAVES;

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

template <int D>
__global__ __launch_bounds__(64 * kRollWaves) void k_rollout(rx_kargs a, rx_rollout_io r) {
  using L = rx_policy::Lay<D>;
  constexpr int H = rx_policy::kH, NA = rx_policy::kNA;
  __shared__ float sW1[2][D * H];  // [trunk][d][j] = W1[j][d]
  __shared__ float sW2[2][H * H];  // [trunk][k][j] = W2[j][k]
  __shared__ float sX[2][D], sH1[2][H], sH2[2][H];
  __shared__ float sW3[NA * H];  // actor head
  const int b = blockIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int64_t n = a.n_dyn_waves;  // = envs (one per dynamics wave)
  const int pos = a.dyn_waves[b].perm_start;  // working-state position of this workgroup's env
  const int e = a.perm[pos];                   // its env id: the rollout buffers' row
  const float* __restrict__ P = r.params;
  for (int i = threadIdx.x; i < D * H; i += blockDim.x) {
    const int j = i / D, d = i - j * D;
    sW1[0][d * H + j] = P[L::aW1 + i];
    sW1[1][d * H + j] = P[L::cW1 + i];
  }
  for (int i = threadIdx.x; i < H * H; i += blockDim.x) {
    const int j = i / H, k = i - j * H;
    sW2[0][k * H + j] = P[L::aW2 + i];
    sW2[1][k * H + j] = P[L::cW2 + i];
  }
  for (int i = threadIdx.x; i < NA * H; i += blockDim.x) sW3[i] = P[L::aW3 + i];
  // every other policy constant in LDS too: the per-step chain then waits on
  // no global load (biases, the critic head, the actor's scale terms)
  __shared__ float sB[2][2][H];  // [trunk][layer][unit]
  __shared__ float sW3c[H];      // critic head
  __shared__ float sK[8];        // ab3[0..1], cb3, scale[0..1], log scale[0..1]
  __shared__ float2 sAct;        // actions[t] of this env: actor -> the dynamics wave
  __shared__ int sObsTaken;      // steps whose obs the critic wave has copied (split step: KIN waits for it)
  if (threadIdx.x == 0) sObsTaken = 0;
  for (int i = threadIdx.x; i < H; i += blockDim.x) {
    sB[0][0][i] = P[L::ab1 + i], sB[0][1][i] = P[L::ab2 + i];
    sB[1][0][i] = P[L::cb1 + i], sB[1][1][i] = P[L::cb2 + i];
    sW3c[i] = P[L::cW3 + i];
  }
  if (threadIdx.x < NA) {  // Normal(mu, exp(log_std)): the same expf / logf per step as before, once
    const float scale = expf(r.log_std[threadIdx.x]);
    sK[threadIdx.x] = P[L::ab3 + threadIdx.x];
    sK[3 + threadIdx.x] = scale;
    sK[5 + threadIdx.x] = logf(scale);
  }
  if (threadIdx.x == 0) sK[2] = P[L::cb3];
  // the env's slot, read every step by the argmins, the collision test and the
  // 11 raycasts: LDS latency instead of L2 round trips (rx_rollout sizes it)
  extern __shared__ double4 sSlot[];  // [2W] segments, then [W] waypoints, [W] normals (double2)
  const int k = a.st.track[e];
  const int wp0 = a.tr.wp_off[k], W = a.tr.wp_off[k + 1] - wp0;
  {
    const double4* __restrict__ gseg = reinterpret_cast<const double4*>(a.tr.seg) + 2 * wp0;
    const double2* __restrict__ gwp = reinterpret_cast<const double2*>(a.tr.wp) + wp0;
    const double2* __restrict__ gnrm = reinterpret_cast<const double2*>(a.tr.nrm) + wp0;
    double2* lwp = reinterpret_cast<double2*>(sSlot + 2 * W);
    for (int i = threadIdx.x; i < 2 * W; i += blockDim.x) sSlot[i] = gseg[i];
    for (int i = threadIdx.x; i < W; i += blockDim.x) {
      lwp[i] = gwp[i];
      lwp[W + i] = gnrm[i];
    }
  }
  const rx_slot_lds sl{reinterpret_cast<const double2*>(sSlot + 2 * W),
                       reinterpret_cast<const double2*>(sSlot + 2 * W) + W, sSlot};
  // The env's working-state row, KIN's cos / sin and its observation row live
  // in LDS for the whole rollout (read back at the end): the device functions
  // index state by position p = pos and obs by env id e, so they get pointers
  // offset by -pos / -e*D into LDS (generic addressing) and every per-step
  // state round trip is an LDS access instead of an L2 / HBM one.  The obs row
  // is copied to the rollout buffer once per step, off the critical path.
  __shared__ double sStD[9];   // x, y, angle, vx, vy, progress, last_progress, last_steering, ep_return
  __shared__ double2 sCs;      // KIN -> REWARD: cos / sin of the stepped angle
  __shared__ int32_t sStI[3];  // finished_step, steps, ep_length
  __shared__ uint8_t sStB[2];  // flags, env_flags
  __shared__ float sObs[D];
  const rx_state& G = a.st;
  if (threadIdx.x == 0) {
    sStD[0] = G.x[pos], sStD[1] = G.y[pos], sStD[2] = G.angle[pos], sStD[3] = G.vx[pos], sStD[4] = G.vy[pos];
    sStD[5] = G.progress[pos], sStD[6] = G.last_progress[pos], sStD[7] = G.last_steering[pos];
    sStD[8] = G.ep_return[pos];
    sStI[0] = G.finished_step ? G.finished_step[pos] : -1;
    sStI[1] = G.steps[pos], sStI[2] = G.ep_length[pos];
    sStB[0] = G.flags[pos], sStB[1] = G.env_flags[pos];
  }
  __syncthreads();
  rx_kargs at = a;
  at.st.x = sStD + 0 - pos, at.st.y = sStD + 1 - pos, at.st.angle = sStD + 2 - pos, at.st.vx = sStD + 3 - pos;
  at.st.vy = sStD + 4 - pos, at.st.progress = sStD + 5 - pos, at.st.last_progress = sStD + 6 - pos;
  at.st.last_steering = sStD + 7 - pos, at.st.ep_return = sStD + 8 - pos;
  at.st.finished_step = G.finished_step ? sStI + 0 - pos : nullptr;
  at.st.steps = sStI + 1 - pos, at.st.ep_length = sStI + 2 - pos;
  at.st.flags = sStB + 0 - pos, at.st.env_flags = sStB + 1 - pos;
  at.cs_scratch = reinterpret_cast<double*>(&sCs) - 2 * (ptrdiff_t)pos;
  // next-step / no autoreset: the split step's KIN / REWARD halves (as k_kin1 /
  // k_step2), so the argmins and the reward run beside the 11 raycast waves
  const bool split = a.autoreset != RX_AUTORESET_SAME_STEP;
#ifdef RX_ROLL_STAMPS  // profiling build (tools/rollout_stamps.py): phase boundaries of workgroup 0
#define RX_RSTAMP(j) \
  if (b == 0 && (threadIdx.x & 63) == 0 && a.io.counters && t < 512) a.io.counters[16 + 16 * t + (j)] = wall_clock64()
#else
#define RX_RSTAMP(j)
#endif
  for (int t = 0; t < r.T; ++t) {
    if (w == 0) RX_RSTAMP(0);
    const bool last = t + 1 == r.T;
    const int64_t row = (int64_t)t * n + e;
    // ---- policy (k_policy_act's operations, one row): the trunk of tr on
    // sX[tr] (0 = actor, 1 = critic), then the heads
    auto trunk = [&](int tr) {
      // k_policy_act's MFMA chains (rx_ppo.hip): inputs d = 0 .. D-1 then the
      // zero padding to a multiple of 4; hidden units in the order t, r, q
      // (h = 16t + 4q + r)
      float z = 0.0f;
#pragma unroll
      for (int d = 0; d < D; ++d) z = fmaf(sW1[tr][d * H + lane], sX[tr][d], z);
#pragma unroll
      for (int d = D; d < (D + 3) / 4 * 4; ++d) z = fmaf(0.0f, 0.0f, z);
      sH1[tr][lane] = rx_policy::tanh_fast(z + sB[tr][0][lane]);
      wave_sync();
      z = 0.0f;
#pragma unroll 16
      for (int k = 0; k < H; ++k) {
        const int h = (k & ~15) + 4 * (k & 3) + ((k >> 2) & 3);  // k = 16t + 4r + q -> h = 16t + 4q + r
        z = fmaf(sW2[tr][h * H + lane], sH1[tr][h], z);
      }
      sH2[tr][lane] = rx_policy::tanh_fast(z + sB[tr][1][lane]);
      wave_sync();
    };
    auto actor_head = [&](float eps) {
      float lp = 0.0f;
      if (lane < NA) {
        const int j = lane;
        // k_policy_act's VALU head (rx_ppo.hip mlp_forward): 4 partial chains
        // over h = 16t + 4q + r in the order t, r, then (p0 + p1) + (p2 + p3)
        float pq[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          pq[q] = 0.0f;
#pragma unroll
          for (int k = 0; k < 16; ++k) {
            const int h = 16 * (k >> 2) + 4 * q + (k & 3);
            pq[q] = fmaf(sW3[j * H + h], sH2[0][h], pq[q]);
          }
        }
        const float zz = (pq[0] + pq[1]) + (pq[2] + pq[3]);
        const float mu = rx_policy::tanh_fast(zz + sK[j]);
        const float scale = sK[3 + j];
        const float var = scale * scale;
        const float smp = eps * scale + mu;  // mul_(std).add_(mu): two roundings
        const float act = fminf(fmaxf(smp, -1.0f), 1.0f);
        r.actions[row * NA + j] = act;
        reinterpret_cast<float*>(&sAct)[j] = act;
        lp = rx_policy::normal_logp(act - mu, var, sK[5 + j]);
      }
      const float lp1 = __shfl(lp, 1, 64);
      if (lane == 0) r.logprobs[row] = (0.0f + lp) + lp1;  // logp = 0; logp += lp_j in j order
    };
    auto critic_head = [&]() {
      if (lane != 0) return;
      float pq[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        pq[q] = 0.0f;
        for (int k = 0; k < 16; ++k) {
          const int h = 16 * (k >> 2) + 4 * q + (k & 3);
          pq[q] = fmaf(sW3c[h], sH2[1][h], pq[q]);
        }
      }
      const float v = (pq[0] + pq[1]) + (pq[2] + pq[3]);
      r.values[row] = v + sK[2];
    };
    auto load_obs = [&](int tr) {  // obs[t] of the env -> sX[tr]
      if (lane < D) sX[tr][lane] = t == 0 ? r.obs[row * D + lane] : sObs[lane];
      wave_sync();
    };
    at.io.actions = reinterpret_cast<const float*>(&sAct) - (ptrdiff_t)e * NA;  // actions[t] row e, from LDS
    at.io.obs = sObs - (ptrdiff_t)e * D;  // obs[t+1] row in LDS, copied out below
    at.io.reward = r.rewards + (size_t)t * n;
    at.io.done_f32 = last ? r.next_done : r.dones + (size_t)(t + 1) * n;
    double ang[1], ep[3] = {0.0, 0.0, 0.0};
    int ee = -1;
    if (split) {
      // RacingEnv.step as the split step: the actor, then KIN on wave 0 (KIN only
      // waits for the critic wave to have copied obs[t], since it overwrites the
      // non-ray columns of sObs); REWARD beside the raycast, and the critic's
      // trunk on wave 1 ahead of its ray (wave 1's ray ends first otherwise)
      if (w == 0) {
        const float eps = lane < NA ? r.eps[row * NA + lane] : 0.0f;  // in flight during the trunk
        load_obs(0);
        trunk(0);
        actor_head(eps);
        while (__hip_atomic_load(&sObsTaken, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) <= t)
          __builtin_amdgcn_s_sleep(1);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        RX_RSTAMP(1);
        dyn1_env<64, RX_PART_KIN>(at, b, ang, ee, ep, 0, &sl);
      } else if (w == 1) {
        load_obs(1);
        if (lane == 0) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          __hip_atomic_store(&sObsTaken, t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
      __syncthreads();  // stepped pose -> the raycast waves
      if (w == 0) RX_RSTAMP(2);
      if (w == 0) {
        dyn1_env<64, RX_PART_REWARD>(at, b, ang, ee, ep, 0, &sl);
        add_episode_stats(at, ep);
        RX_RSTAMP(4);
      } else {
        if (w == 1) {
          trunk(1);
          critic_head();
        }
        for (int ray = w - 1; ray < a.n_sensors; ray += kRollWaves - 1) ray_wide<1>(at, pos, ray, sl.seg);
        RX_RSTAMP(4 + w);  // ray waves 1 .. 11: slots 5 .. 15
      }
    } else {  // same-step autoreset: the policy, then the whole step (k_dyn1's order), then the rays
      if (w < 2) {
        const float eps = (w == 0 && lane < NA) ? r.eps[row * NA + lane] : 0.0f;
        load_obs(w);
        trunk(w);
        if (w == 0)
          actor_head(eps);
        else
          critic_head();
      }
      __syncthreads();  // actions[t] -> the dynamics wave
      if (w == 0) {
        dyn1_env<64, RX_PART_FULL>(at, b, ang, ee, ep, 0, &sl);
        add_episode_stats(at, ep);
      }
      __syncthreads();
      for (int ray = w; ray < a.n_sensors; ray += kRollWaves) ray_wide<1>(at, pos, ray, sl.seg);
    }
    __syncthreads();  // obs[t+1] complete before the next policy step
    if (w == 2 && lane < D) (last ? r.next_obs : r.obs + (size_t)(t + 1) * n * D)[(size_t)e * D + lane] = sObs[lane];
    if (w == 0) RX_RSTAMP(3);
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // the working state back to HBM
    G.x[pos] = sStD[0], G.y[pos] = sStD[1], G.angle[pos] = sStD[2], G.vx[pos] = sStD[3], G.vy[pos] = sStD[4];
    G.progress[pos] = sStD[5], G.last_progress[pos] = sStD[6], G.last_steering[pos] = sStD[7];
    G.ep_return[pos] = sStD[8];
    if (G.finished_step) G.finished_step[pos] = sStI[0];
    G.steps[pos] = sStI[1], G.ep_length[pos] = sStI[2];
    G.flags[pos] = sStB[0], G.env_flags[pos] = sStB[1];
  }
}

// ============================================================ GAE
// PPO.compute_advantages, agent/ppo.py:134-154: float32, no FMA, lane = env.
__global__ __launch_bounds__(256) void k_gae(int T, int N, const float* __restrict__ r, const float* __restrict__ v,
                                             const float* __restrict__ d, const float* __restrict__ nv,
                                             const float* __restrict__ nd, float g, float gl,
                                             float* __restrict__ adv, float* __restrict__ ret) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float run = 0.0f;
  float nnt = 1.0f - nd[n];
  float nvv = nv[n];
#pragma unroll 8
  for (int t = T - 1; t >= 0; --t) {
    const size_t o = (size_t)t * N + n;
    const float vt = v[o];
    const float delta = (r[o] + (g * nnt) * nvv) - vt;
    run = delta + (gl * nnt) * run;
    adv[o] = run;
    ret[o] = run + vt;
    nnt = 1.0f - d[o];
    nvv = vt;
  }
}

// Wavefront-prefix variant: one wave per env; lane l owns the time chunk
// [l*L, (l+1)*L).  Pass 1: each lane composes its chunk's affine map
// A_in = alpha + beta * A_out (backwards).  Pass 2: a 64-lane suffix scan of
// the maps gives every lane its incoming A_out.  Pass 3: the chunk is replayed
// with the reference recurrence from that carry-in.
__global__ __launch_bounds__(256) void k_gae_scan(int T, int N, const float* __restrict__ r,
                                                  const float* __restrict__ v, const float* __restrict__ d,
                                                  const float* __restrict__ nv, const float* __restrict__ nd, float g,
                                                  float gl, float* __restrict__ adv, float* __restrict__ ret) {
  const int n = uniform(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (n >= N) return;
  const int lane = threadIdx.x & 63;
  const int L = (T + 63) / 64;
  const int t0 = lane * L;
  const int t1 = min(T, t0 + L);
  auto nnt_at = [&](int t) -> float {  // next_nonterminal used at time t
    return (t == T - 1) ? 1.0f - nd[n] : 1.0f - d[(size_t)(t + 1) * N + n];
  };
  auto nv_at = [&](int t) -> float { return (t == T - 1) ? nv[n] : v[(size_t)(t + 1) * N + n]; };
  float alpha = 0.0f, beta = 1.0f;
  for (int t = t1 - 1; t >= t0; --t) {
    const size_t o = (size_t)t * N + n;
    const float nnt = nnt_at(t);
    const float delta = (r[o] + (g * nnt) * nv_at(t)) - v[o];
    const float c = gl * nnt;
    alpha = delta + c * alpha;
    beta = c * beta;
  }
  // inclusive suffix scan of maps: S_l = M_l o M_{l+1} o ... o M_63
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const float ao = __shfl_down(alpha, off, 64);
    const float bo = __shfl_down(beta, off, 64);
    if (lane + off < 64) {
      alpha = alpha + beta * ao;
      beta = beta * bo;
    }
  }
  float carry = __shfl_down(alpha, 1, 64);  // A_out(l) = S_{l+1}(0)
  if (lane == 63) carry = 0.0f;
  float run = carry;
  for (int t = t1 - 1; t >= t0; --t) {
    const size_t o = (size_t)t * N + n;
    const float nnt = nnt_at(t);
    const float vt = v[o];
    const float delta = (r[o] + (g * nnt) * nv_at(t)) - vt;
    run = delta + (gl * nnt) * run;
    adv[o] = run;
    ret[o] = run + vt;
  }
}

}  // namespace

// ------------------------------------------------------------ launchers
// dynamic LDS of k_dyn1 / k_dyn2 (k_kin1 / k_kin2): per wave the sort's sector
// counters and its staging row of 64 x 16 A task ids, only when the launch sorts
static size_t task_sort_lds_bytes(const rx_kargs* a, int n_agents, int waves_per_wg) {
  if (!a->tasks_out) return 0;
  return (size_t)waves_per_wg * (kTaskSectors + 64 * 16 * n_agents) * sizeof(int32_t);
}
// k_step2<A, RLPE, LPR> for the handle's schedule (a->reward_lpe, a->ray_lpr:
// 1, 2 or 4 each, validated by rx_assign)
template <int A, int RLPE>
static void launch_step2_lpr(const rx_kargs* a, dim3 grid, int n_rw, hipStream_t s) {
  if (a->ray_lpr == 4)
    hipLaunchKernelGGL((k_step2<A, RLPE, 4>), grid, dim3(64), 0, s, *a, n_rw);
  else if (a->ray_lpr == 2)
    hipLaunchKernelGGL((k_step2<A, RLPE, 2>), grid, dim3(64), 0, s, *a, n_rw);
  else
    hipLaunchKernelGGL((k_step2<A, RLPE, 1>), grid, dim3(64), 0, s, *a, n_rw);
}

extern "C" int rx_launch_split(const rx_kargs* a, int n_agents, int part, hipStream_t s) {
  if (n_agents == 2) {  // k_kin2, then k_step2<2> (REWARD waves padded to 8, as below)
    const int n_rw2 = a->reward_lpe * ((a->n_dyn_waves + 7) / 8 * 8);
    if (part == RX_SPLIT_KIN) {
      hipLaunchKernelGGL((k_dyn2<RX_PART_KIN>), dim3(a->n_dyn_waves), dim3(64), task_sort_lds_bytes(a, 2, 1), s, *a);
    } else {
      const dim3 grid(n_rw2 + (part == RX_SPLIT_REWARD ? 0 : a->n_ray_waves));
      if (a->reward_lpe == 2)
        launch_step2_lpr<2, 2>(a, grid, n_rw2, s);
      else
        launch_step2_lpr<2, 1>(a, grid, n_rw2, s);
    }
    return (int)hipGetLastError();
  }
  const int n_rw = a->reward_lpe * ((a->n_dyn_waves + 7) / 8 * 8);
  if (a->lane_tracks) {  // lane-varying slots (rx_assign: one lane per env and per ray, no task sort)
    if (part == RX_SPLIT_KIN)
      hipLaunchKernelGGL((k_dyn1<1, RX_PART_KIN, true>), dim3(a->n_dyn_waves), dim3(64), 0, s, *a);
    else
      hipLaunchKernelGGL((k_step2<1, 1, 1, true>), dim3(n_rw + (part == RX_SPLIT_REWARD ? 0 : a->n_ray_waves)),
                         dim3(64), 0, s, *a, n_rw);
    return (int)hipGetLastError();
  }
  if (part == RX_SPLIT_KIN) {
    // one wave per workgroup: block b's k_kin1 wave lands on XCD b % 8, the XCD of
    // block b's REWARD and raycast waves in k_step2, so they read its stores from one L2
    hipLaunchKernelGGL((k_dyn1<1, RX_PART_KIN>), dim3(a->n_dyn_waves), dim3(64), task_sort_lds_bytes(a, 1, 1), s, *a);
    return (int)hipGetLastError();
  }
  // RX_SPLIT_REWARD: the REWARD half alone; RX_SPLIT_REWARD_RAYS: both halves in one launch
  const dim3 grid(n_rw + (part == RX_SPLIT_REWARD ? 0 : a->n_ray_waves));
  if (a->reward_lpe == 4)
    launch_step2_lpr<1, 4>(a, grid, n_rw, s);
  else if (a->reward_lpe == 2)
    launch_step2_lpr<1, 2>(a, grid, n_rw, s);
  else
    launch_step2_lpr<1, 1>(a, grid, n_rw, s);
  return (int)hipGetLastError();
}

extern "C" int rx_launch_step(const rx_kargs* a, int n_agents, int phases, hipStream_t s) {
  const dim3 blk(256);
  if ((phases & RX_PHASE_DYNAMICS) && a->n_dyn_waves > 0) {
    const dim3 grd((a->n_dyn_waves + 3) / 4);
    const size_t lds = task_sort_lds_bytes(a, n_agents, 4);
    if (n_agents == 1 && a->lane_tracks)
      hipLaunchKernelGGL((k_dyn1<1, RX_PART_FULL, true>), grd, blk, 0, s, *a);
    else if (n_agents == 1 && a->dyn_lpe == 64)
      hipLaunchKernelGGL((k_dyn1<64, RX_PART_FULL>), grd, blk, lds, s, *a);
    else if (n_agents == 1 && a->dyn_lpe == 4)
      hipLaunchKernelGGL((k_dyn1<4, RX_PART_FULL>), grd, blk, lds, s, *a);
    else if (n_agents == 1 && a->dyn_lpe == 2)
      hipLaunchKernelGGL((k_dyn1<2, RX_PART_FULL>), grd, blk, lds, s, *a);
    else if (n_agents == 1)
      hipLaunchKernelGGL((k_dyn1<1, RX_PART_FULL>), grd, blk, lds, s, *a);
    else
      hipLaunchKernelGGL((k_dyn2<RX_PART_FULL>), grd, blk, lds, s, *a);
  }
  if ((phases & RX_PHASE_RAYS) && a->wide) {
    const dim3 wg((a->n_wide_tasks + 3) / 4);
    if (n_agents == 1)
      hipLaunchKernelGGL(k_rays_wide<1>, wg, blk, 0, s, *a);
    else
      hipLaunchKernelGGL(k_rays_wide<2>, wg, blk, 0, s, *a);
  } else if ((phases & RX_PHASE_RAYS) && a->n_ray_waves > 0) {
    // one wave per workgroup: finer-grained dispatch fills the tail, and the XCD
    // placement of rx_assign's ray-wave order holds per wave
    if (n_agents == 1 && a->lane_tracks)
      hipLaunchKernelGGL((k_rays<1, true>), dim3(a->n_ray_waves), dim3(64), 0, s, *a);
    else if (n_agents == 1)
      hipLaunchKernelGGL(k_rays<1>, dim3(a->n_ray_waves), dim3(64), 0, s, *a);
    else
      hipLaunchKernelGGL(k_rays<2>, dim3(a->n_ray_waves), dim3(64), 0, s, *a);
  }
  return (int)hipGetLastError();
}

extern "C" int rx_launch_rollout(const rx_kargs* a, const rx_rollout_io* r, int max_w, hipStream_t s) {
  const size_t lds = (size_t)max_w * (2 * sizeof(double4) + 2 * sizeof(double2));  // one slot, staged
  if (r->obs_dim == 15)
    hipLaunchKernelGGL(k_rollout<15>, dim3(a->n_dyn_waves), dim3(64 * kRollWaves), lds, s, *a, *r);
  else
    hipLaunchKernelGGL(k_rollout<19>, dim3(a->n_dyn_waves), dim3(64 * kRollWaves), lds, s, *a, *r);
  return (int)hipGetLastError();
}

// Self-play rollout (rx_selfplay_rollout_steps): agent q's observation row and
// reward out of a two-car handle's [N][2][D] / [N][2] step outputs into the
// rollout's [N][D] / [N] rows.  Lane = one float.
__global__ __launch_bounds__(256) void k_agent_rows(int N, int D, int q, const float* __restrict__ obs,
                                                    const float* __restrict__ rew, float* __restrict__ obs_out,
                                                    float* __restrict__ rew_out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < N * D) {
    const int e = i / D, d = i - e * D;
    obs_out[i] = obs[(size_t)(2 * e + q) * D + d];
  }
  if (i < N) rew_out[i] = rew[2 * i + q];
}

// k_reset_rank (rx_set_start_draws): one workgroup.  Pass 1 lays the reset flags
// out in env order (RX_MODE_STEP: a working-state row's next-step autoreset flag
// goes to its env perm[p]); pass 2 ranks them -- thread t counts a contiguous run
// of envs, an LDS scan over the 1,024 counts gives each run's offset -- so the
// j-th resetting env in env order gets rank j, as the reference's SyncVectorEnv
// loop draws them.  Thread 0 hands the launch its base and advances the cursor.
__global__ __launch_bounds__(1024) void k_reset_rank(int N, int mode, const uint8_t* __restrict__ mask,
                                                     const uint8_t* __restrict__ env_flags,
                                                     const int32_t* __restrict__ perm, int32_t* __restrict__ tmp,
                                                     int32_t* __restrict__ rank, int64_t* cursor, int64_t* base,
                                                     int64_t n_draws) {
  __shared__ int32_t cnt[1024];
  const int t = threadIdx.x;
  if (mode == RX_MODE_RESET) {
    for (int e = t; e < N; e += 1024) tmp[e] = mask ? (mask[e] != 0) : 1;
  } else {
    for (int p = t; p < N; p += 1024) tmp[perm[p]] = (env_flags[p] & RX_EF_PENDING_RESET) != 0;
  }
  __syncthreads();
  const int run = (N + 1023) / 1024, e0 = t * run, e1 = min(N, e0 + run);
  int c = 0;
  for (int e = e0; e < e1; ++e) c += tmp[e];
  cnt[t] = c;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {  // inclusive Hillis-Steele scan
    const int v = t >= o ? cnt[t - o] : 0;
    __syncthreads();
    cnt[t] += v;
    __syncthreads();
  }
  int r = cnt[t] - c;
  for (int e = e0; e < e1; ++e) {
    const int f = tmp[e];
    rank[e] = f ? r : -1;
    r += f;
  }
  if (t == 1023) {
    const int64_t b = cursor[0], total = cnt[1023];
    *base = b;
    cursor[0] = b + total;
    if (b + total > n_draws) cursor[1] += b + total - max(b, n_draws);
  }
}

extern "C" int rx_launch_reset_rank(int N, int mode, const uint8_t* mask, const uint8_t* env_flags, const int32_t* perm,
                                    int32_t* tmp, int32_t* rank, int64_t* cursor, int64_t* base, int64_t n_draws,
                                    hipStream_t s) {
  hipLaunchKernelGGL(k_reset_rank, dim3(1), dim3(1024), 0, s, N, mode, mask, env_flags, perm, tmp, rank, cursor, base,
                     n_draws);
  return (int)hipGetLastError();
}

extern "C" int rx_launch_agent_rows(int N, int D, int q, const float* obs, const float* rew, float* obs_out,
                                    float* rew_out, hipStream_t s) {
  const int n = N * D > N ? N * D : N;
  hipLaunchKernelGGL(k_agent_rows, dim3((n + 255) / 256), dim3(256), 0, s, N, D, q, obs, rew, obs_out, rew_out);
  return (int)hipGetLastError();
}

extern "C" int rx_launch_gae(int T, int N, const float* r, const float* v, const float* d, const float* nv,
                             const float* nd, float g, float gl, float* adv, float* ret, int scan, hipStream_t s) {
  if (scan) {
    hipLaunchKernelGGL(k_gae_scan, dim3((N + 3) / 4), dim3(256), 0, s, T, N, r, v, d, nv, nd, g, gl, adv, ret);
  } else {
    hipLaunchKernelGGL(k_gae, dim3((N + 255) / 256), dim3(256), 0, s, T, N, r, v, d, nv, nd, g, gl, adv, ret);
  }
  return (int)hipGetLastError();
}
