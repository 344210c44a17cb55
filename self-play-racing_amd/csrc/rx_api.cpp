// rx_api.cpp -- C ABI (include/rx.h): handle lifetime, argument validation,
// track-table upload, env->wavefront grouping, launches.
//
// Everything that allocates or copies synchronously (rx_upload_tracks,
// rx_assign) happens outside the step path; rx_reset / rx_step / rx_gae only
// enqueue kernels on the caller's stream, so they can be graph-captured.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <type_traits>
#include <string>
#include <vector>

#include "rx.h"
#include "rx_internal.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define RX_HIP(call)                                                                      \
  do {                                                                                    \
    hipError_t e_ = (call);                                                               \
    if (e_ != hipSuccess) return fail(RX_EHIP, "%s: %s", #call, hipGetErrorString(e_)); \
  } while (0)

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

template <class T>
int upload(DevBuf<T>& b, const T* host, size_t n) {
  if (n > b.n) {
    b.release();
    if (hipMalloc(&b.p, std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess) {
      b.p = nullptr;
      return fail(RX_ENOMEM, "hipMalloc(%zu bytes) failed", n * sizeof(T));
    }
    b.n = n;
  }
  if (n) RX_HIP(hipMemcpy(b.p, host, n * sizeof(T), hipMemcpyHostToDevice));
  return RX_OK;
}

}  // namespace

struct rx_env {
  rx_config cfg{};
  int D = 0;
  // track table
  int32_t n_tracks = 0;
  std::vector<int32_t> wp_off_h;
  DevBuf<int32_t> wp_off;
  DevBuf<double> wp, nrm, seg, meta;
  // raycast culling tables (derived from the track table)
  DevBuf<int32_t> chunk_off;
  DevBuf<double> chunk_box, slot_geo, wchunk_box;
  DevBuf<int32_t> wchunk_off;
  DevBuf<int32_t> super_off;  // two-level culling: super-chunk boxes per slot
  DevBuf<double> super_box;
  DevBuf<int32_t> wsuper_off;  // two-level closest-waypoint culling
  DevBuf<double> wsuper_box;
  DevBuf<float> chunk_box_f, super_box_f;  // outward-rounded float32 copies (raycast box tests) + 4 quadrant blocks
  int32_t n_chunk_boxes = 0, n_super_boxes = 0;
  DevBuf<float> seg_f;  // [2*Wtot][4] float32 (start.x, start.y, v2.x, v2.y): the raycast's segment pre-filter
  DevBuf<rx_slot_hdr> slot_hdr;  // [n] per-slot headers (lane-varying kernels)
  // assignment
  bool assigned = false;
  DevBuf<int32_t> perm[2];  // the env order (perm[0]: env id at each position) and the re-sort's shadow
  DevBuf<rx_wave> dyn_waves, ray_waves;
  std::vector<rx_wave> ray_waves_h;  // host copy of the ray-wave table (rx_ray_waves)
  DevBuf<int32_t> slot_n;   // envs per slot (ray-major decode)
  DevBuf<uint32_t> resets;  // per-env reset count: keys the 2-car start-slot draw (graph-replay safe)
  // rx_set_start_draws: the caller's MT19937 outputs and cursor; ranks of the resetting envs
  const uint32_t* draws = nullptr;
  int64_t n_draws = 0;
  int64_t* draw_cursor = nullptr;
  DevBuf<int32_t> draw_rank, draw_tmp;
  DevBuf<int64_t> draw_base;
  int32_t n_dyn_waves = 0, n_ray_waves = 0;
  int32_t dyn_lpe = 1;
  int32_t ray_lpr = 1;  // lanes per ray task (ray_order 2, not wide): 64 / ray_lpr tasks a ray wave
  int32_t reward_lpe = 1;  // split step, single-agent: lanes per env in k_step2's REWARD half
  int32_t argmin_window = 2;
  int32_t ray_dispatch = RX_RAY_DISPATCH;  // resolved class order of the ray-wave table (rx_config.ray_dispatch)
  int32_t ray_tail = 0, ray_tail_lpr = 2;  // tail classes cast at ray_tail_lpr lanes per ray (0 = none)
  int32_t task_sort = 1;                   // ray-task direction sort every task_sort dynamics launches
  int32_t lane_tracks = 0;                 // lane-varying slots (rx_config.lane_tracks, rx_assign's choice)
  DevBuf<int32_t> pos_slot;                // with lane_tracks: [N] slot of the env at each position
  DevBuf<uint8_t> policy_frag;  // the bf16 rollout's operand fragments of both trunks (k_policy_frag, rx_rollout_steps)
  int32_t ray_tail_from = -1;              // first ray wave of the tail (-1 = none)
  DevBuf<double> rel_angles;
  std::vector<double> rel_angles_h;
  // spatial sort (scheduling only)
  DevBuf<uint32_t> keys_in;              // [N] bin per perm position (REWARD half)
  DevBuf<uint32_t> keys_off;             // [N] the position's rank within its bin (the count's atomic)
  bool sort_pending = false;             // keys written, the re-sort runs after this step's raycast
  bool sort_hist_done = false;           // the REWARD half of the keys' launch also counted the bins
  DevBuf<uint32_t> sort_hist, sort_cursor;  // [sort_bins]
  DevBuf<int32_t> sort_base;             // [n_tracks] first bin of each slot
  int32_t sort_bins = 0, sort_shift = 0;
  bool sort_on = false;
  uint64_t dyn_calls = 0;
  // ray-task direction sort (ray_order 2): every RX_TASK_SORT_INTERVAL dynamics
  // launches, and always on the first launch after a block's membership changed
  bool tasks_stale = true;
  uint64_t task_calls = 0;
  // ray_order 2: direction-sorted (agent, ray) task ids, rewritten by k_dyn every step
  DevBuf<int32_t> tasks;
  // split step (k_kin1 + k_step2): cos / sin of the stepped angles; RX_SPLIT=0 disables
  DevBuf<double> cs_scratch;
  bool split = true;
  // rx_profile: per recorded launch, [RX_PROF_SLOTS] wave start + [RX_PROF_SLOTS] wave end stamps
  bool prof = false;
  DevBuf<unsigned long long> prof_buf;
  std::vector<int> prof_kinds;
  // state: the caller's arrays (env order, rx_bind_state) and the engine's
  // working copy in wave order (position p = env perm[p]; the kernels read and
  // write it coalesced) plus the shadow the re-sort moves rows into
  bool bound = false;
  rx_state st{};
  rx_state work{}, work_tmp{};
  std::vector<void*> work_mem;
};

namespace {
// Culling tables for every slot: chunks of G consecutive boundary segments
// (per side), their end-point boxes, and per slot the bounding circle of all
// boundary points and the longest segment (kernel margins).
int build_headers(rx_env* h, int32_t n_tracks, const int32_t* wp_off, const double* meta,
                  const std::vector<int32_t>& off, const std::vector<int32_t>& soff, const std::vector<int32_t>& woff,
                  const std::vector<int32_t>& wsoff, const std::vector<double>& geo);
int build_chunks(rx_env* h, int32_t n_tracks, const int32_t* wp_off, const double* wp, const double* seg,
                 const double* meta) {
  const int G = h->cfg.cull_chunk;
  if (G <= 0) return build_headers(h, n_tracks, wp_off, meta, {}, {}, {}, {}, {});
  const int SG = h->cfg.cull_super;  // leaves per super-chunk (0 = one level)
  std::vector<int32_t> off(n_tracks + 1, 0), woff(n_tracks + 1, 0), soff(n_tracks + 1, 0), wsoff(n_tracks + 1, 0);
  std::vector<double> boxes, wboxes, sboxes, wsboxes, geo(4 * (size_t)n_tracks);
  for (int k = 0; k < n_tracks; ++k) {
    const int W = wp_off[k + 1] - wp_off[k];
    const int nch = (W + G - 1) / G;
    const double* s = seg + 8 * (size_t)wp_off[k];  // 2W segments x 4
    double xmin = 1e300, ymin = 1e300, xmax = -1e300, ymax = -1e300, L = 0.0;
    for (int j = 0; j < 2 * W; ++j) {
      const double* g = s + 4 * j;
      const double ex = g[0] + g[2], ey = g[1] + g[3];
      xmin = std::min({xmin, g[0], ex});
      xmax = std::max({xmax, g[0], ex});
      ymin = std::min({ymin, g[1], ey});
      ymax = std::max({ymax, g[1], ey});
      L = std::max(L, std::sqrt(g[2] * g[2] + g[3] * g[3]));
    }
    const double cx = 0.5 * (xmin + xmax), cy = 0.5 * (ymin + ymax);
    double rad = 0.0;
    for (int j = 0; j < 2 * W; ++j) {
      const double* g = s + 4 * j;
      const double ex = g[0] + g[2], ey = g[1] + g[3];
      rad = std::max({rad, std::hypot(g[0] - cx, g[1] - cy), std::hypot(ex - cx, ey - cy)});
    }
    geo[4 * k + 0] = cx;
    geo[4 * k + 1] = cy;
    geo[4 * k + 2] = rad * (1.0 + 1e-12) + 1e-9;  // round up: the kernel needs an upper bound
    geo[4 * k + 3] = L * (1.0 + 1e-12) + 1e-12;
    for (int side = 0; side < 2; ++side) {
      for (int c = 0; c < nch; ++c) {
        double bx0 = 1e300, by0 = 1e300, bx1 = -1e300, by1 = -1e300;
        for (int j = side * W + c * G; j < side * W + std::min(W, (c + 1) * G); ++j) {
          const double* g = s + 4 * j;
          const double ex = g[0] + g[2], ey = g[1] + g[3];
          bx0 = std::min({bx0, g[0], ex});
          bx1 = std::max({bx1, g[0], ex});
          by0 = std::min({by0, g[1], ey});
          by1 = std::max({by1, g[1], ey});
        }
        boxes.insert(boxes.end(), {bx0, by0, bx1, by1});
      }
    }
    off[k + 1] = off[k] + 2 * nch;
    if (SG > 0) {  // super-chunk boxes: union of SG consecutive leaf boxes, per side
      const int nsup = (nch + SG - 1) / SG;
      const double* lb = boxes.data() + 4 * (size_t)off[k];
      for (int side = 0; side < 2; ++side)
        for (int u = 0; u < nsup; ++u) {
          double bx0 = 1e300, by0 = 1e300, bx1 = -1e300, by1 = -1e300;
          for (int c = u * SG; c < std::min(nch, (u + 1) * SG); ++c) {
            const double* b = lb + 4 * (side * nch + c);
            bx0 = std::min(bx0, b[0]);
            by0 = std::min(by0, b[1]);
            bx1 = std::max(bx1, b[2]);
            by1 = std::max(by1, b[3]);
          }
          sboxes.insert(sboxes.end(), {bx0, by0, bx1, by1});
        }
      soff[k + 1] = soff[k] + 2 * nsup;
    }
    // waypoint chunks (argmin culling): RX_WP_CHUNK consecutive waypoints each
    const double* w = wp + 2 * (size_t)wp_off[k];
    const int nwc = (W + RX_WP_CHUNK - 1) / RX_WP_CHUNK;
    for (int c = 0; c < nwc; ++c) {
      double bx0 = 1e300, by0 = 1e300, bx1 = -1e300, by1 = -1e300;
      for (int i = c * RX_WP_CHUNK; i < std::min(W, (c + 1) * RX_WP_CHUNK); ++i) {
        bx0 = std::min(bx0, w[2 * i]);
        bx1 = std::max(bx1, w[2 * i]);
        by0 = std::min(by0, w[2 * i + 1]);
        by1 = std::max(by1, w[2 * i + 1]);
      }
      wboxes.insert(wboxes.end(), {bx0, by0, bx1, by1});
    }
    woff[k + 1] = woff[k] + nwc;
    const int nws = (nwc + RX_WP_SUPER - 1) / RX_WP_SUPER;
    for (int u = 0; u < nws; ++u) {
      double bx0 = 1e300, by0 = 1e300, bx1 = -1e300, by1 = -1e300;
      for (int c = u * RX_WP_SUPER; c < std::min(nwc, (u + 1) * RX_WP_SUPER); ++c) {
        const double* b = wboxes.data() + 4 * ((size_t)woff[k] + c);
        bx0 = std::min(bx0, b[0]);
        by0 = std::min(by0, b[1]);
        bx1 = std::max(bx1, b[2]);
        by1 = std::max(by1, b[3]);
      }
      wsboxes.insert(wsboxes.end(), {bx0, by0, bx1, by1});
    }
    wsoff[k + 1] = wsoff[k] + nws;
  }
  // float32 copies rounded outward (min corner down, max corner up): each f32
  // box contains its f64 box, so a test that keeps the f32 box keeps the f64 one
  auto to_f32 = [](const std::vector<double>& b) {
    std::vector<float> f(b.size());
    for (size_t i = 0; i < b.size(); ++i) {
      float v = (float)b[i];
      if ((i & 3) < 2 && (double)v > b[i]) v = std::nextafter(v, -HUGE_VALF);
      if ((i & 3) >= 2 && (double)v < b[i]) v = std::nextafter(v, HUGE_VALF);
      f[i] = v;
    }
    return f;
  };
  // then 4 quadrant-ordered copies: block q = (near.x, near.y, far.x, far.y) for
  // a ray direction whose x (bit 0) / y (bit 1) component is negative -- the
  // slab planes k_rays' single-quadrant waves enter and leave through
  auto with_quadrants = [](std::vector<float> f) {
    const size_t n = f.size();
    f.resize(5 * n);
    for (int q = 0; q < 4; ++q)
      for (size_t i = 0; i < n; i += 4) {
        float* o = f.data() + (q + 1) * n + i;
        const float* b = f.data() + i;
        o[0] = (q & 1) ? b[2] : b[0];
        o[1] = (q & 2) ? b[3] : b[1];
        o[2] = (q & 1) ? b[0] : b[2];
        o[3] = (q & 2) ? b[1] : b[3];
      }
    return f;
  };
  const std::vector<float> boxes_f = with_quadrants(to_f32(boxes)), sboxes_f = with_quadrants(to_f32(sboxes));
  h->n_chunk_boxes = (int32_t)(boxes.size() / 4);
  h->n_super_boxes = (int32_t)(sboxes.size() / 4);
  int rc;
  if ((rc = upload(h->chunk_box_f, boxes_f.data(), boxes_f.size()))) return rc;
  if (SG > 0 && (rc = upload(h->super_box_f, sboxes_f.data(), sboxes_f.size()))) return rc;
  if ((rc = upload(h->chunk_off, off.data(), off.size()))) return rc;
  if ((rc = upload(h->chunk_box, boxes.data(), boxes.size()))) return rc;
  if ((rc = upload(h->slot_geo, geo.data(), geo.size()))) return rc;
  if ((rc = upload(h->wchunk_off, woff.data(), woff.size()))) return rc;
  if ((rc = upload(h->wchunk_box, wboxes.data(), wboxes.size()))) return rc;
  if ((rc = upload(h->wsuper_off, wsoff.data(), wsoff.size()))) return rc;
  if ((rc = upload(h->wsuper_box, wsboxes.data(), wsboxes.size()))) return rc;
  if (SG > 0) {
    if ((rc = upload(h->super_off, soff.data(), soff.size()))) return rc;
    if ((rc = upload(h->super_box, sboxes.data(), sboxes.size()))) return rc;
  }
  return build_headers(h, n_tracks, wp_off, meta, off, soff, woff, wsoff, geo);
}

// The per-slot headers (rx_slot_hdr) from the host tables rx_upload_tracks and
// build_chunks produced.
int build_headers(rx_env* h, int32_t n_tracks, const int32_t* wp_off, const double* meta,
                  const std::vector<int32_t>& off, const std::vector<int32_t>& soff, const std::vector<int32_t>& woff,
                  const std::vector<int32_t>& wsoff, const std::vector<double>& geo) {
  std::vector<rx_slot_hdr> hd((size_t)n_tracks);
  for (int k = 0; k < n_tracks; ++k) {
    rx_slot_hdr& r = hd[k];
    r.wp0 = wp_off[k];
    r.W = wp_off[k + 1] - wp_off[k];
    r.chunk_off = off.empty() ? 0 : off[k];
    r.super_off = soff.empty() ? 0 : soff[k];
    r.wchunk_off = woff.empty() ? 0 : woff[k];
    r.wsuper_off = wsoff.empty() ? 0 : wsoff[k];
    r.pad0 = r.pad1 = 0;
    for (int i = 0; i < 4; ++i) r.geo[i] = geo.empty() ? 0.0 : geo[4 * (size_t)k + i];
    for (int i = 0; i < 8; ++i) r.meta[i] = meta[8 * (size_t)k + i];
  }
  return upload(h->slot_hdr, hd.data(), hd.size());
}
}  // namespace

extern "C" {

const char* rx_last_error(void) { return g_err.c_str(); }
int rx_abi_version(void) { return RX_ABI_VERSION; }

int rx_create(const rx_config* cfg, rx_env** out) {
  if (!cfg || !out) return fail(RX_EINVAL, "rx_create: null argument");
  *out = nullptr;
  if (cfg->n_envs <= 0) return fail(RX_EINVAL, "n_envs must be > 0 (got %d)", cfg->n_envs);
  if (cfg->n_agents != 1 && cfg->n_agents != 2) return fail(RX_EINVAL, "n_agents must be 1 or 2 (got %d)", cfg->n_agents);
  if (cfg->n_sensors <= 0 || cfg->n_sensors > 256) return fail(RX_EINVAL, "n_sensors out of range (%d)", cfg->n_sensors);
  if (cfg->max_steps <= 0) return fail(RX_EINVAL, "max_steps must be > 0");
  if (cfg->ray_order < 0 || cfg->ray_order > 2)
    return fail(RX_EINVAL, "ray_order must be 0, 1 or 2 (got %d)", cfg->ray_order);
  if (cfg->cull_super < 0 || cfg->cull_super > 64) return fail(RX_EINVAL, "cull_super out of range (%d)", cfg->cull_super);
  if (cfg->autoreset < RX_AUTORESET_NEXT_STEP || cfg->autoreset > RX_AUTORESET_DISABLED)
    return fail(RX_EINVAL, "bad autoreset mode %d", cfg->autoreset);
  // launch schedule (ABI v17): 0 = auto, -1 = off where there is an off state
  auto tri = [](int32_t v) { return v == 0 || v == 1 || v == -1; };
  auto lanes = [](int32_t v, bool wide) { return v == 0 || v == 1 || v == 2 || v == 4 || (wide && v == 64); };
  if (!tri(cfg->split)) return fail(RX_EINVAL, "split must be 0 (auto), 1 or -1 (got %d)", cfg->split);
  if (!tri(cfg->seg_filter)) return fail(RX_EINVAL, "seg_filter must be 0 (auto), 1 or -1 (got %d)", cfg->seg_filter);
  if (!tri(cfg->box_quadrants))
    return fail(RX_EINVAL, "box_quadrants must be 0 (auto), 1 or -1 (got %d)", cfg->box_quadrants);
  if (cfg->wide_n < -1) return fail(RX_EINVAL, "wide_n must be >= -1 (got %d)", cfg->wide_n);
  if (!lanes(cfg->dyn_lpe, true)) return fail(RX_EINVAL, "dyn_lpe must be 0 (auto), 1, 2, 4 or 64 (got %d)", cfg->dyn_lpe);
  if (!lanes(cfg->ray_lpr, false)) return fail(RX_EINVAL, "ray_lpr must be 0 (auto), 1, 2 or 4 (got %d)", cfg->ray_lpr);
  if (!lanes(cfg->reward_lpe, false))
    return fail(RX_EINVAL, "reward_lpe must be 0 (auto), 1, 2 or 4 (got %d)", cfg->reward_lpe);
  if (cfg->argmin_window < -1 || cfg->argmin_window > 32)
    return fail(RX_EINVAL, "argmin_window must be 0 (auto), -1 (none) or 1 .. 32 (got %d)", cfg->argmin_window);
  if (cfg->ray_dispatch < -1 || cfg->ray_dispatch > 3)
    return fail(RX_EINVAL, "ray_dispatch must be 0 (auto), -1, 1, 2 or 3 (got %d)", cfg->ray_dispatch);
  if (cfg->ray_tail < -1 || cfg->ray_tail > 16)
    return fail(RX_EINVAL, "ray_tail must be 0 (auto), -1 (none) or 1 .. 16 (got %d)", cfg->ray_tail);
  if (cfg->ray_tail_lpr != 0 && cfg->ray_tail_lpr != 2 && cfg->ray_tail_lpr != 4)
    return fail(RX_EINVAL, "ray_tail_lpr must be 0 (auto), 2 or 4 (got %d)", cfg->ray_tail_lpr);
  if (cfg->lane_tracks < -1 || cfg->lane_tracks > 1)
    return fail(RX_EINVAL, "lane_tracks must be 0 (auto), 1 or -1 (got %d)", cfg->lane_tracks);
  if (cfg->reserved0 != 0)
    return fail(RX_EINVAL, "reserved0 must be 0 (ABI v23 dropped the kin_sort schedule; got %d)", cfg->reserved0);
  if (cfg->task_sort < 0 || cfg->task_sort > 16)
    return fail(RX_EINVAL, "task_sort must be 0 (auto) or 1 .. 16 (got %d)", cfg->task_sort);
  if (cfg->n_agents == 2 && (cfg->dyn_lpe > 1 || cfg->reward_lpe > 2))
    return fail(RX_EINVAL, "n_agents = 2: dyn_lpe > 1 is a single-agent schedule, and reward_lpe is 1 or 2 "
                           "(a lane per car)");
  if ((long long)cfg->n_envs * cfg->n_agents * cfg->n_sensors > 0x7fffffffLL)
    return fail(RX_EINVAL, "n_envs * n_agents * n_sensors overflows int32");
  int ndev = 0;
  RX_HIP(hipGetDeviceCount(&ndev));
  if (cfg->device < 0 || cfg->device >= ndev) return fail(RX_EINVAL, "device %d not present (%d devices)", cfg->device, ndev);
  RX_HIP(hipSetDevice(cfg->device));
  rx_env* h = new rx_env();
  h->cfg = *cfg;
  if (!(h->cfg.speed_weight == h->cfg.speed_weight)) h->cfg.speed_weight = 8.0;
  h->D = cfg->n_sensors + 4 + 4 * (cfg->n_agents - 1);
  // sensor angles = np.linspace(-c, c, n) (racing_env.py:45, multi_racing_env.py:50):
  // numpy computes start + i*step with step = (stop-start)/(n-1), and sets the
  // last element to stop exactly.
  {
    const int n = cfg->n_sensors;
    std::vector<double> rel(n);
    const double start = -cfg->sensor_half_cone, stop = cfg->sensor_half_cone;
    if (n == 1) {
      rel[0] = start;
    } else {
      const double div = (double)(n - 1);
      const double delta = stop - start;
      const double step = delta / div;
      for (int i = 0; i < n; ++i) rel[i] = (double)i * step + start;
      rel[n - 1] = stop;
    }
    h->rel_angles_h = rel;
    int rc = upload(h->rel_angles, rel.data(), rel.size());
    if (rc) {
      delete h;
      return rc;
    }
  }
  *out = h;
  return RX_OK;
}

int rx_sensor_angles(const rx_env* h, double* out) {
  if (!h || !out) return fail(RX_EINVAL, "rx_sensor_angles: null argument");
  std::copy(h->rel_angles_h.begin(), h->rel_angles_h.end(), out);
  return RX_OK;
}

int rx_env_order(rx_env* h, int32_t* perm_out, int32_t* sort_bins, int32_t* sort_shift) {
  if (!h || !perm_out) return fail(RX_EINVAL, "rx_env_order: null argument");
  if (!h->assigned) return fail(RX_ESTATE, "rx_env_order before rx_assign");
  RX_HIP(hipSetDevice(h->cfg.device));
  RX_HIP(hipDeviceSynchronize());
  RX_HIP(hipMemcpy(perm_out, h->perm[0].p, (size_t)h->cfg.n_envs * sizeof(int32_t), hipMemcpyDeviceToHost));
  if (sort_bins) *sort_bins = h->sort_on ? h->sort_bins : 0;
  if (sort_shift) *sort_shift = h->sort_shift;
  return RX_OK;
}

// the split step applies (k_kin + k_step2): STEP mode, next-step or no autoreset,
// single-agent envs at one lane per env
static bool split_step(const rx_env* h, int mode) {
  return h->split && mode == RX_MODE_STEP && (h->cfg.n_agents == 2 || h->dyn_lpe == 1) &&
         h->cfg.autoreset != RX_AUTORESET_SAME_STEP && h->cs_scratch.p;
}

int rx_schedule(const rx_env* h, int32_t* out) {
  if (!h || !out) return fail(RX_EINVAL, "rx_schedule: null argument");
  if (!h->assigned) return fail(RX_ESTATE, "rx_schedule before rx_assign");
  const int32_t v[RX_SCHEDULE_W] = {h->split ? 1 : 0, h->dyn_lpe == 64 ? 1 : 0, h->dyn_lpe, h->ray_lpr, h->reward_lpe,
                                    h->argmin_window, h->cfg.seg_filter >= 0 ? 1 : 0,
                                    h->cfg.box_quadrants >= 0 ? 1 : 0, h->n_dyn_waves, h->n_ray_waves,
                                    h->ray_dispatch, h->ray_tail, h->ray_tail_lpr, h->ray_tail_from,
                                    h->task_sort, h->lane_tracks, (int32_t)h->dyn_calls, 0};
  std::copy(v, v + RX_SCHEDULE_W, out);
  return RX_OK;
}

int rx_destroy(rx_env* h) {
  if (!h) return RX_OK;
  (void)hipSetDevice(h->cfg.device);
  for (auto* b : {&h->wp, &h->nrm, &h->seg, &h->meta, &h->chunk_box, &h->slot_geo, &h->wchunk_box, &h->super_box,
                  &h->wsuper_box, &h->rel_angles})
    b->release();
  for (auto* b : {&h->wp_off, &h->chunk_off, &h->wchunk_off, &h->super_off, &h->wsuper_off, &h->perm[0], &h->perm[1],
                  &h->slot_n, &h->tasks})
    b->release();
  h->cs_scratch.release();
  h->policy_frag.release();
  h->pos_slot.release();
  h->prof_buf.release();
  h->resets.release();
  h->draw_rank.release();
  h->draw_tmp.release();
  h->draw_base.release();
  h->chunk_box_f.release();
  h->super_box_f.release();
  h->seg_f.release();
  h->slot_hdr.release();
  h->dyn_waves.release();
  h->ray_waves.release();
  for (void* m : h->work_mem) (void)hipFree(m);
  h->work_mem.clear();
  h->keys_in.release();
  h->keys_off.release();
  h->sort_hist.release();
  h->sort_cursor.release();
  h->sort_base.release();
  delete h;
  return RX_OK;
}

int rx_upload_tracks(rx_env* h, int32_t n_tracks, const int32_t* wp_off, const double* wp, const double* nrm,
                     const double* seg, const double* meta) {
  if (!h) return fail(RX_EINVAL, "null handle");
  if (n_tracks <= 0 || !wp_off || !wp || !nrm || !seg || !meta) return fail(RX_EINVAL, "rx_upload_tracks: bad arguments");
  if (wp_off[0] != 0) return fail(RX_EINVAL, "wp_off[0] must be 0");
  for (int k = 0; k < n_tracks; ++k) {
    const int W = wp_off[k + 1] - wp_off[k];
    if (W < 2) return fail(RX_EINVAL, "track %d has %d waypoints (need >= 2)", k, W);
    if (W > 64 * RX_WP_CHUNK * RX_WP_SUPER)  // closest-waypoint super-chunk mask is 64 bits
      return fail(RX_EINVAL, "track %d has %d waypoints (at most %d)", k, W, 64 * RX_WP_CHUNK * RX_WP_SUPER);
    if (!(meta[8 * k + 3] >= 0)) return fail(RX_EINVAL, "track %d width invalid", k);
    if (!(meta[8 * k + 4] > 0)) return fail(RX_EINVAL, "track %d max_track_distance must be > 0", k);
  }
  const size_t Wt = (size_t)wp_off[n_tracks];
  RX_HIP(hipSetDevice(h->cfg.device));
  int rc;
  if ((rc = upload(h->wp_off, wp_off, (size_t)n_tracks + 1))) return rc;
  if ((rc = upload(h->wp, wp, 2 * Wt))) return rc;
  if ((rc = upload(h->nrm, nrm, 2 * Wt))) return rc;
  if ((rc = upload(h->seg, seg, 8 * Wt))) return rc;
  {  // float32 copy of the segments (nearest rounding; the kernel's error bound covers it)
    std::vector<float> sf(8 * (size_t)Wt);
    for (size_t i = 0; i < sf.size(); ++i) sf[i] = (float)seg[i];
    if ((rc = upload(h->seg_f, sf.data(), sf.size()))) return rc;
  }
  if ((rc = upload(h->meta, meta, 8 * (size_t)n_tracks))) return rc;
  if ((rc = build_chunks(h, n_tracks, wp_off, wp, seg, meta))) return rc;
  h->wp_off_h.assign(wp_off, wp_off + n_tracks + 1);
  h->n_tracks = n_tracks;
  h->assigned = false;  // slots may have changed meaning: require rx_assign again
  return RX_OK;
}

static int sync_state(rx_env* h, int to_user, void* stream = nullptr, bool blocking = true);

int rx_assign(rx_env* h, const int32_t* track_of_env) {
  if (!h) return fail(RX_EINVAL, "null handle");
  if (h->n_tracks <= 0) return fail(RX_ESTATE, "rx_assign before rx_upload_tracks");
  if (!track_of_env) return fail(RX_EINVAL, "track_of_env is null");
  const int N = h->cfg.n_envs, A = h->cfg.n_agents, R = h->cfg.n_sensors;
  for (int e = 0; e < N; ++e)
    if (track_of_env[e] < 0 || track_of_env[e] >= h->n_tracks)
      return fail(RX_EINVAL, "env %d assigned to track %d (have %d)", e, track_of_env[e], h->n_tracks);
  // group envs by slot (stable: env order inside a slot is preserved)
  std::vector<int32_t> perm(N);
  std::iota(perm.begin(), perm.end(), 0);
  std::stable_sort(perm.begin(), perm.end(), [&](int32_t a, int32_t b) { return track_of_env[a] < track_of_env[b]; });
  std::vector<rx_wave> dyn, ray;
  std::vector<int> ray_groups;  // end index (in ray) of each 64-env block's waves
  if (h->cfg.ray_order == 2 && A * R > 16 * A)
    return fail(RX_EINVAL, "ray_order 2 supports at most 16 sensors (got %d)", R);
  // launch schedule (rx_config ABI v17 fields; 0 = the measured default for N)
  const rx_config& c = h->cfg;
  h->dyn_lpe = (A == 1 && N <= RX_DYN1_SMALL_N) ? RX_DYN1_LPE_SMALL : 1;
  const int wide_n = c.wide_n == 0 ? RX_WIDE_N : c.wide_n;  // -1: never
  if (A == 1 && N <= wide_n) h->dyn_lpe = 64;
  if (A == 1 && c.dyn_lpe != 0) h->dyn_lpe = c.dyn_lpe;
  h->argmin_window = c.argmin_window == 0 ? 2 : (c.argmin_window < 0 ? 0 : c.argmin_window);
  {  // the window [prev - H, prev + H] is wrapped into [0, W) by one +-W: needs H <= W of every slot
    int min_w = 1 << 30;
    for (int k = 0; k < h->n_tracks; ++k) min_w = std::min(min_w, h->wp_off_h[k + 1] - h->wp_off_h[k]);
    h->argmin_window = std::min(h->argmin_window, min_w);
  }
  // few envs: the culled raycast is a latency chain over too few waves to
  // fill the chip, so 2 or 4 lanes share one ray and split its leaves
  h->ray_lpr = 1;
  if (h->cfg.ray_order == 2 && h->dyn_lpe != 64) {
    const long long pairs = (long long)N * A, lpr2_n = A == 2 ? RX_RAY2_LPR2_N : RX_RAY_LPR2_N;
    h->ray_lpr = pairs <= RX_RAY_LPR4_N ? 4 : (pairs <= lpr2_n ? 2 : 1);
    if (c.ray_lpr != 0) h->ray_lpr = c.ray_lpr;
  }
  // few single-agent envs: REWARD (a latency chain of argmins) outlasts the
  // raycast beside it in k_step2 unless 2 lanes share an env's five points
  h->reward_lpe = (A == 1 && N <= RX_REWARD_LPE2_N) || (A == 2 && N <= RX_REWARD2_LPE2_N) ? 2 : 1;
  if (c.reward_lpe != 0) h->reward_lpe = c.reward_lpe;
  h->split = c.split >= 0;
  // ray-wave class order and the tail split (ABI v19; scheduling only)
  h->ray_dispatch = c.ray_dispatch == 0 ? RX_RAY_DISPATCH : (c.ray_dispatch < 0 ? 0 : c.ray_dispatch);
  h->ray_tail_lpr = c.ray_tail_lpr == 0 ? RX_RAY_TAIL_LPR : c.ray_tail_lpr;
  // few (env, car) pairs: the ray waves are short and the sort is up to 40 % of
  // k_kin's wave, so every other launch keeps the previous task order
  h->task_sort = c.task_sort != 0 ? c.task_sort : ((long long)N * A <= RX_TASK_SORT2_PAIRS ? 2 : 1);
  h->ray_tail = c.ray_tail == 0 ? RX_RAY_TAIL : (c.ray_tail < 0 ? 0 : c.ray_tail);
  if (h->cfg.ray_order != 2 || h->ray_lpr != 1 || h->ray_dispatch == 0 || h->dyn_lpe == 64) h->ray_tail = 0;
  h->ray_tail_from = -1;
  std::vector<int32_t> slot_n(h->n_tracks, 0);
  for (int e = 0; e < N; ++e) ++slot_n[track_of_env[e]];
  // Lane-varying track slots (ABI v23): grouping envs by slot gives every slot
  // ceil(n_k / 64) dynamics waves; with many distinct slots (gen_tracks(N, seed=None): one env
  // each) those waves hold a lane or two.  Auto rule: take waves of 64 consecutive positions of
  // ANY slots (per-lane track loads) when the grouping would need more than twice ceil(N / 64)
  // waves.  Single-agent envs at one lane per env (the split step or the one-kernel k_dyn1<1>);
  // it implies one lane per ray and per REWARD env and no ray-task sort or spatial re-sort.
  {
    long long grouped = 0;
    for (int k = 0; k < h->n_tracks; ++k) grouped += (slot_n[k] + 63) / 64;
    const long long full = (N + 63) / 64;
    const bool can = A == 1 && h->dyn_lpe == 1;
    h->lane_tracks = can && c.lane_tracks >= 0 && (c.lane_tracks == 1 || grouped > 2 * full) ? 1 : 0;
  }
  if (h->lane_tracks) {
    h->ray_lpr = 1;
    h->reward_lpe = 1;
    h->ray_dispatch = 0;
    h->ray_tail = 0;
  }
  const int tpw = 64 / h->ray_lpr;  // ray tasks per wave
  int g0 = h->lane_tracks ? N : 0;
  for (int ps = 0; h->lane_tracks && ps < N; ps += 64) {  // 64 consecutive positions, (env, agent, ray) tasks
    const int cnt = std::min(64, N - ps), nt = cnt * A * R;
    dyn.push_back(rx_wave{-1, ps, 0, cnt});
    for (int j = 0; j < nt; j += 64) ray.push_back(rx_wave{-1, ps, j, std::min(64, nt - j)});
    ray_groups.push_back((int)ray.size());
  }
  while (g0 < N) {
    const int k = track_of_env[perm[g0]];
    int g1 = g0;
    while (g1 < N && track_of_env[perm[g1]] == k) ++g1;
    const int ng = g1 - g0;
    const int epw = A == 1 ? 64 / h->dyn_lpe : 64;  // envs per dynamics wave
    for (int s = 0; s < ng; s += epw) dyn.push_back(rx_wave{k, g0 + s, 0, std::min(epw, ng - s)});
    if (h->cfg.ray_order == 2) {  // per dynamics wave: its envs' A*R tasks (direction-sorted by k_dyn), tpw a wave
      for (int s = 0; s < ng; s += epw) {
        const int cnt = std::min(epw, ng - s), nt = cnt * A * R, ps = g0 + s;
        for (int j = 0; j < nt; j += tpw) ray.push_back(rx_wave{k, ps, ps * A * R + j, std::min(tpw, nt - j)});
        ray_groups.push_back((int)ray.size());
      }
    } else if (h->cfg.ray_order == 0) {
      const long long tasks = (long long)ng * A * R;
      for (long long s = 0; s < tasks; s += 64)
        ray.push_back(rx_wave{k, g0, (int32_t)s, (int32_t)std::min<long long>(64, tasks - s)});
    } else {  // ray-major: one (agent, ray) x one 64-env block per wave, grouped by block
      for (int b = 0; 64 * b < ng; ++b) {
        for (int qr = 0; qr < A * R; ++qr)
          ray.push_back(rx_wave{k, g0, qr * ng + 64 * b, std::min(64, ng - 64 * b)});
        ray_groups.push_back((int)ray.size());
      }
    }
    g0 = g1;
  }
  if (h->cfg.ray_order >= 1 || h->lane_tracks) {
    // XCD-aware placement: workgroups are dealt round-robin over the 8 XCDs
    // (MI355X_MICROARCH.md, workgroup dispatch), and every wave of one 64-env
    // block writes into the same obs rows, so the (up to) A*R waves of block g
    // go to physical indices p = ((g / 8) * maxw + j) * 8 + g % 8 -- one XCD,
    // one L2 to merge their partial-line writes.  Padding waves have count 0.
    const size_t n_groups = ray_groups.size();
    int maxw = 0;
    for (size_t g = 0; g < n_groups; ++g) maxw = std::max(maxw, ray_groups[g] - (g ? ray_groups[g - 1] : 0));
    const size_t padded = (n_groups + 7) / 8 * 8;
    // ray_dispatch (rx_config, ABI v19): 0 = group-octet-major as just described; 1..3 =
    // class-major, every group's class-j wave in one run, the classes in the order
    // 1 centre first (|2j - (maxw - 1)| ascending), 2 ascending j, 3 edge classes first
    // (|2j - (maxw - 1)| descending, the default).  The XCD of a group's waves is g % 8 in
    // every mode (padded is a multiple of 8).  Dispatch order is scheduling only.
    const int mode = h->ray_dispatch;
    std::vector<int> rank(maxw);
    std::iota(rank.begin(), rank.end(), 0);
    if (mode == 1 || mode == 3) {
      std::vector<int> cls(maxw);
      std::iota(cls.begin(), cls.end(), 0);
      auto off = [&](int j) { return std::abs(2 * j - (maxw - 1)); };
      std::stable_sort(cls.begin(), cls.end(), [&](int x, int y) { return mode == 1 ? off(x) < off(y) : off(x) > off(y); });
      for (int r = 0; r < maxw; ++r) rank[cls[r]] = r;
    }
#ifdef RX_RAY_ORDER_LIST
    {  // A/B builds: an explicit class order for 11-class groups (ray_dispatch >= 1)
      const int lst[] = RX_RAY_ORDER_LIST;
      if (mode >= 1 && maxw == (int)(sizeof(lst) / sizeof(lst[0]))) {
        // the list must be a permutation of 0..maxw-1: a repeated class would give two
        // ray waves one placed slot (one silently overwritten, its rays never cast)
        std::vector<bool> seen(maxw, false);
        for (int r = 0; r < maxw; ++r) {
          if (lst[r] < 0 || lst[r] >= maxw || seen[lst[r]])
            return fail(RX_EINVAL, "RX_RAY_ORDER_LIST is not a permutation of 0..%d", maxw - 1);
          seen[lst[r]] = true;
          rank[lst[r]] = r;
        }
      }
    }
#endif
    // The tail split (ray_tail, class-major modes only): the waves of the last ray_tail
    // ranks run as the chip drains, where a wave's latency chain -- not the shared VALU --
    // sets its duration.  Each of their 64-task records becomes m = ray_tail_lpr records of
    // 64 / m tasks, cast at m lanes per ray (the lanes split each scanned leaf: a shorter
    // chain, the same result, DESIGN.md §3 "Lanes per ray").  Rank r occupies mult[r]
    // consecutive runs of `padded` slots; sub-record s of group g's rank-r wave goes to
    // base[r] + (s * (padded / 8) + g / 8) * 8 + g % 8, so it keeps the group's XCD.  All
    // tail waves sit at the end of the table: ray_tail_from is the first of them.
    const int tail = mode == 0 ? 0 : std::min(h->ray_tail, maxw);
    std::vector<size_t> mult(maxw, 1), base(maxw + 1, 0);
    for (int r = maxw - tail; r < maxw; ++r) mult[r] = (size_t)h->ray_tail_lpr;
    for (int r = 0; r < maxw; ++r) base[r + 1] = base[r] + mult[r] * padded;
    std::vector<rx_wave> placed(base[maxw], rx_wave{0, 0, 0, 0});
    for (size_t g = 0; g < n_groups; ++g) {
      const int w0 = g ? ray_groups[g - 1] : 0;
      for (int j = 0; w0 + j < ray_groups[g]; ++j) {
        const rx_wave w = ray[w0 + j];
        if (mode == 0) {
          placed[((g / 8) * maxw + j) * 8 + g % 8] = w;
          continue;
        }
        const int r = rank[j];
        const int m = (int)mult[r], per = tpw / m;
        for (int sub = 0; sub < m; ++sub) {
          const size_t slot = base[r] + ((size_t)sub * (padded / 8) + g / 8) * 8 + g % 8;
          placed[slot] = rx_wave{w.track, w.perm_start, w.task_start + sub * per,
                                 std::max(0, std::min(per, w.count - sub * per))};
        }
      }
    }
    h->ray_tail = tail;
    h->ray_tail_from = tail > 0 ? (int32_t)base[maxw - tail] : -1;
    ray.swap(placed);
  }
  RX_HIP(hipSetDevice(h->cfg.device));
  int rc;
  if ((rc = upload(h->slot_n, slot_n.data(), slot_n.size()))) return rc;
  if ((rc = upload(h->perm[0], perm.data(), perm.size()))) return rc;
  if ((rc = upload(h->perm[1], perm.data(), perm.size()))) return rc;
  if (A == 2) {
    std::vector<uint32_t> z(N, 0u);
    if ((rc = upload(h->resets, z.data(), z.size()))) return rc;
  }
  h->sort_on = false;
  if (h->lane_tracks) {  // the kernels read each position's slot: the order stays fixed
    std::vector<int32_t> ps(N);
    for (int p = 0; p < N; ++p) ps[p] = track_of_env[perm[p]];
    if ((rc = upload(h->pos_slot, ps.data(), ps.size()))) return rc;
  } else if (h->cfg.sort_interval > 0) {
    // spatial sort bins: slot k owns (W_k >> shift) + 1 consecutive bins from
    // sort_base[k]; the smallest shift that keeps all bins <= RX_SORT_MAX_BINS.
    // More slots than that (at most ~1 env per slot): nothing to regroup, no sort.
    int shift = 0;
    long long total = 0;
    for (;; ++shift) {
      total = 0;
      for (int k = 0; k < h->n_tracks; ++k) total += ((h->wp_off_h[k + 1] - h->wp_off_h[k]) >> shift) + 1;
      if (total <= RX_SORT_MAX_BINS || shift >= 30) break;
    }
    if (total <= RX_SORT_MAX_BINS) {
      std::vector<int32_t> base(h->n_tracks);
      int32_t run = 0;
      for (int k = 0; k < h->n_tracks; ++k) {
        base[k] = run;
        run += ((h->wp_off_h[k + 1] - h->wp_off_h[k]) >> shift) + 1;
      }
      std::vector<uint32_t> zk(std::max<size_t>((size_t)N, (size_t)total), 0u);
      if ((rc = upload(h->sort_base, base.data(), base.size()))) return rc;
      if ((rc = upload(h->keys_in, zk.data(), (size_t)N))) return rc;
      if ((rc = upload(h->keys_off, zk.data(), (size_t)N))) return rc;
      if ((rc = upload(h->sort_hist, zk.data(), (size_t)total))) return rc;
      if ((rc = upload(h->sort_cursor, zk.data(), (size_t)total))) return rc;
      h->sort_bins = (int32_t)total;
      h->sort_shift = shift;
      h->sort_on = true;
    }
  }
  if (h->cfg.ray_order == 2) {  // task ids before the first sort: position-major, (agent, ray) minor -- a valid order
    const size_t nt = (size_t)N * A * R;
    std::vector<int32_t> t0(nt);
    for (size_t o = 0; o < nt; ++o) t0[o] = (int32_t)o;  // task id (A*p + q)*R + r at slot p*A*R + q*R + r
    if ((rc = upload(h->tasks, t0.data(), nt))) return rc;
  }
  {
    std::vector<double> z(2 * (size_t)N * A, 0.0);
    if ((rc = upload(h->cs_scratch, z.data(), z.size()))) return rc;
  }
  if ((rc = upload(h->dyn_waves, dyn.data(), dyn.size()))) return rc;
  if ((rc = upload(h->ray_waves, ray.data(), ray.size()))) return rc;
  h->ray_waves_h = ray;
  h->n_dyn_waves = (int32_t)dyn.size();
  h->n_ray_waves = (int32_t)ray.size();
  if (!h->policy_frag.p) {  // allocated here, not in rx_rollout_steps: it may run inside a graph capture
    RX_HIP(hipSetDevice(h->cfg.device));
    if (hipMalloc(&h->policy_frag.p, rx_policy_frag_bytes()) != hipSuccess)
      return fail(RX_ENOMEM, "rx_assign: policy fragment image");
    h->policy_frag.n = rx_policy_frag_bytes();
  }
  h->assigned = true;
  h->tasks_stale = true;
  h->sort_pending = false;
  h->sort_hist_done = false;  // the histogram was re-uploaded as zeros above (or sorting is off)
  if (h->bound && h->st.track) RX_HIP(hipMemcpy(h->st.track, track_of_env, N * sizeof(int32_t), hipMemcpyHostToDevice));
  if (h->bound) return sync_state(h, 0);  // the new wave order: re-read the caller's arrays
  return RX_OK;
}

// working copy <-> the caller's arrays (env order); blocking = finish before
// returning (bind / assign), else enqueued on the caller's stream
static int sync_state(rx_env* h, int to_user, void* stream, bool blocking) {
  if (!h->bound || !h->assigned) return fail(RX_ESTATE, "state sync needs rx_bind_state and rx_assign");
  RX_HIP(hipSetDevice(h->cfg.device));
  rx_state user = h->st, work = h->work;
  if (!user.finished_step) work.finished_step = nullptr;  // A == 1 without the array: nothing to move
  int rc = rx_state_sync(&work, &user, h->perm[0].p, h->cfg.n_envs, h->cfg.n_agents, to_user, (hipStream_t)stream);
  if (rc) return fail(RX_EHIP, "state sync failed: %s", hipGetErrorString((hipError_t)rc));
  if (blocking) RX_HIP(hipDeviceSynchronize());
  return RX_OK;
}

int rx_bind_state(rx_env* h, const rx_state* st) {
  if (!h || !st) return fail(RX_EINVAL, "rx_bind_state: null argument");
  if (!st->x || !st->y || !st->angle || !st->vx || !st->vy || !st->progress || !st->last_progress ||
      !st->last_steering || !st->flags || !st->steps || !st->track || !st->env_flags || !st->ep_return ||
      !st->ep_length)
    return fail(RX_EINVAL, "rx_bind_state: every state array except finished_step is required");
  if (h->cfg.n_agents == 2 && !st->finished_step) return fail(RX_EINVAL, "rx_bind_state: finished_step required for 2 agents");
  h->st = *st;
  if (!h->work.x) {  // working copy + shadow, same shapes as the caller's arrays
    const size_t N = (size_t)h->cfg.n_envs, NA = N * (size_t)h->cfg.n_agents;
    for (rx_state* w : {&h->work, &h->work_tmp}) {
      auto alloc = [&](auto** ptr, size_t bytes) -> int {
        void* m = nullptr;
        if (hipMalloc(&m, std::max<size_t>(bytes, 16)) != hipSuccess) return fail(RX_ENOMEM, "working state alloc");
        RX_HIP(hipMemset(m, 0, std::max<size_t>(bytes, 16)));
        h->work_mem.push_back(m);
        *ptr = reinterpret_cast<std::remove_reference_t<decltype(*ptr)>>(m);
        return RX_OK;
      };
      int rc;
      for (double** f : {&w->x, &w->y, &w->angle, &w->vx, &w->vy, &w->progress, &w->last_progress, &w->last_steering})
        if ((rc = alloc(f, NA * sizeof(double)))) return rc;
      if ((rc = alloc(&w->flags, NA))) return rc;
      if ((rc = alloc(&w->finished_step, NA * sizeof(int32_t)))) return rc;
      if ((rc = alloc(&w->steps, N * sizeof(int32_t)))) return rc;
      if ((rc = alloc(&w->env_flags, N))) return rc;
      if ((rc = alloc(&w->ep_return, N * sizeof(double)))) return rc;
      if ((rc = alloc(&w->ep_length, N * sizeof(int32_t)))) return rc;
    }
  }
  h->bound = true;
  if (h->assigned) return sync_state(h, 0);
  return RX_OK;
}

int rx_state_import(rx_env* h, void* stream) {
  if (!h) return fail(RX_EINVAL, "null handle");
  return sync_state(h, 0, stream, false);
}

int rx_state_export(rx_env* h, void* stream) {
  if (!h) return fail(RX_EINVAL, "null handle");
  return sync_state(h, 1, stream, false);
}

int rx_set_speed_weight(rx_env* h, double w) {
  if (!h) return fail(RX_EINVAL, "null handle");
  if (!(w == w)) return fail(RX_EINVAL, "speed_weight is NaN");
  h->cfg.speed_weight = w;
  return RX_OK;
}

// rx_profile: give the next launch its stamp record (nullptr when not
// profiling or the record is full).
static constexpr int kProfMax = 512;  // launches per record
static int prof_stride(const rx_env* h) {
  const int wide = h->cfg.n_envs * h->cfg.n_agents * h->cfg.n_sensors;  // k_rays_wide: one wave per ray
  return std::max(h->reward_lpe * ((h->n_dyn_waves + 7) / 8 * 8) + h->n_ray_waves, wide) + 8;
}
static void prof_arm(rx_env* h, rx_kargs& a, int kind) {
  a.prof_ts = nullptr;
  if (!h->prof || !h->prof_buf.p || (int)h->prof_kinds.size() >= kProfMax) return;
  a.prof_stride = prof_stride(h);
  a.prof_ts = h->prof_buf.p + (size_t)h->prof_kinds.size() * 2 * a.prof_stride;
  h->prof_kinds.push_back(kind);
}

static void make_kargs(rx_env* h, const rx_io* io, int mode, const uint8_t* mask, rx_kargs& a) {
  a.tr = rx_track_view{h->wp_off.p,    h->wp.p,        h->nrm.p,      h->seg.p,        h->meta.p,
                       h->chunk_off.p, h->chunk_box.p, h->slot_geo.p, h->wchunk_off.p, h->wchunk_box.p,
                       h->super_off.p, h->super_box.p, h->wsuper_off.p, h->wsuper_box.p,
                       h->chunk_box_f.p, h->super_box_f.p, h->n_chunk_boxes, h->n_super_boxes, h->seg_f.p,
                       h->slot_hdr.p};
  a.st = h->work;
  a.st.track = h->st.track;                // read-only, env order
  a.st.speed_weight = h->st.speed_weight;  // read-only, env order (or nullptr)
  a.io = *io;
  a.dyn_waves = h->dyn_waves.p;
  a.ray_waves = h->ray_waves.p;
  a.perm = h->perm[0].p;
  a.rel_angles = h->rel_angles.p;
  a.reset_mask = mask;
  a.n_dyn_waves = h->n_dyn_waves;
  a.n_ray_waves = h->n_ray_waves;
  a.n_sensors = h->cfg.n_sensors;
  a.D = h->D;
  a.max_steps = h->cfg.max_steps;
  a.autoreset = h->cfg.autoreset;
  a.mode = mode;
  a.cull_chunk = h->chunk_box.p ? h->cfg.cull_chunk : 0;
  a.cull_super = h->super_box.p ? h->cfg.cull_super : 0;
  a.speed_weight = h->cfg.speed_weight;
  a.seed = h->cfg.seed;
  a.reset_count = h->resets.p;
  a.ray_order = h->cfg.ray_order;
  a.dyn_lpe = h->dyn_lpe;
  a.ray_lpr = h->ray_lpr;
  a.ray_tail_from = h->ray_tail_from;
  a.ray_tail_lpr = h->ray_tail_lpr;
  a.reward_lpe = h->reward_lpe;
  a.argmin_window = h->argmin_window;
  a.slot_nenv = h->slot_n.p;
  a.wide = h->dyn_lpe == 64;
  a.n_wide_tasks = h->cfg.n_envs * h->cfg.n_agents * h->cfg.n_sensors;
  a.tasks = h->tasks.p;
  a.tasks_out = (h->cfg.ray_order == 2 && !a.wide && !h->lane_tracks) ? h->tasks.p : nullptr;
  a.lane_tracks = h->lane_tracks;
  a.pos_slot = h->lane_tracks ? h->pos_slot.p : nullptr;
  a.cs_scratch = h->cs_scratch.p;
  a.sort_base = h->sort_base.p;
  a.sort_shift = h->sort_shift;
  a.box_quadrants = h->cfg.box_quadrants >= 0;
  a.seg_filter = h->cfg.seg_filter >= 0;
#ifdef RX_AB_NO_EPSTATS  // A/B build only (tools/build_rev.py): drop the episode-statistics atomics
  a.io.ep_stats = nullptr;
#endif
}

static int launch(rx_env* h, const rx_io* io, int mode, const uint8_t* mask, void* stream, int phases = 3) {
  if (phases < 1 || phases > 3) return fail(RX_EINVAL, "phases must be 1, 2 or 3 (got %d)", phases);
  if (!h) return fail(RX_EINVAL, "null handle");
  if (!io) return fail(RX_EINVAL, "io is null");
  if (h->n_tracks <= 0) return fail(RX_ESTATE, "no track table (rx_upload_tracks)");
  if (!h->assigned) return fail(RX_ESTATE, "no env assignment (rx_assign)");
  if (!h->bound) return fail(RX_ESTATE, "no state bound (rx_bind_state)");
  if (!io->obs) return fail(RX_EINVAL, "io->obs is required");
  if (mode == RX_MODE_STEP && !io->actions) return fail(RX_EINVAL, "io->actions is required");
  rx_kargs a{};
  make_kargs(h, io, mode, mask, a);
  hipStream_t s = (hipStream_t)stream;
  int rc;
  // Split step: k_kin1 / k_kin2 (resets, kinematics, [car-car contact,]
  // non-ray obs, ray-task sort), then k_step2<A> = the REWARD part (argmins,
  // collision, reward, done) side by side with the raycast in ONE launch.  STEP
  // with next-step or no autoreset; single-agent envs at one lane per env
  // (same-step autoreset needs done before the observation; explicit resets
  // and small single-agent N use the one-kernel path).
  const int A = h->cfg.n_agents;
  // rx_set_start_draws: rank the envs this launch's dynamics kernel resets (env order)
  if (h->draws && A == 2 && (phases & RX_PHASE_DYNAMICS) &&
      (mode == RX_MODE_RESET || h->cfg.autoreset == RX_AUTORESET_NEXT_STEP)) {
    if ((rc = rx_launch_reset_rank(h->cfg.n_envs, mode, mask, a.st.env_flags, a.perm, h->draw_tmp.p, h->draw_rank.p,
                                   h->draw_cursor, h->draw_base.p, h->n_draws, s)) != 0)
      return fail(RX_EHIP, "k_reset_rank launch failed: %s", hipGetErrorString((hipError_t)rc));
    a.draws = h->draws;
    a.n_draws = h->n_draws;
    a.draw_base = h->draw_base.p;
    a.reset_rank = h->draw_rank.p;
  }
  const bool split = split_step(h, mode);
  // Spatial re-sort, every sort_interval dynamics launches: that launch's
  // REWARD half (or k_dyn) writes the sort keys; the sort -- which moves the
  // working-state rows -- runs after the step's raycast (the ray tasks name
  // positions), so the new order applies from the next step.
  const bool dyn = (phases & RX_PHASE_DYNAMICS) != 0;
  // the ray-task order only steers which rays share a wave (results never depend
  // on it): a launch may reuse the previous one's while the blocks hold the same envs
  if (dyn && a.tasks_out) {
    if (h->tasks_stale || (h->task_calls % (uint64_t)h->task_sort) == 0)
      h->tasks_stale = false;
    else
      a.tasks_out = nullptr;
    ++h->task_calls;
  }
  if (dyn && h->cfg.sort_interval > 0 && h->sort_on && (h->dyn_calls++ % h->cfg.sort_interval) == 0) {
    a.sort_keys = h->keys_in.p;
    // The histogram is zero unless sort_hist_done, when it holds the counts of
    // the keys this launch is about to overwrite (keys requested again before
    // their sort ran: rx_step_phases(1) twice, or a reset in between): clear it,
    // so the fused count below, or k_sort_hist, starts from zero.
    if (h->sort_hist_done) {
      RX_HIP(hipMemsetAsync(h->sort_hist.p, 0, (size_t)h->sort_bins * sizeof(uint32_t), s));
      h->sort_hist_done = false;
    }
    h->sort_pending = true;
  }
  if (split) {
    uint32_t* keys = a.sort_keys;
    if (dyn) {
      a.sort_keys = nullptr;
      prof_arm(h, a, RX_KERNEL_KIN);
      if ((rc = rx_launch_split(&a, A, RX_SPLIT_KIN, s)) != 0)
        return fail(RX_EHIP, "k_kin1 launch failed: %s", hipGetErrorString((hipError_t)rc));
      a.tasks_out = nullptr;
      a.sort_keys = keys;
      // single-agent: the REWARD half also builds the re-sort's histogram (one
      // launch fewer per re-sort: rx_sort_envs skips k_sort_hist)
      if (keys && A == 1) {
        a.sort_hist = h->sort_hist.p;
        a.sort_off = h->keys_off.p;
        h->sort_hist_done = true;
      }
      prof_arm(h, a, phases == 3 ? RX_KERNEL_STEP2 : RX_KERNEL_REWARD);
      if ((rc = rx_launch_split(&a, A, phases == 3 ? RX_SPLIT_REWARD_RAYS : RX_SPLIT_REWARD, s)) != 0)
        return fail(RX_EHIP, "k_step2 launch failed: %s", hipGetErrorString((hipError_t)rc));
    } else {
      a.tasks_out = nullptr;
      prof_arm(h, a, RX_KERNEL_RAYS);
      if ((rc = rx_launch_step(&a, A, RX_PHASE_RAYS, s)) != 0)
        return fail(RX_EHIP, "k_rays launch failed: %s", hipGetErrorString((hipError_t)rc));
    }
  } else {
    if (dyn) {
      prof_arm(h, a, RX_KERNEL_DYN);
      if ((rc = rx_launch_step(&a, h->cfg.n_agents, RX_PHASE_DYNAMICS, s)) != 0)
        return fail(RX_EHIP, "k_dyn launch failed: %s", hipGetErrorString((hipError_t)rc));
    }
    if (phases & RX_PHASE_RAYS) {
      a.sort_keys = nullptr;
      a.tasks_out = nullptr;
      prof_arm(h, a, RX_KERNEL_RAYS);
      if ((rc = rx_launch_step(&a, h->cfg.n_agents, RX_PHASE_RAYS, s)) != 0)
        return fail(RX_EHIP, "k_rays launch failed: %s", hipGetErrorString((hipError_t)rc));
    }
  }
  if (h->sort_pending && (phases & RX_PHASE_RAYS)) {
    h->sort_pending = false;
    h->tasks_stale = true;  // the re-sort moves envs between blocks
    rx_state work = h->work, tmp = h->work_tmp;
    const int hist_done = h->sort_hist_done ? 1 : 0;
    h->sort_hist_done = false;
    if ((rc = rx_sort_envs(h->keys_in.p, h->keys_off.p, h->cfg.n_envs, A, h->sort_hist.p, h->sort_cursor.p, h->sort_bins,
                           h->perm[0].p, h->perm[1].p, &work, &tmp, s, hist_done)) != 0)
      return fail(RX_EHIP, "spatial sort failed: %s", hipGetErrorString((hipError_t)rc));
  }
  return RX_OK;
}

int rx_profile(rx_env* h, int32_t enable) {
  if (!h) return fail(RX_EINVAL, "null handle");
  if (enable == 1) {  // a fresh record, all stamps 0 (= no wave)
    if (!h->assigned) return fail(RX_ESTATE, "rx_profile before rx_assign");
    RX_HIP(hipSetDevice(h->cfg.device));
    RX_HIP(hipDeviceSynchronize());  // no launch of the previous record may still write
    const size_t n = (size_t)kProfMax * 2 * prof_stride(h);
    if (h->prof_buf.n < n) {
      h->prof_buf.release();
      if (hipMalloc(&h->prof_buf.p, n * sizeof(unsigned long long)) != hipSuccess)
        return fail(RX_ENOMEM, "rx_profile: stamp buffer alloc");
      h->prof_buf.n = n;
    }
    RX_HIP(hipMemset(h->prof_buf.p, 0, n * sizeof(unsigned long long)));
    h->prof_kinds.clear();
  }
  h->prof = enable != 0;  // 2 = resume the current record
  return RX_OK;
}

int rx_profile_read(rx_env* h, double* mean_ms, int32_t* count) {
  if (!h || !mean_ms || !count) return fail(RX_EINVAL, "rx_profile_read: null argument");
  double sum[RX_KERNEL_KINDS] = {0};
  int32_t n[RX_KERNEL_KINDS] = {0};
  const size_t nl = h->prof_kinds.size();
  if (nl) {
    RX_HIP(hipSetDevice(h->cfg.device));
    int khz = 0;
    RX_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, h->cfg.device));
    if (khz <= 0) return fail(RX_EHIP, "rx_profile_read: no wall-clock rate");
    RX_HIP(hipDeviceSynchronize());
    const int stride = prof_stride(h);
    std::vector<unsigned long long> st(nl * 2 * stride);
    RX_HIP(hipMemcpy(st.data(), h->prof_buf.p, st.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    for (size_t l = 0; l < nl; ++l) {
      const unsigned long long* r = st.data() + l * 2 * stride;
      unsigned long long t0 = ~0ull, t1 = 0;
      for (int i = 0; i < stride; ++i) {
        if (r[i]) t0 = std::min(t0, r[i]);
        t1 = std::max(t1, r[stride + i]);
      }
      if (t1 == 0 || t0 == ~0ull || t1 < t0) continue;  // launch with no waves
      sum[h->prof_kinds[l]] += (double)(t1 - t0) / (double)khz;  // ticks / kHz = ms
      ++n[h->prof_kinds[l]];
    }
  }
  for (int k = 0; k < RX_KERNEL_KINDS; ++k) {
    mean_ms[k] = n[k] ? sum[k] / n[k] : 0.0;
    count[k] = n[k];
  }
  return RX_OK;
}

int rx_profile_waves(rx_env* h, int32_t launch, uint64_t* start, uint64_t* end, int32_t cap, int32_t* n_waves,
                     int32_t* kind, int32_t* khz) {
  if (!h || !start || !end || !n_waves || !kind || !khz) return fail(RX_EINVAL, "rx_profile_waves: null argument");
  if (launch < 0 || (size_t)launch >= h->prof_kinds.size())
    return fail(RX_EINVAL, "rx_profile_waves: launch %d not recorded (%d in the record)", launch,
                (int)h->prof_kinds.size());
  if (cap < 0) return fail(RX_EINVAL, "rx_profile_waves: cap %d < 0", cap);
  RX_HIP(hipSetDevice(h->cfg.device));
  RX_HIP(hipDeviceGetAttribute(khz, hipDeviceAttributeWallClockRate, h->cfg.device));
  RX_HIP(hipDeviceSynchronize());
  const int stride = prof_stride(h);
  const int n = std::min(stride, cap);
  const unsigned long long* r = h->prof_buf.p + (size_t)launch * 2 * stride;
  if (n > 0) {
    RX_HIP(hipMemcpy(start, r, (size_t)n * sizeof(uint64_t), hipMemcpyDeviceToHost));
    RX_HIP(hipMemcpy(end, r + stride, (size_t)n * sizeof(uint64_t), hipMemcpyDeviceToHost));
  }
  *n_waves = stride;
  *kind = h->prof_kinds[launch];
  return RX_OK;
}

int rx_ray_waves(const rx_env* h, int32_t* out, int32_t cap, int32_t* n_waves) {
  if (!h || !n_waves || (cap > 0 && !out)) return fail(RX_EINVAL, "rx_ray_waves: null argument");
  if (!h->assigned) return fail(RX_ESTATE, "rx_ray_waves before rx_assign");
  const size_t n = h->ray_waves_h.size();
  for (size_t i = 0; i < n && (int64_t)i < (int64_t)cap; ++i) {
    const rx_wave& w = h->ray_waves_h[i];
    out[4 * i + 0] = w.track;
    out[4 * i + 1] = w.perm_start;
    out[4 * i + 2] = w.task_start;
    out[4 * i + 3] = w.count;
  }
  *n_waves = (int32_t)n;
  return RX_OK;
}

int rx_ray_tasks(rx_env* h, int32_t* out, int64_t cap, int64_t* n, void* stream) {
  if (!h || !n || (cap > 0 && !out)) return fail(RX_EINVAL, "rx_ray_tasks: null argument");
  if (!h->assigned) return fail(RX_ESTATE, "rx_ray_tasks before rx_assign");
  const int64_t len = std::min<int64_t>((int64_t)h->tasks.n,
                                        (int64_t)h->cfg.n_envs * h->cfg.n_agents * h->cfg.n_sensors);
  *n = len;
  if (cap <= 0) return RX_OK;
  const hipStream_t s = (hipStream_t)stream;
  if (hipMemcpyAsync(out, h->tasks.p, (size_t)std::min(cap, len) * sizeof(int32_t), hipMemcpyDeviceToHost, s) !=
          hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return fail(RX_EHIP, "rx_ray_tasks: copy failed");
  return RX_OK;
}

int rx_set_start_draws(rx_env* h, const uint32_t* draws, int64_t n_draws, int64_t* cursor) {
  if (!h) return fail(RX_EINVAL, "null handle");
  if (!draws) {
    h->draws = nullptr, h->n_draws = 0, h->draw_cursor = nullptr;
    return RX_OK;
  }
  if (h->cfg.n_agents != 2) return fail(RX_EINVAL, "rx_set_start_draws: single-agent resets draw nothing");
  if (h->cfg.autoreset == RX_AUTORESET_SAME_STEP)
    return fail(RX_EINVAL, "rx_set_start_draws: same-step autoreset draws inside the step (unsupported)");
  if (n_draws < 0 || !cursor) return fail(RX_EINVAL, "rx_set_start_draws: need n_draws >= 0 and a cursor");
  RX_HIP(hipSetDevice(h->cfg.device));
  const size_t N = (size_t)h->cfg.n_envs;
  if (h->draw_rank.n < N) {
    h->draw_rank.release();
    h->draw_tmp.release();
    if (hipMalloc(&h->draw_rank.p, N * sizeof(int32_t)) != hipSuccess ||
        hipMalloc(&h->draw_tmp.p, N * sizeof(int32_t)) != hipSuccess)
      return fail(RX_ENOMEM, "rx_set_start_draws: rank buffers");
    h->draw_rank.n = h->draw_tmp.n = N;
  }
  if (!h->draw_base.p) {
    if (hipMalloc(&h->draw_base.p, sizeof(int64_t)) != hipSuccess) return fail(RX_ENOMEM, "rx_set_start_draws");
    h->draw_base.n = 1;
  }
  h->draws = draws, h->n_draws = n_draws, h->draw_cursor = cursor;
  return RX_OK;
}

int rx_reset(rx_env* h, const uint8_t* mask, const rx_io* io, void* stream) {
  return launch(h, io, RX_MODE_RESET, mask, stream);
}

int rx_step(rx_env* h, const rx_io* io, void* stream) { return launch(h, io, RX_MODE_STEP, nullptr, stream); }

int rx_step_phases(rx_env* h, const rx_io* io, int32_t phases, void* stream) {
  return launch(h, io, RX_MODE_STEP, nullptr, stream, phases);
}

// ABI v21: n_steps steps from one call, each the launches of rx_step on its io rows.
static rx_io io_at(const rx_io* io, const rx_io_strides& st, int64_t s) {
  rx_io o = *io;
  o.actions = io->actions + s * st.actions;
  o.obs = io->obs + s * st.obs;
  if (io->reward) o.reward = io->reward + s * st.reward;
  if (io->reward64) o.reward64 = io->reward64 + s * st.reward64;
  if (io->terminated) o.terminated = io->terminated + s * st.terminated;
  if (io->truncated) o.truncated = io->truncated + s * st.truncated;
  if (io->done_f32) o.done_f32 = io->done_f32 + s * st.done_f32;
  if (io->info) o.info = io->info + s * st.info;
  if (io->ep_done) o.ep_done = io->ep_done + s * st.ep_done;
  return o;
}

int rx_steps(rx_env* h, const rx_io* io, int32_t n_steps, const rx_io_strides* strides, void* stream) {
  if (!h) return fail(RX_EINVAL, "null handle");
  if (!io) return fail(RX_EINVAL, "io is null");
  if (n_steps < 0) return fail(RX_EINVAL, "n_steps must be >= 0 (got %d)", n_steps);
  if (!io->obs || !io->actions) return fail(RX_EINVAL, "io->obs and io->actions are required");
  if (h->n_tracks <= 0 || !h->assigned || !h->bound)
    return fail(RX_ESTATE, "rx_steps needs rx_upload_tracks, rx_assign and rx_bind_state");
  const rx_io_strides st = strides ? *strides : rx_io_strides{};
  int rc;
  for (int32_t k = 0; k < n_steps; ++k) {
    const rx_io o = io_at(io, st, k);
    if ((rc = launch(h, &o, RX_MODE_STEP, nullptr, stream)) != 0) return rc;
  }
  return RX_OK;
}

// rx_rollout: the persistent small-N rollout (k_rollout) on a handle in the
// one-env-per-wave configuration; the per-step io pointers are set in-kernel.
static int max_waypoints(const rx_env* h) {
  int m = 0;
  for (int k = 0; k < h->n_tracks; ++k) m = std::max(m, h->wp_off_h[k + 1] - h->wp_off_h[k]);
  return m;
}

int rx_rollout_supported(const rx_env* h) {
  return h && h->assigned && h->bound && h->cfg.n_agents == 1 && h->dyn_lpe == 64 && (h->D == 15 || h->D == 19) &&
         max_waypoints(h) <= RX_ROLLOUT_MAX_W;
}

int rx_rollout(rx_env* h, const rx_io* io, const rx_rollout_io* r, void* stream) {
  if (!h || !io || !r) return fail(RX_EINVAL, "rx_rollout: null argument");
  if (!rx_rollout_supported(h))
    return fail(RX_ESTATE, "rx_rollout: needs an assigned, bound single-agent handle in the small-N (one env per "
                           "wave) configuration with 15 or 19 observation columns and <= %d waypoints per slot",
                RX_ROLLOUT_MAX_W);
  if (r->T <= 0) return fail(RX_EINVAL, "rx_rollout: T=%d must be > 0", r->T);
  if (r->obs_dim != h->D) return fail(RX_EINVAL, "rx_rollout: obs_dim %d != the handle's %d", r->obs_dim, h->D);
  if (!r->params || !r->log_std || !r->eps || !r->obs || !r->actions || !r->logprobs || !r->values || !r->rewards ||
      !r->dones || !r->next_obs || !r->next_done)
    return fail(RX_EINVAL, "rx_rollout: null rollout buffer");
  if (h->n_dyn_waves != h->cfg.n_envs) return fail(RX_ESTATE, "rx_rollout: expected one env per dynamics wave");
  rx_kargs a{};
  make_kargs(h, io, RX_MODE_STEP, nullptr, a);
  a.sort_keys = nullptr;
  a.tasks_out = nullptr;
  a.prof_ts = nullptr;
  int rc;
  if ((rc = rx_launch_rollout(&a, r, max_waypoints(h), (hipStream_t)stream)) != 0)
    return fail(RX_EHIP, "k_rollout launch failed: %s", hipGetErrorString((hipError_t)rc));
  return RX_OK;
}

int rx_rollout_steps(rx_env* h, const rx_io* io, const rx_rollout_io* r, int32_t precision, void* stream) {
  if (!h || !io || !r) return fail(RX_EINVAL, "rx_rollout_steps: null argument");
  if (!h->assigned || !h->bound) return fail(RX_ESTATE, "rx_rollout_steps: needs an assigned, bound handle");
  if (h->cfg.n_agents != 1) return fail(RX_EINVAL, "rx_rollout_steps: single-agent handles only");
  if (r->T <= 0) return fail(RX_EINVAL, "rx_rollout_steps: T=%d must be > 0", r->T);
  if (r->obs_dim != h->D) return fail(RX_EINVAL, "rx_rollout_steps: obs_dim %d != the handle's %d", r->obs_dim, h->D);
  if (!r->params || !r->log_std || !r->eps || !r->obs || !r->actions || !r->logprobs || !r->values || !r->rewards ||
      !r->dones || !r->next_obs || !r->next_done)
    return fail(RX_EINVAL, "rx_rollout_steps: null rollout buffer");
  if (precision != RX_PREC_FP32 && precision != RX_PREC_BF16)
    return fail(RX_EINVAL, "rx_rollout_steps: precision=%d (RX_PREC_FP32 or RX_PREC_BF16)", precision);
  const int64_t N = h->cfg.n_envs, D = h->D;
  // bf16: the parameters are fixed for the whole rollout, so their bf16 operand
  // fragments are built once (k_policy_frag) and every step's policy launch
  // reads them -- the same bf16 values rx_policy_act converts per use
  const void* frag = nullptr;
  if (precision == RX_PREC_BF16) {
    if (rx_launch_policy_frag(r->obs_dim, r->params, h->policy_frag.p, (hipStream_t)stream))
      return fail(RX_EHIP, "rx_rollout_steps: fragment launch failed");
    frag = h->policy_frag.p;
  }
  for (int32_t t = 0; t < r->T; ++t) {
    const bool last = t + 1 == r->T;
    const rx_policy_io pio{r->obs_dim, N, r->obs + t * N * D, r->eps + t * N * 2, r->params, r->log_std,
                           r->actions + t * N * 2, r->logprobs + t * N, r->values + t * N, 0, 0, precision,
                           nullptr, 0};
    int rc = rx_launch_policy_act(&pio, (hipStream_t)stream, frag);
    if (rc) return fail(RX_EHIP, "rx_rollout_steps: policy launch failed: %s", hipGetErrorString((hipError_t)rc));
    rx_io s = *io;
    s.actions = r->actions + t * N * 2;
    s.obs = last ? r->next_obs : r->obs + (t + 1) * N * D;
    s.reward = r->rewards + t * N;
    s.done_f32 = last ? r->next_done : r->dones + (t + 1) * N;
    if ((rc = launch(h, &s, RX_MODE_STEP, nullptr, stream)) != 0) return rc;
  }
  return RX_OK;
}

int rx_selfplay_rollout_steps(rx_env* h, const rx_io* io, const rx_rollout_io* r, const rx_selfplay_io* sp,
                              int32_t precision, void* stream) {
  if (!h || !io || !r || !sp) return fail(RX_EINVAL, "rx_selfplay_rollout_steps: null argument");
  if (!h->assigned || !h->bound) return fail(RX_ESTATE, "rx_selfplay_rollout_steps: needs an assigned, bound handle");
  if (h->cfg.n_agents != 2) return fail(RX_EINVAL, "rx_selfplay_rollout_steps: two-car handles only");
  if (r->T <= 0) return fail(RX_EINVAL, "rx_selfplay_rollout_steps: T=%d must be > 0", r->T);
  if (r->obs_dim != h->D) return fail(RX_EINVAL, "rx_selfplay_rollout_steps: obs_dim %d != the handle's %d", r->obs_dim, h->D);
  if (sp->agent != 0 && sp->agent != 1) return fail(RX_EINVAL, "rx_selfplay_rollout_steps: agent must be 0 or 1");
  if (!r->params || !r->log_std || !r->eps || !r->obs || !r->actions || !r->logprobs || !r->values || !r->rewards ||
      !r->dones || !r->next_obs || !r->next_done || !sp->opp_params || !sp->opp_log_std || !sp->opp_eps ||
      !sp->env_actions || !sp->env_obs || !sp->env_reward || !sp->sink)
    return fail(RX_EINVAL, "rx_selfplay_rollout_steps: null buffer");
  if (h->D != 19) return fail(RX_EINVAL, "rx_selfplay_rollout_steps: obs_dim %d (19)", h->D);
  if ((precision != RX_PREC_FP32 && precision != RX_PREC_BF16) ||
      (sp->opp_precision != RX_PREC_FP32 && sp->opp_precision != RX_PREC_BF16))
    return fail(RX_EINVAL, "rx_selfplay_rollout_steps: precision %d / opponent %d", precision, sp->opp_precision);
  const int64_t N = h->cfg.n_envs, D = h->D;
  const int q = sp->agent, o = 1 - q;
  hipStream_t hs = (hipStream_t)stream;
  for (int32_t t = 0; t < r->T; ++t) {
    const bool last = t + 1 == r->T;
    // ONE launch for both policies (k_selfplay_act): the frozen opponent's actor on
    // its rows of the env's observation buffer (wrappers.py:36-39), actions into its
    // slot of the env's action buffer; the learning agent on obs[t] -- the caller's
    // rows at t = 0 (they may predate an env rebuild), afterwards its rows of the
    // env's buffer, which the launch also copies into obs[t] together with the
    // agent's reward of step t - 1 -- actions into the rollout row and its env slot
    const rx_policy_io opp{(int32_t)D, N, sp->env_obs + o * D, sp->opp_eps + t * N * 2, sp->opp_params,
                           sp->opp_log_std, sp->env_actions + 2 * o, nullptr, sp->sink, 2 * D, 4,
                           sp->opp_precision, nullptr, 0};
    const rx_policy_io pio{(int32_t)D, N, t == 0 ? r->obs : sp->env_obs + q * D, r->eps + t * N * 2, r->params,
                           r->log_std, r->actions + t * N * 2, r->logprobs + t * N, r->values + t * N,
                           t == 0 ? 0 : 2 * D, 0, precision, sp->env_actions + 2 * q, 4};
    int rc = rx_launch_selfplay_act(&pio, &opp, t == 0 ? nullptr : r->obs + t * N * D, sp->env_reward,
                                    t == 0 ? nullptr : r->rewards + (t - 1) * N, q, hs);
    if (rc) return fail(RX_EHIP, "self-play policy launch failed: %s", hipGetErrorString((hipError_t)rc));
    rx_io s = *io;
    s.actions = sp->env_actions;
    s.obs = sp->env_obs;
    s.reward = sp->env_reward;
    s.done_f32 = last ? r->next_done : r->dones + (t + 1) * N;  // dones['__all__'] (wrappers.py:51)
    if ((rc = launch(h, &s, RX_MODE_STEP, nullptr, stream)) != 0) return rc;
  }
  // the last step's agent rows: next_obs and rewards[T - 1]
  const int rc = rx_launch_agent_rows((int)N, (int)D, q, sp->env_obs, sp->env_reward, r->next_obs,
                                      r->rewards + (r->T - 1) * N, hs);
  if (rc) return fail(RX_EHIP, "agent-row copy launch failed: %s", hipGetErrorString((hipError_t)rc));
  return RX_OK;
}

static int gae(int32_t T, int32_t N, const float* r, const float* v, const float* d, const float* nv, const float* nd,
               double gamma, double lam, float* adv, float* ret, int scan, void* stream) {
  if (T <= 0 || N <= 0) return fail(RX_EINVAL, "rx_gae: T=%d N=%d must be > 0", T, N);
  if (!r || !v || !d || !nv || !nd || !adv || !ret) return fail(RX_EINVAL, "rx_gae: null buffer");
  if ((long long)T * N > 0x7fffffffffffLL) return fail(RX_EINVAL, "rx_gae: T*N too large");
  // agent/ppo.py:149,151: c["gamma"] * nnt is float32(gamma) * nnt; the Python
  // double product gamma*lambda is rounded to float32 once.
  const float g = (float)gamma;
  const float gl = (float)(gamma * lam);
  const int rc = rx_launch_gae(T, N, r, v, d, nv, nd, g, gl, adv, ret, scan, (hipStream_t)stream);
  if (rc != 0) return fail(RX_EHIP, "gae launch failed: %s", hipGetErrorString((hipError_t)rc));
  return RX_OK;
}

int rx_gae(int32_t T, int32_t N, const float* r, const float* v, const float* d, const float* nv, const float* nd,
           double gamma, double lam, float* adv, float* ret, void* stream) {
  return gae(T, N, r, v, d, nv, nd, gamma, lam, adv, ret, 0, stream);
}

int rx_gae_scan(int32_t T, int32_t N, const float* r, const float* v, const float* d, const float* nv,
                const float* nd, double gamma, double lam, float* adv, float* ret, void* stream) {
  return gae(T, N, r, v, d, nv, nd, gamma, lam, adv, ret, 1, stream);
}

static int adam_cfg_error(const rx_adam_config* cfg) {
  if (!cfg) return fail(RX_EINVAL, "rx_adam: cfg is null");
  if (cfg->n_tensors <= 0 || cfg->n_tensors > RX_ADAM_MAX_TENSORS)
    return fail(RX_EINVAL, "rx_adam: n_tensors=%d not in [1, %d]", cfg->n_tensors, RX_ADAM_MAX_TENSORS);
  if (cfg->offsets[0] != 0) return fail(RX_EINVAL, "rx_adam: offsets[0] must be 0");
  for (int k = 0; k < cfg->n_tensors; ++k)
    if (cfg->offsets[k + 1] < cfg->offsets[k]) return fail(RX_EINVAL, "rx_adam: offsets not ascending");
  if (!(cfg->beta1 >= 0.0 && cfg->beta1 < 1.0 && cfg->beta2 >= 0.0 && cfg->beta2 < 1.0 && cfg->eps >= 0.0))
    return fail(RX_EINVAL, "rx_adam: bad betas/eps");
  return RX_OK;
}

size_t rx_adam_workspace_floats(const rx_adam_config* cfg) {
  if (adam_cfg_error(cfg) != RX_OK) return 0;
  const int64_t n = cfg->offsets[cfg->n_tensors];
  const int64_t nb = n > 0 ? (n + RX_ADAM_NORM_ELEMS - 1) / RX_ADAM_NORM_ELEMS : 1;
  return (size_t)(nb * cfg->n_tensors) + 2;  // + Adam's two step scalars
}

int rx_adam_clip_step(const rx_adam_config* cfg, float* params, float* grads, float* exp_avg, float* exp_avg_sq,
                      float* step, const double* lr, const uint8_t* stop, float* ws, void* stream) {
  if (const int rc = adam_cfg_error(cfg)) return rc;
  if (!params || !grads || !exp_avg || !exp_avg_sq || !step || !lr || !ws)
    return fail(RX_EINVAL, "rx_adam_clip_step: null buffer");
  const int rc = rx_launch_adam(cfg, params, grads, exp_avg, exp_avg_sq, step, lr, stop, ws, (hipStream_t)stream);
  if (rc != 0) return fail(RX_EHIP, "adam launch failed: %s", hipGetErrorString((hipError_t)rc));
  return RX_OK;
}

int rx_ppo_n_params(int32_t obs_dim);  // rx_ppo.hip

size_t rx_ppo_workspace_floats(int32_t obs_dim, int32_t mb) {
  return (obs_dim == 15 || obs_dim == 19) && mb > 0 ? rx_ppo_partial_floats(obs_dim, mb) : 0;
}

size_t rx_ppo_workspace_doubles(int32_t mb) { return mb > 0 ? (size_t)rx_ppo_n_wg(mb) : 0; }

static int check_ppo_batch(const rx_ppo_batch* b) {
  if (!b) return fail(RX_EINVAL, "rx_ppo: batch is null");
  if (b->obs_dim != 15 && b->obs_dim != 19) return fail(RX_EINVAL, "rx_ppo: obs_dim=%d (15 or 19)", b->obs_dim);
  if (b->mb <= 0 || b->n_rows <= 0) return fail(RX_EINVAL, "rx_ppo: mb=%d n_rows=%lld", b->mb, (long long)b->n_rows);
  if (b->precision != RX_PREC_FP32 && b->precision != RX_PREC_BF16)
    return fail(RX_EINVAL, "rx_ppo: precision=%d (RX_PREC_FP32 or RX_PREC_BF16)", b->precision);
  if (!b->obs || !b->actions || !b->logprobs || !b->advantages || !b->returns || !b->values || !b->perm ||
      !b->params || !b->log_std)
    return fail(RX_EINVAL, "rx_ppo: null buffer");
  return RX_OK;
}

int rx_ppo_adv_stats(const rx_ppo_batch* b, int32_t n_mb, float* stats, void* stream) {
  int rc = check_ppo_batch(b);
  if (rc) return rc;
  if (n_mb <= 0 || !stats) return fail(RX_EINVAL, "rx_ppo_adv_stats: n_mb=%d stats=%p", n_mb, (void*)stats);
  if ((int64_t)n_mb * b->mb > b->n_rows) return fail(RX_EINVAL, "rx_ppo_adv_stats: n_mb*mb > n_rows");
  if ((rc = rx_launch_adv_stats(b, n_mb, stats, nullptr, (hipStream_t)stream)) != 0)
    return fail(RX_EHIP, "adv stats launch failed: %s", hipGetErrorString((hipError_t)rc));
  return RX_OK;
}

int rx_ppo_adv_moments(const rx_ppo_batch* b, int32_t n_mb, double* moments, void* stream) {
  int rc = check_ppo_batch(b);
  if (rc) return rc;
  if (n_mb <= 0 || !moments) return fail(RX_EINVAL, "rx_ppo_adv_moments: n_mb=%d moments=%p", n_mb, (void*)moments);
  if ((int64_t)n_mb * b->mb > b->n_rows) return fail(RX_EINVAL, "rx_ppo_adv_moments: n_mb*mb > n_rows");
  if ((rc = rx_launch_adv_stats(b, n_mb, nullptr, moments, (hipStream_t)stream)) != 0)
    return fail(RX_EHIP, "adv moments launch failed: %s", hipGetErrorString((hipError_t)rc));
  return RX_OK;
}

size_t rx_ppo_adv_workspace_doubles(int32_t mb, int32_t n_mb) {
  return mb > 0 && n_mb > 0 ? 2 * (size_t)n_mb * (size_t)rx_adv_chunks(mb) : 0;
}

int rx_ppo_adv_stats_ws(const rx_ppo_batch* b, int32_t n_mb, double* ws, float* stats, double* moments, void* stream) {
  int rc = check_ppo_batch(b);
  if (rc) return rc;
  if (n_mb <= 0 || !ws || (!stats && !moments))
    return fail(RX_EINVAL, "rx_ppo_adv_stats_ws: n_mb=%d ws=%p stats=%p moments=%p", n_mb, (void*)ws, (void*)stats,
                (void*)moments);
  if ((int64_t)n_mb * b->mb > b->n_rows) return fail(RX_EINVAL, "rx_ppo_adv_stats_ws: n_mb*mb > n_rows");
  if ((rc = rx_launch_adv_stats_ws(b, n_mb, ws, moments ? nullptr : stats, moments, (hipStream_t)stream)) != 0)
    return fail(RX_EHIP, "adv stats launch failed: %s", hipGetErrorString((hipError_t)rc));
  return RX_OK;
}

int rx_ppo_adv_finalize(const double* moments, int32_t n_mb, int64_t count, float* stats, void* stream) {
  if (n_mb <= 0 || count <= 0 || !moments || !stats)
    return fail(RX_EINVAL, "rx_ppo_adv_finalize: n_mb=%d count=%lld moments=%p stats=%p", n_mb, (long long)count,
                (const void*)moments, (void*)stats);
  const int rc = rx_launch_adv_finalize(moments, n_mb, count, stats, (hipStream_t)stream);
  if (rc != 0) return fail(RX_EHIP, "adv finalize launch failed: %s", hipGetErrorString((hipError_t)rc));
  return RX_OK;
}

int rx_ppo_minibatch_grad(const rx_ppo_batch* b, int32_t m, float* ws_f32, double* ws_f64, float* grad,
                          uint8_t* stop, float* kl_at_stop, void* stream) {
  int rc = check_ppo_batch(b);
  if (rc) return rc;
  if (!b->adv_stats) return fail(RX_EINVAL, "rx_ppo_minibatch_grad: adv_stats is null");
  if (m < 0 || (int64_t)(m + 1) * b->mb > b->n_rows) return fail(RX_EINVAL, "rx_ppo_minibatch_grad: m=%d out of range", m);
  if (!ws_f32 || !ws_f64 || !grad || !stop || !kl_at_stop) return fail(RX_EINVAL, "rx_ppo_minibatch_grad: null buffer");
  if ((rc = rx_launch_ppo_grad(b, m, 1.0f, stop, kl_at_stop, nullptr, ws_f32, ws_f64, grad, (hipStream_t)stream)) != 0)
    return fail(RX_EHIP, "ppo grad launch failed: %s", hipGetErrorString((hipError_t)rc));
  return RX_OK;
}

size_t rx_ppo_update_workspace_floats(int32_t obs_dim, const rx_adam_config* cfg) {
  if ((obs_dim != 15 && obs_dim != 19) || adam_cfg_error(cfg) != RX_OK) return 0;
  // the per-tensor sums of squares of every reduce block + Adam's two step scalars
  return (size_t)rx_ppo_reduce_blocks(obs_dim) * cfg->n_tensors + 2;
}

int rx_ppo_minibatch_update(const rx_ppo_batch* b, int32_t m, const rx_adam_config* cfg, float* params,
                            float* ws_f32, double* ws_f64, float* grad, float* exp_avg, float* exp_avg_sq, float* step,
                            const double* lr, uint8_t* stop, float* kl_at_stop, float* adam_ws, void* stream) {
  int rc = check_ppo_batch(b);
  if (rc) return rc;
  if ((rc = adam_cfg_error(cfg))) return rc;
  if (!b->adv_stats) return fail(RX_EINVAL, "rx_ppo_minibatch_update: adv_stats is null");
  if (m < 0 || (int64_t)(m + 1) * b->mb > b->n_rows)
    return fail(RX_EINVAL, "rx_ppo_minibatch_update: m=%d out of range", m);
  if (!params || params != b->params) return fail(RX_EINVAL, "rx_ppo_minibatch_update: params must be b->params");
  if (cfg->offsets[cfg->n_tensors] != rx_ppo_n_params(b->obs_dim))
    return fail(RX_EINVAL, "rx_ppo_minibatch_update: cfg covers %lld parameters, the policy has %d",
                (long long)cfg->offsets[cfg->n_tensors], rx_ppo_n_params(b->obs_dim));
  if (!ws_f32 || !ws_f64 || !grad || !exp_avg || !exp_avg_sq || !step || !lr || !stop || !kl_at_stop || !adam_ws)
    return fail(RX_EINVAL, "rx_ppo_minibatch_update: null buffer");
  const hipStream_t s = (hipStream_t)stream;
  if ((rc = rx_launch_ppo_grad(b, m, 1.0f, stop, kl_at_stop, nullptr, ws_f32, ws_f64, grad, s, cfg, adam_ws, step, lr)))
    return fail(RX_EHIP, "ppo grad launch failed: %s", hipGetErrorString((hipError_t)rc));
  if ((rc = rx_launch_adam_apply(cfg, params, grad, exp_avg, exp_avg_sq, step, lr, stop, adam_ws,
                                 rx_ppo_reduce_blocks(b->obs_dim), s)))
    return fail(RX_EHIP, "adam launch failed: %s", hipGetErrorString((hipError_t)rc));
  return RX_OK;
}

int rx_ppo_minibatch_grad_shard(const rx_ppo_batch* b, int32_t m, float scale, float* ws_f32, double* ws_f64,
                                float* grad, float* kl_out, const uint8_t* stop, void* stream) {
  int rc = check_ppo_batch(b);
  if (rc) return rc;
  if (!b->adv_stats) return fail(RX_EINVAL, "rx_ppo_minibatch_grad_shard: adv_stats is null");
  if (m < 0 || (int64_t)(m + 1) * b->mb > b->n_rows)
    return fail(RX_EINVAL, "rx_ppo_minibatch_grad_shard: m=%d out of range", m);
  if (!(scale > 0.0f)) return fail(RX_EINVAL, "rx_ppo_minibatch_grad_shard: scale=%g", (double)scale);
  if (!ws_f32 || !ws_f64 || !grad || !kl_out || !stop)
    return fail(RX_EINVAL, "rx_ppo_minibatch_grad_shard: null buffer");
  // the kernels only read *stop in shard mode (the decision is rx_ppo_kl_check's)
  if ((rc = rx_launch_ppo_grad(b, m, scale, const_cast<uint8_t*>(stop), nullptr, kl_out, ws_f32, ws_f64, grad,
                               (hipStream_t)stream)) != 0)
    return fail(RX_EHIP, "ppo grad launch failed: %s", hipGetErrorString((hipError_t)rc));
  return RX_OK;
}

int rx_random_permutation(int64_t n, uint64_t seed, int64_t* out, void* stream) {
  if (n < 0 || n > (1ll << 62)) return fail(RX_EINVAL, "rx_random_permutation: n = %lld out of range", (long long)n);
  if (n > 0 && !out) return fail(RX_EINVAL, "rx_random_permutation: null output");
  const int rc = rx_launch_permutation(n, seed, out, (hipStream_t)stream);
  if (rc) return fail(RX_EHIP, "rx_random_permutation launch failed: %s", hipGetErrorString((hipError_t)rc));
  return RX_OK;
}

int rx_ppo_kl_check(const float* kl, float kl_target, uint8_t* stop, float* kl_at_stop, void* stream) {
  if (!kl || !stop || !kl_at_stop) return fail(RX_EINVAL, "rx_ppo_kl_check: null buffer");
  const int rc = rx_launch_kl_check(kl, kl_target, stop, kl_at_stop, (hipStream_t)stream);
  if (rc != 0) return fail(RX_EHIP, "kl check launch failed: %s", hipGetErrorString((hipError_t)rc));
  return RX_OK;
}

int rx_policy_act(const rx_policy_io* io, void* stream) {
  if (!io) return fail(RX_EINVAL, "rx_policy_act: io is null");
  if (io->obs_dim != 15 && io->obs_dim != 19) return fail(RX_EINVAL, "rx_policy_act: obs_dim=%d (15 or 19)", io->obs_dim);
  if (io->n <= 0) return fail(RX_EINVAL, "rx_policy_act: n=%lld", (long long)io->n);
  if (io->precision != RX_PREC_FP32 && io->precision != RX_PREC_BF16)
    return fail(RX_EINVAL, "rx_policy_act: precision=%d (RX_PREC_FP32 or RX_PREC_BF16)", io->precision);
  if ((io->obs_stride != 0 && io->obs_stride < io->obs_dim) || (io->act_stride != 0 && io->act_stride < 2) ||
      (io->act2_stride != 0 && io->act2_stride < 2))
    return fail(RX_EINVAL, "rx_policy_act: row strides overlap (obs %lld, act %lld)", (long long)io->obs_stride,
                (long long)io->act_stride);
  if (!io->obs || !io->eps || !io->params || !io->log_std || !io->actions || !io->logprobs || !io->values)
    return fail(RX_EINVAL, "rx_policy_act: null buffer");
  const int rc = rx_launch_policy_act(io, (hipStream_t)stream);
  if (rc != 0) return fail(RX_EHIP, "policy launch failed: %s", hipGetErrorString((hipError_t)rc));
  return RX_OK;
}

}  // extern "C"
