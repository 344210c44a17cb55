// rx_internal.h -- kernel argument block shared by rx_api.cpp (host) and
// rx_kernels.hip (device).  Not part of the public ABI (include/rx.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rx.h"

#define RX_MODE_STEP 0
#define RX_MODE_RESET 1

// One wavefront's work item: 64 consecutive tasks of ONE track slot.
//  dyn waves: lane -> env perm[perm_start + lane], lane < count
//  ray waves: lane -> task task_start + lane (task = env_local*A*R + agent*R + ray),
//             env = perm[perm_start + env_local]
struct rx_wave {
  int32_t track;
  int32_t perm_start;
  int32_t task_start;
  int32_t count;
};

// Every per-slot scalar the lane-varying kernels read, in ONE 128-byte record (one
// cache line per env instead of one per table: the slot's waypoint range, its culling
// table offsets, bounding circle and meta).  Built by rx_upload_tracks.
struct rx_slot_hdr {
  int32_t wp0, W, chunk_off, super_off, wchunk_off, wsuper_off, pad0, pad1;
  double geo[4];   // slot_geo: bounding-circle centre x, y, radius, longest segment
  double meta[8];  // rx_upload_tracks meta row
};
static_assert(sizeof(rx_slot_hdr) == 128, "one cache line per slot");

struct rx_track_view {
  const int32_t* wp_off;     // [n+1]
  const double* wp;          // [Wtot][2]
  const double* nrm;         // [Wtot][2]
  const double* seg;         // [2*Wtot][4]
  const double* meta;        // [n][8]
  // raycast culling (derived by rx_upload_tracks)
  const int32_t* chunk_off;  // [n+1] first chunk of each slot (2*ceil(W/G) chunks per slot: left side, right side)
  const double* chunk_box;   // [n_chunks][4] xmin, ymin, xmax, ymax of the chunk's segment end points
  const double* slot_geo;    // [n][4] bounding-circle centre x, y, radius of all boundary points; max |v2|
  // closest-waypoint culling: chunks of RX_WP_CHUNK consecutive waypoints
  const int32_t* wchunk_off; // [n+1]
  const double* wchunk_box;  // [n_wchunks][4]
  // two-level raycast culling: super-chunks of cull_super consecutive chunks
  const int32_t* super_off;  // [n+1] first super-chunk of each slot (both sides)
  const double* super_box;   // [n_super][4] union of the member chunk boxes
  // closest-waypoint super-chunks: RX_WP_SUPER consecutive waypoint chunks
  const int32_t* wsuper_off; // [n+1]
  const double* wsuper_box;  // [n_wsuper][4]
  const float* chunk_box_f;  // chunk_box / super_box in float32, rounded outward (k_rays' packed-f32 box tests),
  const float* super_box_f;  // then 4 quadrant blocks of (near.x, near.y, far.x, far.y) (rx_api.cpp)
  int32_t n_chunk_boxes;     // boxes per block
  int32_t n_super_boxes;
  const float* seg_f;        // [2*Wtot][4] float32 copy of seg (culled raycast: segment pre-filter)
  const rx_slot_hdr* hdr;    // [n] per-slot header (lane-varying kernels)
};

#ifndef RX_WP_CHUNK
#define RX_WP_CHUNK 8  // waypoints per closest-waypoint culling leaf
#endif
#ifndef RX_WP_SUPER
#define RX_WP_SUPER 4  // leaves per waypoint super-chunk
#endif

// lanes per env in k_dyn1 (a dynamics wave holds 64 / lpe envs): 4 when there
// are few envs (latency-bound: more lanes per env shorten the chain), 1 when
// the chip is fuller.  One lane per env also selects the split step (k_kin1 +
// k_step2: the REWARD half beside the raycast), which beats k_dyn1<4> + k_rays
// from 4,096 envs on (41.4 vs 52.8 us at 4,096, 42.7 vs 54.3 at 8,192; equal
// at 2,048, where the wide kernels run anyway: tools/gpu_lpe_ab.sh)
#define RX_DYN1_LPE_SMALL 4
#define RX_DYN1_SMALL_N 2048
// Lanes per ray task (ray_order 2): 4 (16 tasks a ray wave) up to
// RX_RAY_LPR4_N (env, agent) pairs, 2 up to RX_RAY_LPR2_N, 1 above: with few
// envs the raycast is a latency chain over too few waves to fill the chip
// ("Lanes per ray"; crossovers measured on MI355X)
#ifndef RX_RAY_LPR4_N
#define RX_RAY_LPR4_N 8192
#endif
#ifndef RX_RAY_LPR2_N
#define RX_RAY_LPR2_N 16384
#endif
// k_step2<1>'s REWARD half at 2 lanes per env up to this many envs (it is the
// launch's critical path there once the raycast runs at 4 lanes per ray;
// from 8,192 envs on it only slows the raycast beside it)
#ifndef RX_REWARD_LPE2_N
#define RX_REWARD_LPE2_N 4096
#endif
// two-car envs: k_step2<2>'s REWARD half with a lane per car (one closest-waypoint
// pass per wave instead of two) up to this many envs.  Same-session A/B
// (profiles/r04/ab_two_car_*.jsonl): 4,096 envs 67.2 -> 79.2 M env-steps/s,
// 8,192 128.1 -> 134.7 M (with one lane per ray), 16,384 213.2 -> 220.3 M,
// 65,536 389 -> 387 M (off there)
#ifndef RX_REWARD2_LPE2_N
#define RX_REWARD2_LPE2_N 16384
#endif
// two-car envs: 2 lanes per ray only up to this many (env, car) pairs (the
// single-agent RX_RAY_LPR2_N band is empty for them: with the REWARD half at a
// lane per car, 8,192 envs run 134.7 M at 1 lane per ray vs 128.6 M at 2)
#ifndef RX_RAY2_LPR2_N
#define RX_RAY2_LPR2_N 8192
#endif
// Ray-wave dispatch order (rx_assign's placement of the ray-wave table, ray_order 2).
// Class j of a 64-env group = its j-th wave of direction-sorted tasks (the cars of a
// group head alike, so class j ~ sensor ray j: the edge classes look sideways, the
// centre ones down the track and cost ~1.3x).  0 = group-octet-major (round 2),
// 1 = class-major centre classes first, 2 = class-major ascending j, 3 = class-major
// EDGE classes first, the centre ones last (default: 65,536 envs 752 -> 826-833 M
// env-steps/s, 4,096 envs +3 %, same session, DESIGN.md §3 "Ray-wave dispatch order").
#ifndef RX_RAY_DISPATCH
#define RX_RAY_DISPATCH 3
#endif
// rx_config.ray_tail / ray_tail_lpr automatic values: the last RX_RAY_TAIL classes of the
// dispatch order cast at RX_RAY_TAIL_LPR lanes per ray (0 = no tail split)
#ifndef RX_RAY_TAIL
#define RX_RAY_TAIL 0
#endif
#ifndef RX_RAY_TAIL_LPR
#define RX_RAY_TAIL_LPR 2
#endif
// rx_config.task_sort automatic value: the ray-task direction sort every other
// dynamics launch up to this many (env, car) pairs, every launch above.  Same-session
// A/B (profiles/r04/ab_task_sort.txt): 4,096 single-agent envs 129.8 / 128.9 ->
// 132.3 / 132.7 M env-steps/s (k_kin1 6.2 -> 3.6 us), 8,192 two-car envs 135.1 / 136.7
// -> 137.2 / 138.8 M; 65,536 envs 833 -> 804-810 M (every 4th / 8th: 761 / 715 M) and
// 65,536 two-car envs -0.5 %: the stale order costs more ray work than the sort
#ifndef RX_TASK_SORT2_PAIRS
#define RX_TASK_SORT2_PAIRS 16384
#endif
// at most this many single-agent envs: one env per dynamics wave and one ray
// per raycast wave (k_rays_wide), brute force over the lanes -- the kernels
// are latency chains there, and 64 lanes shorten them
#define RX_WIDE_N 2048

struct rx_kargs {
  rx_track_view tr;
  rx_state st;                // the engine's working state, position order (element A*p + q is agent q of
                              // env perm[p]); track and speed_weight are the caller's (env order)
  rx_io io;
  const rx_wave* dyn_waves;
  const rx_wave* ray_waves;
  const int32_t* perm;        // env order the kernels read (sorted by slot, then position)
  const double* rel_angles;   // [n_sensors]
  const uint8_t* reset_mask;  // RX_MODE_RESET: [N] or nullptr (= all)
  uint32_t* sort_keys;        // [N] k_dyn writes the sort bin (sort_base[slot] + (waypoint >> sort_shift)) at its perm position, or nullptr
  uint32_t* sort_hist;        // with sort_keys: the REWARD half also counts the bins (the re-sort then skips k_sort_hist), or nullptr
  uint32_t* sort_off;         // with sort_hist: [N] the position's rank within its bin (the count atomic's return + lane rank)
  const int32_t* sort_base;   // [n_tracks] first sort bin of each slot (ascending with the slot id)
  int32_t sort_shift;         // waypoints per sort bin = 1 << sort_shift
  // ray_order 2: k_dyn writes the direction-sorted (agent, ray) task ids of
  // each dynamics wave's envs to tasks_out[perm_start*A*R ..]; k_rays reads
  // tasks[task_start + lane] (the same buffer)
  int32_t* tasks_out;
  const int32_t* tasks;
  int32_t n_dyn_waves;
  int32_t n_ray_waves;
  int32_t n_sensors;
  int32_t D;
  int32_t max_steps;
  int32_t autoreset;
  int32_t mode;
  int32_t cull_chunk;         // segments per culling chunk G (0 = brute force over all segments)
  int32_t ray_order;          // rx_config.ray_order
  int32_t cull_super;         // leaves per super-chunk (0 = one-level culling)
  int32_t dyn_lpe;            // k_dyn1 lanes per env (1 or RX_DYN1_LPE_SMALL)
  int32_t argmin_window;      // half-width of the closest-waypoint scan around the previous one
  int32_t wide;               // small N: k_dyn1 one env per wave (dyn_lpe 64), k_rays_wide one ray per wave
  int32_t n_wide_tasks;       // N * A * R ray tasks of k_rays_wide
  double* cs_scratch;         // split step: [N*A][2] cos / sin of the stepped angle, k_kin -> k_step2
  unsigned long long* prof_ts;  // rx_profile: [2][prof_stride] per-wave start / end wall-clock stamps, or nullptr
  int32_t prof_stride;          // waves per stamp array (>= waves of any launch)
  const int32_t* slot_nenv;   // [n_tracks] envs assigned to each slot (ray-major task decode)
  double speed_weight;
  uint64_t seed;
  uint32_t* reset_count;  // [N] (2-car envs), advanced by k_dyn2 at every reset
  int32_t box_quadrants;  // k_rays: single-quadrant waves use the quadrant-ordered box tables (RX_BOX_QUAD=0: off)
  int32_t seg_filter;     // k_rays: float32 pre-filter before each exact segment test (RX_SEG_FILTER=0: off)
  int32_t ray_lpr;        // culled raycast: lanes per ray task (1; 4 for few envs, 16 tasks a ray wave)
  int32_t reward_lpe;     // k_step2<1> REWARD half: lanes per env (1, 2 or 4; more for few envs)
  int32_t lane_tracks;    // lane-varying slots (rx_config.lane_tracks): waves of 64 positions of any slots
  const int32_t* pos_slot;  // with lane_tracks: [N] the slot of the env at each position (the order is fixed)
  int32_t ray_tail_from;  // ray waves >= this one (the dispatch tail) hold 64 / ray_tail_lpr tasks each, cast at
  int32_t ray_tail_lpr;   // ray_tail_lpr lanes per ray (2 or 4); -1 = no tail split (rx_config.ray_tail)
  // rx_set_start_draws (two-car envs): the start-slot order of the env that is the
  // j-th to reset in this launch, in env order, comes from draws[*draw_base + j]
  // (j = reset_rank[e], k_reset_rank) instead of the device hash; nullptr = hash
  const uint32_t* draws;
  int64_t n_draws;
  const int64_t* draw_base;
  const int32_t* reset_rank;
};

extern "C" int rx_launch_step(const rx_kargs* a, int n_agents, int phases, hipStream_t s);
// split step (STEP mode, next-step / no autoreset): k_kin1 / k_kin2, then k_step2<A>
#define RX_SPLIT_KIN 0
#define RX_SPLIT_REWARD 1
#define RX_SPLIT_REWARD_RAYS 2
extern "C" int rx_launch_split(const rx_kargs* a, int n_agents, int part, hipStream_t s);
// persistent small-N rollout (k_rollout): a->n_dyn_waves workgroups, one env
// each, its slot staged in max_w * 96 bytes of dynamic LDS
#define RX_ROLLOUT_MAX_W 1024
extern "C" int rx_launch_rollout(const rx_kargs* a, const rx_rollout_io* r, int max_w, hipStream_t s);
// rx_set_start_draws: ranks (env order) of the envs the next dynamics launch resets
// (mode RX_MODE_RESET: mask[e] or all; RX_MODE_STEP: the next-step autoreset flag of
// the env's working-state row), *base = cursor[0], cursor[0] += their count,
// cursor[1] += the draws missing when the count overruns n_draws
extern "C" int rx_launch_reset_rank(int N, int mode, const uint8_t* mask, const uint8_t* env_flags, const int32_t* perm,
                                    int32_t* tmp, int32_t* rank, int64_t* cursor, int64_t* base, int64_t n_draws,
                                    hipStream_t s);
extern "C" int rx_launch_agent_rows(int N, int D, int q, const float* obs, const float* rew, float* obs_out,
                                    float* rew_out, hipStream_t s);
extern "C" int rx_launch_gae(int T, int N, const float* r, const float* v, const float* d, const float* nv,
                             const float* nd, float g, float gl, float* adv, float* ret, int scan, hipStream_t s);
// Adam's per-step scalars for step count s (torch.optim.Adam, non-capturable):
// out[0] = step_size = -lr / (1 - beta1^s), out[1] = sqrt(1 - beta2^s).  Written
// once per optimizer step next to the clip-norm partials (rx_adam_workspace_floats
// counts the 2 floats) by the launch that bumps the step count.
__device__ __forceinline__ void rx_adam_scalars(const rx_adam_config& cfg, float step, double lr, float* out) {
  const double s = (double)step;
  out[0] = (float)(-(lr / (1.0 - pow(cfg.beta1, s))));
  out[1] = (float)sqrt(1.0 - pow(cfg.beta2, s));
}
// torch.optim.Adam's element update (foreach, non-capturable) after the clip
// coefficient: g *= coef; m = lerp(m, g, 1-b1); v = v*b2 + (1-b2)*g*g;
// p += step_size * m / (sqrt(v)/bc2_sqrt + eps).  ONE definition for
// k_adam_apply (rx_optim.hip) and the fused minibatch tail (rx_ppo.hip), so both
// optimizer paths round every element identically.
__device__ __forceinline__ void rx_adam_elem(float& g, float& m, float& v, float& p, float coef, float w1, float fb2,
                                             float w2, float eps, float step_size, float bc2_sqrt) {
  g = g * coef;
  m = m + w1 * (g - m);  // torch.lerp, weight < 0.5 branch
  v = v * fb2;
  v = v + w2 * g * g;
  const float den = sqrtf(v) / bc2_sqrt + eps;
  p = p + step_size * (m / den);
}
// The re-sort's bin count for the wave's calling lanes (one per env, key =
// its bin): lanes grouped by bin (ballot), then ONE vector atomic in which
// every group leader adds its group size to hist[bin]; the returned old count
// plus the lane's rank inside its group is the env's rank within its bin --
// the scatter's offset, so k_sort_scatter needs no atomics of its own.
__device__ __forceinline__ uint32_t rx_bin_count(uint32_t* hist, uint32_t key) {
  const int lane = (int)(threadIdx.x & 63);
  unsigned long long pending = __ballot(1);
  uint32_t cnt = 0, rank = 0;
  int leader_of_mine = lane;
  while (pending) {  // wave-uniform: one iteration per distinct bin of the wave
    const int leader = __builtin_ctzll(pending);
    const uint32_t lb = (uint32_t)__builtin_amdgcn_readlane((int)key, leader);
    const unsigned long long m = __ballot(key == lb);
    if (key == lb) {
      leader_of_mine = leader;
      rank = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    }
    if (lane == leader) cnt = (uint32_t)__builtin_popcountll(m);
    pending &= ~m;
  }
  uint32_t old = 0;
  if (cnt) old = atomicAdd(&hist[key], cnt);
  old = (uint32_t)__builtin_amdgcn_ds_bpermute(leader_of_mine << 2, (int)old);
  return old + rank;
}
extern "C" int rx_launch_adam(const rx_adam_config* cfg, float* p, float* g, float* m, float* v, float* step,
                              const double* lr, const uint8_t* stop, float* ws, hipStream_t s);
extern "C" size_t rx_ppo_partial_floats(int obs_dim, int mb);
extern "C" int rx_ppo_n_wg(int mb);
// frag: NULL, or (bf16) the rollout's fragment image from rx_launch_policy_frag
extern "C" int rx_launch_policy_act(const rx_policy_io* io, hipStream_t s, const void* frag = nullptr);
extern "C" size_t rx_policy_frag_bytes();
extern "C" int rx_launch_policy_frag(int obs_dim, const float* params, void* img, hipStream_t s);
// both self-play policies of a rollout step in one launch (obs_dim 19; k_selfplay_act)
extern "C" int rx_launch_selfplay_act(const rx_policy_io* ag, const rx_policy_io* op, float* obs_out,
                                      const float* rew_src, float* rew_out, int agent, hipStream_t s);
extern "C" int rx_launch_adv_stats(const rx_ppo_batch* b, int n_mb, float* stats, double* moments, hipStream_t s);
extern "C" int rx_adv_chunks(int mb);
extern "C" int rx_launch_adv_stats_ws(const rx_ppo_batch* b, int n_mb, double* ws, float* stats, double* moments,
                                      hipStream_t s);
extern "C" int rx_launch_adv_finalize(const double* moments, int n_mb, int64_t count, float* stats, hipStream_t s);
extern "C" int rx_launch_kl_check(const float* kl, float kl_target, uint8_t* stop, float* kl_at_stop, hipStream_t s);
extern "C" int rx_launch_ppo_grad(const rx_ppo_batch* b, int m, float scale, uint8_t* stop, float* kl_at_stop,
                                  float* kl_out, float* partial, double* klp, float* grad, hipStream_t s,
                                  const rx_adam_config* cfg = nullptr, float* norm_ws = nullptr,
                                  float* step = nullptr, const double* lr = nullptr);
extern "C" int rx_ppo_reduce_blocks(int obs_dim);
extern "C" int rx_launch_adam_apply(const rx_adam_config* cfg, float* p, float* g, float* m, float* v, float* step,
                                    const double* lr, const uint8_t* stop, float* ws, int nb, hipStream_t s);
// spatial re-sort (rx_sort.hip): counting sort of the perm positions by the
// bin keys the REWARD half wrote; hist must be zero on entry and is left zero
#define RX_SORT_MAX_BINS 65536
// and moves the working state rows with their envs (perm, work -> perm_tmp,
// tmp -> back); rx_state_sync: working copy <-> the caller's arrays
extern "C" int rx_sort_envs(const uint32_t* keys, uint32_t* off, int n, int A, uint32_t* hist, uint32_t* cursor, int nbins,
                            int32_t* perm, int32_t* perm_tmp, const rx_state* work, const rx_state* tmp,
                            hipStream_t s, int hist_done = 0);
extern "C" int rx_launch_permutation(int64_t n, uint64_t seed, int64_t* out, hipStream_t s);
extern "C" int rx_state_sync(const rx_state* work, const rx_state* user, const int32_t* perm, int n, int A,
                             int to_user, hipStream_t s);
