/* rx.h -- C ABI of the MI355X racing-env engine (librx.so).
 *
 * The reference (LucasHJin/self-play-racing) is pure Python and has no FFI; its
 * hot path is the per-env Gymnasium step loop that agent/ppo.py drives through
 * gymnasium.vector.SyncVectorEnv.  This header is the boundary a maintainer
 * binds (ctypes stub: INTEGRATION.md) to replace that loop with one batched
 * device call.  Each entry point names the reference interface it replaces.
 *
 * Conventions
 *  - Every function returns RX_OK (0) or a negative RX_E* code; rx_last_error()
 *    returns a thread-local message for the last failure on this thread.
 *  - "dev" pointers are device memory owned by the CALLER (e.g. torch tensors);
 *    the library never frees them.  Host arrays are read during the call only.
 *  - Work is enqueued on the caller's stream (a hipStream_t passed as void*,
 *    NULL = the legacy default stream) with no host synchronisation, so the
 *    step can sit inside a captured hipGraph.
 *  - One host thread per handle; handles are independent (one per GPU rank).
 *  - Agents: A = 1 (environment/racing_env.py RacingEnv) or A = 2
 *    (environment/multi_racing_env.py MultiRacingEnv with 2 cars).
 *    Observation width D = n_sensors + 4 + 4*(A-1)   (racing_env.py:37-42,
 *    multi_racing_env.py:38).
 *  - All env arithmetic is binary64 in the reference's operation order; see
 *    DESIGN.md §Parity for the two libm calls (sin/cos, pow(x,2)) whose
 *    results may differ from glibc's by 1 ulp.
 */
#ifndef RX_H_
#define RX_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RX_OK 0
#define RX_EINVAL (-1)   /* bad argument / shape / state */
#define RX_EHIP (-2)     /* HIP runtime error */
#define RX_ENOMEM (-3)   /* device allocation failed */
#define RX_ESTATE (-4)   /* call order: tracks/assignment/state not set */

#define RX_ABI_VERSION 23
#define RX_EP_SHARDS 64  /* episode-statistics accumulator rows (rx_io.ep_stats) */

/* state flag bits (rx_state.flags, per agent) */
#define RX_F_CRASHED 1u      /* Car.crashed                      car.py:22,80 */
#define RX_F_FINISHED 2u     /* Car.finished                     racing_env.py:147 */
#define RX_F_CP25 4u         /* checkpoints[0.25]                racing_env.py:21-25 */
#define RX_F_CP50 8u         /* checkpoints[0.50] */
#define RX_F_CP75 16u        /* checkpoints[0.75] */
#define RX_F_HAS_CRASHED 32u /* agents_data['has_crashed']       multi_racing_env.py:147,192-194 */
/* env flag bits (rx_state.env_flags, per env) */
#define RX_EF_PENDING_RESET 1u /* episode ended last step: next-step autoreset */

/* autoreset modes (gymnasium 1.x SyncVectorEnv: NEXT_STEP is its default) */
#define RX_AUTORESET_NEXT_STEP 0 /* step after a terminal one resets, reward 0 */
#define RX_AUTORESET_SAME_STEP 1 /* terminal step returns the reset obs (SB3 style) */
#define RX_AUTORESET_DISABLED 2  /* caller resets explicitly (rx_reset) */

/* info columns (rx_io.info, f64 [N][A][RX_INFO_W]) */
#define RX_INFO_W 4
#define RX_INFO_SPEED 0          /* info['speed']          racing_env.py:80 */
#define RX_INFO_PROGRESS 1       /* info['progress'] (1.0 once finished) :81,158-159 */
#define RX_INFO_PROGRESS_DELTA 2 /* info['progress_delta'] :157 (single-agent) */
#define RX_INFO_PLACEMENT 3      /* info['placement'] (0 = none) multi_racing_env.py:210-211,252-259 */

typedef struct rx_env rx_env;

typedef struct {
  int32_t n_envs;          /* N */
  int32_t n_agents;        /* A: 1 or 2 */
  int32_t n_sensors;       /* rays per agent (11 in train.py:47-49,94-101) */
  int32_t max_steps;       /* truncation, 3000 (racing_env.py:162) */
  int32_t autoreset;       /* RX_AUTORESET_* */
  int32_t device;          /* HIP device ordinal */
  uint64_t seed;           /* device RNG (two-car start-slot shuffle) */
  double sensor_half_cone; /* pi/3 (racing_env.py:45) or pi/2 (multi_racing_env.py:50) */
  double speed_weight;     /* RacingEnv.speed_weight, 8.0 (racing_env.py:9,26) */
  int32_t cull_chunk;      /* raycast culling: segments per chunk (16 recommended; 0 = test every segment) */
  int32_t sort_interval;   /* re-sort envs by track position every k dynamics launches (0 = never): a
                              counting sort by (slot, waypoint bin), rx_sort.hip; scheduling only.  Skipped
                              when the pool has more than 65,536 slots (at most ~1 env per slot). */
  int32_t ray_order;       /* raycast lane order: 0 = (env, agent, ray), 11 rays of ~6 envs per wave;
                              1 = ray-major: one (agent, ray) of 64 consecutive envs per wave -- with
                              sort_interval > 0 those envs are track neighbours, so a wave's rays are
                              nearly parallel and share culling chunks; 2 = sorted ray tasks: every
                              step the dynamics kernel orders the A*R tasks of each 64-env wave by the
                              absolute direction of the ray (64 sectors, LDS counting sort), so a ray
                              wave holds rays with nearby origins and nearly equal directions.
                              Scheduling only: same results. */
  int32_t cull_super;      /* two-level raycast culling: chunks per super-chunk box (0 = one level) */
  /* ABI v17: launch schedule.  Scheduling only -- every setting gives bit-identical results (the tests
     force each path) -- so 0 = automatic (the measured best for the env count) everywhere; -1 = off /
     none where a field has an off state.  Out-of-range values fail rx_create with RX_EINVAL.  These
     replace the RX_* environment variables earlier versions read: the library reads no environment. */
  int32_t split;           /* split step (k_kin + k_step2: REWARD beside the raycast): 0 auto (on), 1 on, -1 off */
  int32_t wide_n;          /* wide kernels (a wave per env / per ray) up to this many single-agent envs:
                              0 auto (2,048), -1 never, > 0 the threshold */
  int32_t dyn_lpe;         /* k_dyn1 lanes per env: 0 auto, or 1, 2, 4, 64 */
  int32_t ray_lpr;         /* lanes per ray task (ray_order 2): 0 auto (4 / 2 / 1 by (env, car) pairs; two cars:
                              4 / 1), or 1, 2, 4 */
  int32_t reward_lpe;      /* k_step2 REWARD lanes per env: 0 auto (single agent: 2 up to 4,096 envs; two cars:
                              2 = a lane per car up to 16,384 envs), or 1, 2, 4 (two cars: 1 or 2) */
  int32_t argmin_window;   /* closest-waypoint scan half-width around the previous one: 0 auto (2), -1 none,
                              1 .. 32 */
  int32_t seg_filter;      /* float32 pre-filter before each exact segment test: 0 auto (on), 1 on, -1 off */
  int32_t box_quadrants;   /* quadrant-ordered float32 box tables for single-quadrant ray waves: 0 auto (on),
                              1 on, -1 off */
  /* ABI v19: ray-wave dispatch (ray_order 2).  Class j of a 64-env group = its j-th wave of
     direction-sorted ray tasks (the group's cars head alike, so class j ~ sensor ray j). */
  int32_t ray_dispatch;    /* order in which the classes are dispatched: 0 auto (3), 1 centre classes first,
                              2 ascending j, 3 edge classes first / centre last, -1 group-octet-major */
  int32_t ray_tail;        /* the LAST ray_tail classes of that order (the tail of the launch, whose waves
                              run as the chip drains) cast at ray_tail_lpr lanes per ray: each of their
                              64-task waves becomes ray_tail_lpr waves of 64 / ray_tail_lpr tasks.  Only
                              with 1 lane per ray elsewhere.  0 auto, -1 none, 1 .. 16 */
  int32_t ray_tail_lpr;    /* 0 auto (2), 2 or 4 */
  /* ABI v20: the dynamics kernel re-sorts each block's ray tasks by direction every task_sort
     launches (and after every spatial re-sort); in between the ray waves keep the previous
     order.  0 auto (2 up to 16,384 (env, car) pairs, 1 above), 1 .. 16 */
  int32_t task_sort;
  /* ABI v23: lane-varying track slots.  Normally every wavefront holds envs of ONE track slot, so its
     track-table reads are wave-uniform scalar loads; a pool of many distinct tracks (SURVEY.md §8(d)'s
     stress variant: gen_tracks(N, seed=None), one slot per env) then leaves a wave with one env.  With
     lane_tracks on, the single-agent kernels take waves of 64 consecutive envs of ANY slots and every lane
     reads its own slot's tables with vector loads (culling decisions per lane).  0 auto: on when grouping
     by slot would fill the dynamics waves less than half on average (more than 2 x ceil(N / 64) waves);
     1 on; -1 off.  Single-agent envs on the split step at one lane per env and per ray only (wide kernels,
     two-car envs: off).  Scheduling only: bit-identical results. */
  int32_t lane_tracks;
  int32_t reserved0;       /* ABI v23: must be 0 (was kin_sort, a dropped A/B schedule) */
} rx_config;

/* Per-env / per-agent SoA state, caller-owned device memory.  [N*A] arrays are
 * agent-minor: element e*A + a.  Mirrors Car (car.py:15-24), RacingEnv
 * (racing_env.py:17-26), MultiRacingEnv.agents_data (multi_racing_env.py:
 * 142-148) and RecordEpisodeStatistics' episode counters.
 * The engine steps a working copy of these arrays kept in wave order (ABI
 * v15: coalesced state traffic; see rx_state_import / rx_state_export): the
 * bound arrays are read at rx_bind_state / rx_assign and otherwise only
 * synchronised on request.  track and speed_weight are read in place. */
typedef struct {
  double* x;             /* [N*A] */
  double* y;             /* [N*A] */
  double* angle;         /* [N*A] */
  double* vx;            /* [N*A] */
  double* vy;            /* [N*A] */
  double* progress;      /* [N*A] Car.progress */
  double* last_progress; /* [N*A] */
  double* last_steering; /* [N*A] */
  int32_t* finished_step;/* [N*A] -1 = None (A==2 only; may be NULL for A==1) */
  uint8_t* flags;        /* [N*A] RX_F_* */
  int32_t* steps;        /* [N] */
  int32_t* track;        /* [N] track slot (read-only for the kernels; set by rx_assign) */
  uint8_t* env_flags;    /* [N] RX_EF_* */
  double* ep_return;     /* [N] episode return of agent 0 */
  int32_t* ep_length;    /* [N] */
  const double* speed_weight; /* [N] per-env RacingEnv.speed_weight, or NULL = rx_config.speed_weight */
} rx_state;

/* One step's inputs/outputs, caller-owned device memory.  NULL = not wanted
 * (except actions/obs, which are required). */
typedef struct {
  const float* actions;  /* [N][A][2] float32, as the Box(float32) action space */
  float* obs;            /* [N][A][D] float32 */
  float* reward;         /* [N][A] float32 (rollout buffer dtype, agent/ppo.py:116-117) */
  double* reward64;      /* [N][A] float64 (SyncVectorEnv's reward dtype) */
  uint8_t* terminated;   /* [N] */
  uint8_t* truncated;    /* [N] */
  float* done_f32;       /* [N] float(terminated | truncated): next_done, agent/ppo.py:120 */
  double* info;          /* [N][A][RX_INFO_W] */
  uint8_t* ep_done;      /* [N] an episode ended this step (infos['_episode']) */
  double* ep_stats;      /* [RX_EP_SHARDS][4] += (sum return, sum length, count, -) of episodes ended;
                            the caller sums the shard rows */
  unsigned long long* counters; /* [4] profiling, NULL = off: += per wave (raycast chunk tests,
                                   raycast chunks scanned, waypoint chunk tests, waypoint chunks scanned) */
} rx_io;

const char* rx_last_error(void);
int rx_abi_version(void);

/* Create/destroy a handle.  Replaces gym.vector.SyncVectorEnv([...]) construction,
 * agent/ppo.py:70,85-95. */
int rx_create(const rx_config* cfg, rx_env** out);
int rx_destroy(rx_env* h);

/* Host copy of the sensor angle offsets the kernels use: [n_sensors] =
 * np.linspace(-half_cone, half_cone, n_sensors) (racing_env.py:45). */
int rx_sensor_angles(const rx_env* h, double* out);

/* Diagnostics (ABI v15): the env id at each position of the current wave
 * order (envs grouped by slot, re-sorted by track position every
 * sort_interval dynamics launches), host array [n_envs]; synchronises the
 * device.  *sort_bins / *sort_shift (either may be NULL) receive the spatial
 * sort's bin count and waypoints-per-bin shift (0 bins = no re-sort).  The
 * reference has no counterpart (its SyncVectorEnv steps envs in order). */
int rx_env_order(rx_env* h, int32_t* perm_out, int32_t* sort_bins, int32_t* sort_shift);

/* Diagnostics (ABI v17, v19, v20): the launch schedule rx_assign resolved from rx_config
 * for this handle, out int32 [RX_SCHEDULE_W] = split step (0/1), wide kernels
 * (0/1), k_dyn1 lanes per env, lanes per ray task, REWARD lanes per env,
 * closest-waypoint window half-width, segment pre-filter (0/1), quadrant box
 * tables (0/1), dynamics waves, ray waves, ray-wave dispatch order, tail
 * classes, tail lanes per ray, first tail wave (-1 = none), ray-task sort interval, lane-varying
 * track slots (0/1, ABI v23), dynamics launches so far (the re-sort cadence counter: the launch
 * with count % sort_interval == 0 writes the re-sort keys; ABI v21), 0 (reserved).  Host only,
 * no device call. */
#define RX_SCHEDULE_W 18
int rx_schedule(const rx_env* h, int32_t* out);

/* Track table (host arrays, copied to the device).  Replaces the per-env
 * Track.__init__ geometry (environment/track.py:61-148): slot k has
 * W_k = wp_off[k+1]-wp_off[k] waypoints and 2*W_k boundary segments.
 *   wp_off int32 [n+1];  wp, nrm f64 [Wtot][2];
 *   seg f64 [2*Wtot][4] = (start.x, start.y, v2.x, v2.y): left boundary
 *       segments then right ones, per slot (track.py:134-148);
 *   meta f64 [n][8] = start x, y, angle (Track.get_start_pos, track.py:154-157),
 *       track_width, max_track_distance (track.py:88-91), normals[0].x,
 *       normals[0].y, 0. */
int rx_upload_tracks(rx_env* h, int32_t n_tracks, const int32_t* wp_off, const double* wp, const double* nrm,
                     const double* seg, const double* meta);

/* Assign a track slot to every env (host int32 [N]); also written to
 * state.track.  Replaces Track(track_pool, track_id, track_width) per env
 * (train.py:47-49,94-101).  Groups envs by slot so a wavefront shares one
 * track (segment loads become scalar/broadcast). */
int rx_assign(rx_env* h, const int32_t* track_of_env);

/* Bind the caller-owned device state (pointers are kept until re-bound).
 * Once both rx_bind_state and rx_assign have run, the engine copies the bound
 * arrays into its working copy (blocking). */
int rx_bind_state(rx_env* h, const rx_state* st);

/* ABI v15.  The engine keeps the env state in wave order (position p holds
 * env rx_env_order()[p]) so its kernels read and write it coalesced, and
 * moves it with each spatial re-sort.  rx_state_export writes the working
 * copy to the bound arrays (env order) -- call before reading them;
 * rx_state_import reads the bound arrays into the working copy -- call after
 * writing them (state injection).  Both are enqueued on `stream` (a
 * hipStream_t, NULL = legacy default) without a host sync.  The reference
 * keeps this state in per-env Python objects (car.py:15-24, racing_env.py:
 * 17-26), always current. */
int rx_state_import(rx_env* h, void* stream);
int rx_state_export(rx_env* h, void* stream);

int rx_set_speed_weight(rx_env* h, double speed_weight);

/* Reset envs (mask: device uint8 [N], NULL = all).  Replaces
 * SyncVectorEnv.reset -> RacingEnv.reset (racing_env.py:86-102) /
 * MultiRacingEnv.reset (multi_racing_env.py:118-153).  Writes obs (and zeros
 * reward/terminated/truncated/done_f32 of the reset envs when given). */
int rx_reset(rx_env* h, const uint8_t* mask, const rx_io* io, void* stream);

/* ABI v20.  The two-car start-slot order from the reference's own RNG stream:
 * MultiRacingEnv.reset draws it with np.random.shuffle(agent_order) on the
 * global numpy RNG (multi_racing_env.py:127-128), one MT19937 output u per
 * reset (j = u & 1: the two cars swap when j == 0), and SyncVectorEnv resets
 * its envs in env order.  With draws set, the env that is the j-th to reset in
 * a launch (env order: rx_reset's mask, or the next-step autoreset of rx_step)
 * takes draws[cursor[0] + j], and the launch advances cursor[0] by its reset
 * count.  draws: device uint32 [n_draws], the caller's upcoming MT19937 outputs
 * (e.g. np.random.randint(0, 2**32, n, dtype=np.uint32) from a copy of the
 * global state); cursor: device int64 [2], cursor[1] += the draws a launch
 * needed beyond n_draws (those resets are then wrong: refill and redo).
 * draws = NULL restores the device hash.  Two-car handles, next-step or no
 * autoreset (same-step autoreset draws inside the step: RX_EINVAL). */
int rx_set_start_draws(rx_env* h, const uint32_t* draws, int64_t n_draws, int64_t* cursor);

/* One vectorised step.  Replaces SyncVectorEnv.step -> RecordEpisodeStatistics
 * -> RacingEnv.step (racing_env.py:104-167) / SelfPlayWrapper.step ->
 * MultiRacingEnv.step (multi_racing_env.py:213-269), with the configured
 * autoreset semantics. */
int rx_step(rx_env* h, const rx_io* io, void* stream);

/* ABI v21.  n_steps consecutive steps from one call, each equal to an rx_step of
 * the io rows at that step (bit for bit: the same kernels' arithmetic on the same
 * rows).  Step s reads actions + s * strides->actions and writes obs + s *
 * strides->obs, reward + s * strides->reward, ... (element strides; a stride of 0
 * writes every step into the same rows, which then hold the last step's outputs;
 * strides = NULL: all 0).  ep_stats and counters accumulate.  The actions of all
 * n_steps steps must be in device memory when the call is made: open-loop
 * action sequences (the env-throughput benchmark: a bank of random actions) --
 * a policy-in-the-loop rollout is rx_rollout_steps.  Replaces n_steps iterations
 * of SyncVectorEnv.step (agent/ppo.py:112) with precomputed actions. */
typedef struct {
  int64_t actions, obs, reward, reward64, terminated, truncated, done_f32, info, ep_done;
} rx_io_strides;
int rx_steps(rx_env* h, const rx_io* io, int32_t n_steps, const rx_io_strides* strides, void* stream);

/* rx_step split into its two kernels, for per-kernel timing with stream
 * events: phases bit 0 = dynamics/reward/done/autoreset (k_dyn), bit 1 =
 * raycast observations (k_rays).  rx_step == phases 3.  Running bit 1 alone
 * recomputes the ray observations of the current state. */
#define RX_PHASE_DYNAMICS 1
#define RX_PHASE_RAYS 2
int rx_step_phases(rx_env* h, const rx_io* io, int32_t phases, void* stream);

/* Kernel timing for benchmarks.  While profiling, every wave of a recorded
 * launch stamps the device wall clock (s_memrealtime, 100 MHz, one chip-wide
 * counter) at its start and end; a launch's duration is last end - first
 * start: its execution span, as rocprofv3 --kernel-trace measures it, without
 * the dispatch and end-of-kernel cache-flush time that stream events around a
 * launch include.  rx_profile(h, 1) starts a fresh record of the kernels that
 * rx_step / rx_reset / rx_step_phases launch (up to 512 launches; the call
 * synchronises the device), rx_profile(h, 0) pauses recording and
 * rx_profile(h, 2) resumes it (record selected steps only), rx_profile_read
 * synchronises and returns per kernel kind the mean duration (ms) and the
 * launch count.  No counterpart in the reference (it has no benchmarks). */
#define RX_KERNEL_DYN 0    /* k_dyn1 / k_dyn2: one-kernel dynamics (reset, small N, two-car) */
#define RX_KERNEL_RAYS 1   /* k_rays launched on its own (rx_step_phases, one-kernel step) */
#define RX_KERNEL_KIN 2    /* k_kin1: first kernel of the split step */
#define RX_KERNEL_STEP2 3  /* k_step2: REWARD half + raycast in one launch (split step) */
#define RX_KERNEL_REWARD 4 /* k_step2 with the REWARD half only (rx_step_phases dynamics) */
#define RX_KERNEL_KINDS 5
int rx_profile(rx_env* h, int32_t enable);
int rx_profile_read(rx_env* h, double* mean_ms, int32_t* count);
/* Diagnostics (ABI v18): the raw per-wave stamps of recorded launch `launch`
 * (0-based, record order; synchronises).  *n_waves = the launch's wave slots
 * (wave index = workgroup index for k_step2: REWARD waves first, then the ray
 * waves); start[i] / end[i] = device wall-clock ticks (0 = no wave in that
 * slot) for i < min(*n_waves, cap); *kind = its RX_KERNEL_*; *khz = the clock
 * rate.  Used to see how a launch's waves fill the chip over time (tail,
 * per-wave cost by dispatch order).  No counterpart in the reference. */
int rx_profile_waves(rx_env* h, int32_t launch, uint64_t* start, uint64_t* end, int32_t cap, int32_t* n_waves,
                     int32_t* kind, int32_t* khz);
/* Diagnostics (ABI v19): the ray-wave table rx_assign built, host int32 [cap][4]
 * = (track slot, perm start, first task, task count) per ray wave in dispatch
 * order (wave i is k_step2 workgroup n_reward + i, k_rays workgroup i);
 * *n_waves = the table length.  A wave's class j within its 64-env group is
 * (first task - perm start * A * n_sensors) / 64 (ray_order 2, 1 lane per ray
 * outside the tail).  Host only, no device call.  No counterpart in the
 * reference. */
int rx_ray_waves(const rx_env* h, int32_t* out, int32_t cap, int32_t* n_waves);
/* Diagnostics (ABI v22): the device ray-task list the last sorting launch wrote
 * (ray_order 2: per 64-env block its A * n_sensors task ids (A p + q) R + r in
 * direction-sector order), copied to host int32 out[cap] after the stream
 * drains; *n = its length (N * A * n_sensors).  cap = 0 queries *n only. */
int rx_ray_tasks(rx_env* h, int32_t* out, int64_t cap, int64_t* n, void* stream);

/* GAE (agent/ppo.py:134-154), float32, bit-exact lane-per-env recurrence.
 * rewards/values/dones [T][N]; next_value/next_done [N]; adv/returns [T][N]. */
int rx_gae(int32_t T, int32_t N, const float* rewards, const float* values, const float* dones,
           const float* next_value, const float* next_done, double gamma, double gae_lambda, float* advantages,
           float* returns, void* stream);

/* Same recurrence evaluated as a wavefront-parallel affine scan over T
 * (chunks of T per lane, combined with a 64-lane prefix scan): for few envs
 * and long horizons.  Not bit-exact (different association); |error| <=
 * ~1e-6 * max|A| (tests/test_gae_gpu.py). */
int rx_gae_scan(int32_t T, int32_t N, const float* rewards, const float* values, const float* dones,
                const float* next_value, const float* next_done, double gamma, double gae_lambda, float* advantages,
                float* returns, void* stream);

/* Fused optimizer step of PPO.ppo_update (agent/ppo.py:204-207):
 * nn.utils.clip_grad_norm_(params, max_grad_norm) then torch.optim.Adam.step()
 * (the default eps=1e-5 Adam of agent/ppo.py:83, no weight decay/amsgrad),
 * over parameters stored back to back in ONE float32 buffer: tensor k owns
 * elements [offsets[k], offsets[k+1]).  Two launches: per-slice, per-tensor
 * sums of squares into ws, then per element: global norm -> clip coefficient
 * -> Adam update.
 *
 *   step    device f32 scalar, the Adam step count (incremented here);
 *   lr      device f64 scalar (read at run time, so a captured graph follows
 *           the host-side lr anneal);
 *   stop    device bool or NULL: when *stop != 0 the launch changes nothing
 *           (the KL early stop of agent/ppo.py:178-182 without a host sync);
 *   ws      device f32 scratch of rx_adam_workspace_floats(cfg) elements
 *           (the clip-norm partials, then Adam's two step scalars),
 *           owned by the caller (one per concurrently stepping optimizer).
 * max_grad_norm <= 0 disables clipping.  Grads are scaled in place, as
 * clip_grad_norm_ does.  Equal to torch's clip + Adam within float rounding
 * (tests/test_optim_gpu.py), not bit for bit (reduction order). */
#define RX_ADAM_MAX_TENSORS 32
typedef struct rx_adam_config {
  int32_t n_tensors;
  int64_t offsets[RX_ADAM_MAX_TENSORS + 1];
  double beta1, beta2, eps, max_grad_norm;
} rx_adam_config;
#define RX_ADAM_NORM_ELEMS 64  /* gradient entries per clip-norm partial (rx_adam_workspace_floats) */
size_t rx_adam_workspace_floats(const rx_adam_config* cfg); /* 0 for an invalid cfg */
int rx_adam_clip_step(const rx_adam_config* cfg, float* params, float* grads, float* exp_avg, float* exp_avg_sq,
                      float* step, const double* lr, const uint8_t* stop, float* ws, void* stream);

/* Fused PPO minibatch gradient (agent/ppo.py:170-203) for the reference's
 * actor-critic (agent/ppo.py:11-62: Linear(D,64)-tanh-Linear(64,64)-tanh-
 * Linear(64,2)-tanh actor, same trunk with a 1-wide linear head for the
 * critic, fixed log_std buffer), parameters flat in module.parameters() order
 * (rx_adam_clip_step layout).  For minibatch m of an epoch (rows
 * perm[m*mb .. (m+1)*mb)) it computes the gradient of
 *   pg_loss - ent_coef * entropy + vf_coef * v_loss
 * (the entropy term has no parameter gradient: it depends on log_std only)
 * into grad [P], and approx_kl = mean(old_logp - new_logp); if approx_kl >
 * kl_target it sets *stop (and *kl_at_stop) so the rx_adam_clip_step that
 * follows is skipped.  With *stop already set the call does nothing.
 * fp32; equal to torch autograd within float rounding (tests/test_ppo_fused_gpu.py). */
/* Matrix-core precision of the policy kernels (rx_ppo_batch / rx_policy_io):
 * FP32 = v_mfma_f32_16x16x4_f32, exact float32 products (an fmaf chain);
 * BF16 = v_mfma_f32_16x16x32_bf16: weights / activations / gradients rounded to
 * bf16 as matrix operands, float32 accumulation, float32 everywhere else
 * (BASELINE.json configs[1], "PPO bf16"). */
#define RX_PREC_FP32 0
#define RX_PREC_BF16 1
typedef struct rx_ppo_batch {
  int32_t obs_dim;          /* D: 15 (single-agent) or 19 (two-car) */
  int32_t mb;               /* minibatch rows */
  int64_t n_rows;           /* B = rows of the flattened rollout; perm entries must be < B */
  const float* obs;         /* [B][D] */
  const float* actions;     /* [B][2] */
  const float* logprobs;    /* [B] */
  const float* advantages;  /* [B] */
  const float* returns;     /* [B] */
  const float* values;      /* [B] */
  const int64_t* perm;      /* [n_mb*mb] this epoch's shuffled row indices (b_inds) */
  const float* params;      /* [P] flat parameters */
  const float* log_std;     /* [2] Agent.log_std buffer */
  const float* adv_stats;   /* [n_mb][2] (mean, unbiased std) from rx_ppo_adv_stats */
  float clip_coef, vf_coef, kl_target;
  int32_t precision;        /* RX_PREC_FP32 (default) or RX_PREC_BF16 (ABI v14) */
} rx_ppo_batch;
/* P for obs_dim (10,563 for 15, 11,075 for 19; 0 = unsupported). */
int rx_ppo_n_params(int32_t obs_dim);
/* float / double workspace sizes rx_ppo_minibatch_grad needs for minibatch size mb. */
size_t rx_ppo_workspace_floats(int32_t obs_dim, int32_t mb);
size_t rx_ppo_workspace_doubles(int32_t mb);
/* (mean, unbiased std) of advantages[perm[m*mb ..]] for every minibatch m < n_mb. */
int rx_ppo_adv_stats(const rx_ppo_batch* b, int32_t n_mb, float* stats, void* stream);
int rx_ppo_minibatch_grad(const rx_ppo_batch* b, int32_t m, float* ws_f32, double* ws_f64, float* grad,
                          uint8_t* stop, float* kl_at_stop, void* stream);

/* One whole optimizer step of the single-rank update (agent/ppo.py:170-207:
 * minibatch forward / loss / backward, KL check, clip_grad_norm_, Adam) in
 * three launches: rx_ppo_minibatch_grad's gradient + reduce (which also writes
 * the per-tensor sums of squares to adam_ws and bumps *step unless it raises
 * *stop), then the clip + Adam update of params / exp_avg / exp_avg_sq
 * (rx_adam_clip_step's arithmetic; skipped when *stop is set).  params must be
 * b->params; cfg the rx_adam_clip_step layout of the same P parameters;
 * adam_ws holds rx_ppo_update_workspace_floats(obs_dim, cfg) floats (ABI v23: the
 * per-tensor norm partials and Adam's two step scalars; no control block). */
size_t rx_ppo_update_workspace_floats(int32_t obs_dim, const rx_adam_config* cfg);
int rx_ppo_minibatch_update(const rx_ppo_batch* b, int32_t m, const rx_adam_config* cfg, float* params,
                            float* ws_f32, double* ws_f64, float* grad, float* exp_avg, float* exp_avg_sq, float* step,
                            const double* lr, uint8_t* stop, float* kl_at_stop, float* adam_ws, void* stream);

/* Data-parallel variant of the same minibatch step (one rank's shard of a
 * global minibatch; rx.dist).  Replaces the per-rank part of
 * agent/ppo.py:170-207 when the batch is sharded over W ranks:
 *
 *   rx_ppo_adv_moments     per minibatch (sum, square-sum) of this shard's
 *                          advantages, f64 [n_mb][2] -> caller all-reduces;
 *   rx_ppo_adv_finalize    (mean, unbiased std) from all-reduced moments over
 *                          count = W*mb rows -> adv_stats of the batch
 *                          (moments -> finalize with count = mb equals
 *                          rx_ppo_adv_stats bit for bit);
 *   rx_ppo_minibatch_grad_shard
 *                          the shard's gradient times ``scale`` (= 1/W: an
 *                          all-reduce SUM then gives the global-minibatch mean
 *                          gradient) into grad, and scale * mean(old_logp -
 *                          new_logp) into *kl_out.  Reads *stop (does nothing
 *                          when set) but never writes it: with grad and kl_out
 *                          adjacent in one buffer a single all-reduce carries
 *                          both;
 *   rx_ppo_kl_check        after the all-reduce: *kl > kl_target -> *stop = 1,
 *                          *kl_at_stop = *kl (agent/ppo.py:178-182), so the
 *                          rx_adam_clip_step that follows is skipped on every
 *                          rank alike. */
int rx_ppo_adv_moments(const rx_ppo_batch* b, int32_t n_mb, double* moments, void* stream);
/* ABI v17: rx_ppo_adv_stats / rx_ppo_adv_moments spread over many workgroups
 * per minibatch (chunks of 2,048 rows, a partial-moment workspace ws of
 * rx_ppo_adv_workspace_doubles(mb, n_mb) doubles, two launches: chunk moments,
 * then a fold in chunk order).  Writes the raw (sum, square-sum) moments when
 * `moments` is given (data parallel: all-reduce, then rx_ppo_adv_finalize),
 * else (mean, unbiased std) into stats; moments -> rx_ppo_adv_finalize(count =
 * mb) equals the stats output bit for bit.  Its own summation order: not
 * bit-identical to rx_ppo_adv_stats. */
size_t rx_ppo_adv_workspace_doubles(int32_t mb, int32_t n_mb);
int rx_ppo_adv_stats_ws(const rx_ppo_batch* b, int32_t n_mb, double* ws, float* stats, double* moments, void* stream);
int rx_ppo_adv_finalize(const double* moments, int32_t n_mb, int64_t count, float* stats, void* stream);
int rx_ppo_minibatch_grad_shard(const rx_ppo_batch* b, int32_t m, float scale, float* ws_f32, double* ws_f64,
                                float* grad, float* kl_out, const uint8_t* stop, void* stream);
int rx_ppo_kl_check(const float* kl, float kl_target, uint8_t* stop, float* kl_at_stop, void* stream);

/* ABI v16.  The minibatch shuffle of PPO.ppo_update (agent/ppo.py:165-171,
 * np.random.shuffle(b_inds)) on the device, for config shuffle = "device": out
 * [n] int64 receives a pseudo-random permutation of 0 .. n-1 keyed by seed
 * (4-round unbalanced Feistel network on ceil(log2 n) bits, cycle-walked to
 * [0, n)); one launch, no host
 * round trip.  Same seed, same permutation. */
int rx_random_permutation(int64_t n, uint64_t seed, int64_t* out, void* stream);

/* Rollout policy step (agent/ppo.py:105-110: agent.get_action_and_value(obs)
 * under no_grad) for the same policy layout: per row, actor + critic forward,
 *   action = clamp(eps * exp(log_std) + mu, -1, 1)   (Normal.sample(), then
 *            the reference's clamp; eps = N(0,1) noise drawn by the caller,
 *            e.g. torch normal_(), so the sampling stream stays torch's)
 *   logprob = sum_j Normal(mu, std).log_prob(action_j);  value = critic(obs).
 * fp32; equal to the torch forward within float rounding
 * (tests/test_ppo_fused_gpu.py). */
typedef struct rx_policy_io {
  int32_t obs_dim;        /* 15 or 19 */
  int64_t n;              /* rows */
  const float* obs;       /* [n] rows of D floats, obs_stride floats apart (0 = D) */
  const float* eps;       /* [n][2] */
  const float* params;    /* flat parameters */
  const float* log_std;   /* [2] */
  float* actions;         /* [n] rows of 2 floats, act_stride floats apart (0 = 2) out */
  float* logprobs;        /* [n] out */
  float* values;          /* [n] out */
  int64_t obs_stride;     /* e.g. 2*19 for one car's rows of a two-car [n][2][19] buffer */
  int64_t act_stride;     /* e.g. 4 for one car's actions in [n][2][2] */
  int32_t precision;      /* RX_PREC_FP32 (default) or RX_PREC_BF16 (ABI v14) */
  float* actions2;        /* ABI v19: NULL, or a second copy of the actions (e.g. the agent's slot of a two-car
                             env's [n][2][2] action buffer), rows act2_stride floats apart (0 = 2) */
  int64_t act2_stride;
} rx_policy_io;
int rx_policy_act(const rx_policy_io* io, void* stream);

/* A whole rollout of few single-agent envs in ONE persistent launch.
 * Replaces PPO.collect_rollout's step loop (agent/ppo.py:97-132: per step
 * agent.get_action_and_value(next_obs) at :105-110, envs.step(action) at
 * :112-120) for handles in the small-N configuration (one env per dynamics
 * wave: rx_rollout_supported).  Per step t the env's workgroup evaluates the
 * policy on obs[t] exactly as rx_policy_act does with eps[t] (actions,
 * log-probs, values), then steps the env exactly as rx_step does, writing
 * obs[t+1] (next_obs after the last step), rewards[t], dones[t+1] (next_done
 * after the last step).  obs[0] and dones[0] are the caller's.  io supplies the
 * env's terminated / truncated / ep_done / ep_stats buffers (its obs, reward,
 * done and actions pointers are ignored).  Same stream semantics as rx_step. */
typedef struct rx_rollout_io {
  int32_t T;              /* steps */
  int32_t obs_dim;        /* 15 or 19 (= the handle's observation width) */
  const float* params;    /* flat policy parameters (rx_policy_act layout) */
  const float* log_std;   /* [2] */
  const float* eps;       /* [T][N][2] N(0,1) noise */
  float* obs;             /* [T][N][D] */
  float* actions;         /* [T][N][2] out */
  float* logprobs;        /* [T][N] out */
  float* values;          /* [T][N] out */
  float* rewards;         /* [T][N] out */
  float* dones;           /* [T][N] out (rows 1..T-1) */
  float* next_obs;        /* [N][D] out */
  float* next_done;       /* [N] out */
} rx_rollout_io;
int rx_rollout_supported(const rx_env* h);
int rx_rollout(rx_env* h, const rx_io* io, const rx_rollout_io* r, void* stream);

/* ABI v19: the same T-step rollout for ANY single-agent handle as a sequence of
 * launches enqueued by ONE call: per step t, rx_policy_act on obs[t] with
 * eps[t] (actions[t], logprobs[t], values[t]) at matrix-core `precision`, then
 * rx_step of actions[t] writing obs[t+1] (next_obs at t = T-1), rewards[t] and
 * dones[t+1] (next_done).  Every kernel and every output equals the per-step
 * Python loop (rx_policy_act + rx_step per step) with the same eps bit for bit;
 * what it removes is T x (tensor slicing + two ctypes calls + a noise launch)
 * of host time per rollout -- the eager rollout of a few thousand envs was
 * host-bound.  `io` as for rx_rollout.  Replaces the step loop of
 * PPO.collect_rollout, agent/ppo.py:97-132. */
int rx_rollout_steps(rx_env* h, const rx_io* io, const rx_rollout_io* r, int32_t precision, void* stream);

/* ABI v19: the self-play rollout (environment/wrappers.py:29-55 inside
 * agent/self_play_ppo.py's collect_rollout) of a TWO-CAR handle the same way:
 * per step t the frozen opponent's rx_policy_act on its rows of the env's obs
 * buffer (opp_eps[t], actions into its slot of the env's action buffer), the
 * agent's rx_policy_act on obs[t] (eps[t]; actions into actions[t] AND its slot
 * of the env's action buffer), rx_step, then one copy of the agent's obs row and
 * reward out of the env's [N][2] buffers into obs[t+1] / rewards[t].  Five
 * launches per step from one call (the Python step ran nine: two noise draws,
 * three copies).  Every output equals SelfPlayVectorEnv's per-step path with
 * the same noise bit for bit.  `r` is the agent's rollout (obs_dim 19). */
typedef struct rx_selfplay_io {
  const float* opp_params;   /* the frozen opponent's flat parameters */
  const float* opp_log_std;  /* [2] */
  const float* opp_eps;      /* [T][N][2] N(0,1) noise of the opponent */
  float* env_actions;        /* [N][2][2] the handle's action buffer */
  float* env_obs;            /* [N][2][D] the handle's observation buffer (rx_io.obs) */
  float* env_reward;         /* [N][2] the handle's reward buffer (rx_io.reward) */
  float* sink;               /* [2N] float32 scratch: the opponent's log-probs / values */
  int32_t agent;             /* the learning agent's car (0 or 1); the opponent is the other */
  int32_t opp_precision;     /* RX_PREC_* of the opponent's forward */
} rx_selfplay_io;
int rx_selfplay_rollout_steps(rx_env* h, const rx_io* io, const rx_rollout_io* r, const rx_selfplay_io* sp,
                              int32_t precision, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* RX_H_ */
