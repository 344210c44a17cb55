/* rx_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * A plain-C restatement of the reference's CPU environment step path, in the
 * reference's exact floating-point operation order, used by tests/ (and by
 * __graft_entry__.smoke()) to check the HIP kernels.  Only tests/, smoke() and
 * bench.py's cpu_baseline leg may load it.  Nothing in the product
 * (self-play-racing_amd/) links, loads or calls it.
 *
 * Pinned against the reference itself: tests/test_oracle_golden.py checks every
 * function here against the tests/golden npz files, which tests/golden/gen_golden.py
 * produced by importing the reference (/root/reference, read-only) in the
 * build container.  The glibc build (default) is bit-exact against those
 * vectors; see DESIGN.md §Parity.
 *
 * Two libm modes (compile-time):
 *   default           sin/cos/pow from glibc  -- what numpy calls
 *   -DORC_DEVICE_LIBM sin/cos = rx_sincos() (correctly rounded, shared with the
 *                     HIP kernels via csrc/rx_math.h); pow(x,2) = x*x.
 * The second build differs from the reference only through those two
 * functions, so HIP-vs-oracle(device-libm) must agree bit for bit on every
 * output; the glibc build pins the reference semantics.
 *
 * Floating point: compiled with -ffp-contract=off; the only FMAs are the
 * explicit ones at the reference's np.dot call sites (rx_dot2_np).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "rx_math.h"

#ifdef ORC_DEVICE_LIBM
static inline void orc_sincos(double x, double* s, double* c) { rx_sincos(x, s, c); }
static inline double orc_cos(double x) { double s, c; rx_sincos(x, &s, &c); return c; }
static inline double orc_sin(double x) { double s, c; rx_sincos(x, &s, &c); return s; }
static inline double orc_pow2(double x) { return x * x; }
#else
static inline double orc_cos(double x) { return cos(x); }
static inline double orc_sin(double x) { return sin(x); }
static inline double orc_pow2(double x) { return pow(x, 2.0); }
#endif

#define ORC_MAX_SPEED 30.0       /* environment/car.py:5 */
#define ORC_ACCEL 10.0           /* environment/car.py:6 */
#define ORC_STEER_SPEED 3.0      /* environment/car.py:7 */
#define ORC_DRAG 0.985           /* environment/car.py:8 */
#define ORC_LAT_FRICTION 0.85    /* environment/car.py:9 */
#define ORC_GRIP 0.9             /* environment/car.py:10 */
#define ORC_DT 0.05              /* environment/car.py:45 (update default) */
#define ORC_TWO_PI 6.283185307179586 /* 2*np.pi, environment/car.py:54 */
#define ORC_MAX_RANGE 50.0       /* racing_env.py:15, multi_racing_env.py:15 */

/* flags bits (state.flags) */
#define F_CRASHED 1u
#define F_FINISHED 2u
#define F_CP25 4u
#define F_CP50 8u
#define F_CP75 16u
#define F_HAS_CRASHED 32u /* multi env only: agents_data['has_crashed'] */

/* Track table: same layout as the device table (include/rx.h rx_track_table). */
typedef struct {
  int n_tracks;
  const int32_t* wp_off; /* [n+1]; segments of track k: [2*wp_off[k], 2*wp_off[k+1]) */
  const double* wp;      /* [Wtot][2] */
  const double* nrm;     /* [Wtot][2] */
  const double* seg;     /* [Stot][4] = start.x, start.y, v2.x, v2.y */
  const double* meta;    /* [n][8] = start x, y, angle, width, max_track_distance, nrm0.x, nrm0.y, 0 */
} orc_tracks;

/* ---------------------------------------------------------------- track.py */

/* Track.closest_waypoint_idx -- environment/track.py:150-152
 * argmin_i (wx_i - x)^2 + (wy_i - y)^2 (array `**2` = square), first index on ties. */
int orc_closest_wp(const double* wp, int W, double x, double y) {
  int best = 0;
  double bd = 0.0;
  for (int i = 0; i < W; ++i) {
    double dx = wp[2 * i] - x, dy = wp[2 * i + 1] - y;
    double d = dx * dx + dy * dy;
    if (i == 0 || d < bd) {
      bd = d;
      best = i;
    }
  }
  return best;
}

/* Track.check_collision -- environment/track.py:163-171 (early exit kept) */
static int orc_check_collision(const double* wp, const double* nrm, int W, double width, const double cx[4],
                               const double cy[4]) {
  for (int k = 0; k < 4; ++k) {
    int idx = orc_closest_wp(wp, W, cx[k], cy[k]);
    double px = cx[k] - wp[2 * idx], py = cy[k] - wp[2 * idx + 1];
    double dist = fabs(rx_dot2_np(px, py, nrm[2 * idx], nrm[2 * idx + 1])); /* np.dot, :168 */
    if (dist > width) return 1;
  }
  return 0;
}

/* Track.raycast -- environment/track.py:173-199.  Uncapped: min t over hits,
 * else max_dist. */
double orc_raycast(const double* seg, int S, double ox, double oy, double direction, double max_dist) {
  double c = orc_cos(direction), s = orc_sin(direction);
  double v3x = -s, v3y = c;
  int any = 0;
  double best = 0.0;
  for (int j = 0; j < S; ++j) {
    const double* g = seg + 4 * j;
    double v1x = ox - g[0], v1y = oy - g[1];
    double v2x = g[2], v2y = g[3];
    double dotp = v2x * v3x + v2y * v3y;           /* np.sum(v2*v3, 1), :179 */
    if (!(fabs(dotp) > 1e-10)) continue;             /* :182 */
    double t = (v2x * v1y - v2y * v1x) / dotp;       /* :187-189 */
    double sp = (v1x * v3x + v1y * v3y) / dotp;      /* :191-193 */
    if (t >= 0.0 && sp >= 0.0 && sp <= 1.0) {        /* :195 */
      if (!any || t < best) best = t;
      any = 1;
    }
  }
  return any ? best : max_dist;
}

/* ------------------------------------------------------------------ car.py */

/* Car.get_corners -- environment/car.py:26-43 (products by +-2/+-1 are exact,
 * so the 2x2 matmul is order/FMA insensitive) */
static void orc_corners(double x, double y, double angle, double cx[4], double cy[4]) {
  static const double L[4][2] = {{2.0, 1.0}, {2.0, -1.0}, {-2.0, -1.0}, {-2.0, 1.0}};
  double c = orc_cos(angle), s = orc_sin(angle);
  for (int k = 0; k < 4; ++k) {
    cx[k] = (c * L[k][0] + (-s) * L[k][1]) + x;
    cy[k] = (s * L[k][0] + c * L[k][1]) + y;
  }
}

typedef struct {
  double x, y, angle, vx, vy, progress;
  int crashed;
} orc_car;

/* Car.update -- environment/car.py:45-80 */
static void orc_car_update(orc_car* car, double steering, double throttle, const double* wp, const double* nrm,
                           int W, double width) {
  if (car->crashed) return; /* :50-51 */
  double angular_velocity = steering * ORC_STEER_SPEED;
  double angle = car->angle + (angular_velocity * ORC_DT);
  angle = rx_pymod(angle, ORC_TWO_PI); /* :54 */
  double c = orc_cos(angle), s = orc_sin(angle);
  double vf = car->vx * c + car->vy * s;
  double vl = car->vx * (-s) + car->vy * c;
  double accel_forward = throttle * ORC_ACCEL;
  vf = (vf + (accel_forward * ORC_DT)) * ORC_DRAG;
  vl = vl * ORC_LAT_FRICTION * ORC_GRIP; /* (vl*0.85)*0.9, :61 */
  double vx = vf * c - vl * s;
  double vy = vf * s + vl * c;
  double speed = sqrt(orc_pow2(vx) + orc_pow2(vy)); /* np.float64 ** 2 -> pow, :68 */
  if (speed > ORC_MAX_SPEED) {
    double scale = ORC_MAX_SPEED / speed;
    vx *= scale;
    vy *= scale;
  }
  car->angle = angle;
  car->vx = vx;
  car->vy = vy;
  car->x = car->x + (vx * ORC_DT);
  car->y = car->y + (vy * ORC_DT);
  car->progress = (double)orc_closest_wp(wp, W, car->x, car->y) / (double)W; /* track.py:159-161 */
  double cx[4], cy[4];
  orc_corners(car->x, car->y, car->angle, cx, cy);
  car->crashed = orc_check_collision(wp, nrm, W, width, cx, cy);
}

/* f32 np.clip(a, lo, hi) with Python-float bounds (NEP 50: stays float32) */
static inline float orc_clipf(float a, float lo, float hi) {
  float y = a < lo ? lo : a;
  return y > hi ? hi : y;
}

/* --------------------------------------------------------- racing_env.py */

typedef struct {
  double *x, *y, *angle, *vx, *vy, *progress, *last_progress, *last_steering;
  int32_t *steps, *track;
  uint8_t* flags;
} orc_single_state;

/* RacingEnv.get_sensor_readings + _get_obs -- environment/racing_env.py:44-75 */
static void orc_single_obs(const orc_tracks* T, int k, const orc_car* car, double last_steering, int n_sensors,
                           const double* rel_angles, float* obs) {
  int W = T->wp_off[k + 1] - T->wp_off[k];
  const double* seg = T->seg + 4 * (2 * (size_t)T->wp_off[k]);
  for (int i = 0; i < n_sensors; ++i) {
    double world_angle = car->angle + rel_angles[i];
    float d = (float)orc_raycast(seg, 2 * W, car->x, car->y, world_angle, ORC_MAX_RANGE);
    obs[i] = d / 50.0f; /* f32 array / 50.0, :53 */
  }
  double c = orc_cos(car->angle), s = orc_sin(car->angle);
  double vf = car->vx * c + car->vy * s;
  double vl = (-car->vx) * s + car->vy * c;
  vf = rx_clip(vf / ORC_MAX_SPEED, -1.0, 1.0);
  vl = rx_clip(vl / ORC_MAX_SPEED, -1.0, 1.0);
  obs[n_sensors + 0] = (float)vf;
  obs[n_sensors + 1] = (float)vl;
  obs[n_sensors + 2] = (float)rx_clip(0.0 / ORC_STEER_SPEED, -1.0, 1.0); /* angular_velocity == 0 (Q2) */
  obs[n_sensors + 3] = (float)last_steering;
}

/* RacingEnv.reset -- environment/racing_env.py:86-102 (+ Car.reset car.py:17-24).
 * mask: NULL = all envs.  info (may be NULL): [n][3] = speed, progress, 0 */
void orc_single_reset(int n, const orc_tracks* T, orc_single_state st, const uint8_t* mask, int n_sensors,
                      const double* rel_angles, float* obs, double* info) {
  int D = n_sensors + 4;
  for (int e = 0; e < n; ++e) {
    if (mask && !mask[e]) continue;
    int k = st.track[e];
    const double* m = T->meta + 8 * k;
    st.x[e] = m[0];
    st.y[e] = m[1];
    st.angle[e] = m[2];
    st.vx[e] = 0.0;
    st.vy[e] = 0.0;
    st.progress[e] = 0.0;
    st.flags[e] = 0;
    st.steps[e] = 0;
    st.last_progress[e] = 0.0;
    st.last_steering[e] = 0.0;
    orc_car car = {st.x[e], st.y[e], st.angle[e], 0.0, 0.0, 0.0, 0};
    orc_single_obs(T, k, &car, 0.0, n_sensors, rel_angles, obs + (size_t)e * D);
    if (info) {
      info[3 * e + 0] = 0.0;
      info[3 * e + 1] = 0.0;
      info[3 * e + 2] = 0.0;
    }
  }
}

/* RacingEnv.step -- environment/racing_env.py:104-167.
 * info (may be NULL): [n][3] = info['speed'], info['progress'], info['progress_delta'] */
void orc_single_step(int n, const orc_tracks* T, orc_single_state st, const float* actions,
                     const double* speed_weight, int n_sensors, const double* rel_angles, float* obs, double* reward,
                     uint8_t* terminated, uint8_t* truncated, double* info) {
  int D = n_sensors + 4;
  for (int e = 0; e < n; ++e) {
    int k = st.track[e];
    int W = T->wp_off[k + 1] - T->wp_off[k];
    const double* wp = T->wp + 2 * (size_t)T->wp_off[k];
    const double* nrm = T->nrm + 2 * (size_t)T->wp_off[k];
    double width = T->meta[8 * k + 3];
    uint8_t fl = st.flags[e];
    double steering = (double)orc_clipf(actions[2 * e], -1.0f, 1.0f); /* :106 */
    double throttle = (double)orc_clipf(actions[2 * e + 1], 0.0f, 1.0f); /* :107 */
    double last_progress = st.last_progress[e];
    orc_car car = {st.x[e], st.y[e], st.angle[e], st.vx[e], st.vy[e], st.progress[e], (fl & F_CRASHED) != 0};
    orc_car_update(&car, steering, throttle, wp, nrm, W, width);
    int steps = st.steps[e] + 1;
    double p = car.progress;
    double pd = p - last_progress; /* :112-116 */
    if (last_progress > 0.9 && p < 0.1)
      pd = (1.0 - last_progress) + p;
    else if (last_progress < 0.1 && p > 0.9)
      pd = -((1.0 - p) + last_progress);
    double r = pd * 200;
    if (!(fl & F_CP25) && 0.25 <= p && p < 0.35) { fl |= F_CP25; r += 20; }
    if ((fl & F_CP25) && !(fl & F_CP50) && 0.50 <= p && p < 0.60) { fl |= F_CP50; r += 20; }
    if ((fl & F_CP50) && !(fl & F_CP75) && 0.75 <= p && p < 0.85) { fl |= F_CP75; r += 20; }
    if (!car.crashed && pd > 0) { /* :137-140 */
      double speed = sqrt(orc_pow2(car.vx) + orc_pow2(car.vy));
      double ratio = rx_clip(speed / ORC_MAX_SPEED, 0.0, 1.0);
      r += ratio * speed_weight[e];
    }
    if (car.crashed) r -= 60; /* :142-143 */
    int all_cp = (fl & (F_CP25 | F_CP50 | F_CP75)) == (F_CP25 | F_CP50 | F_CP75);
    if (all_cp && last_progress > 0.9 && p < 0.1 && pd > 0) { /* :145-150 */
      fl |= F_FINISHED;
      r += 100;
      double tb = 200 - ((double)steps / 10);
      if (tb > 0) r += tb;
    }
    fl = (uint8_t)((fl & ~F_CRASHED) | (car.crashed ? F_CRASHED : 0));
    orc_single_obs(T, k, &car, steering, n_sensors, rel_angles, obs + (size_t)e * D);
    if (info) {
      info[3 * e + 0] = sqrt(orc_pow2(car.vx) + orc_pow2(car.vy)); /* _get_info :80 */
      info[3 * e + 1] = (fl & F_FINISHED) ? 1.0 : p;                 /* :158-159 */
      info[3 * e + 2] = pd;
    }
    reward[e] = r;
    terminated[e] = (car.crashed || (fl & F_FINISHED)) ? 1 : 0; /* :161 */
    truncated[e] = steps >= 3000 ? 1 : 0;                       /* :162 */
    st.x[e] = car.x;
    st.y[e] = car.y;
    st.angle[e] = car.angle;
    st.vx[e] = car.vx;
    st.vy[e] = car.vy;
    st.progress[e] = p;
    st.last_progress[e] = p; /* :165 */
    st.last_steering[e] = steering;
    st.steps[e] = steps;
    st.flags[e] = fl;
  }
}

/* ------------------------------------------------- multi_track.py / multi_car.py */

/* MultiTrack.ray_seg_intersection -- environment/multi_track.py:28-44; returns
 * -1 for None (t >= 0 always on a hit) */
static double orc_ray_seg(double ox, double oy, double rdx, double rdy, double sx, double sy, double ex, double ey) {
  double v1x = ox - sx, v1y = oy - sy;
  double v2x = ex - sx, v2y = ey - sy;
  double v3x = -rdy, v3y = rdx;
  double dotp = rx_dot2_np(v2x, v2y, v3x, v3y); /* np.dot, :34 */
  if (fabs(dotp) < 1e-10) return -1.0;
  double t = (v2x * v1y - v2y * v1x) / dotp;          /* np.cross, :38 */
  double s = rx_dot2_np(v1x, v1y, v3x, v3y) / dotp;   /* np.dot, :39 */
  if (t >= 0 && 0 <= s && s <= 1) return t;
  return -1.0;
}

/* MultiTrack.raycast_with_cars -- environment/multi_track.py:5-26 */
static double orc_raycast_with_cars(const double* seg, int S, double ox, double oy, double direction, int n_cars,
                                    const orc_car* cars) {
  double wall = orc_raycast(seg, S, ox, oy, direction, ORC_MAX_RANGE);
  double rdx = orc_cos(direction), rdy = orc_sin(direction);
  double min_car = ORC_MAX_RANGE;
  for (int i = 0; i < n_cars; ++i) {
    double dx = cars[i].x - ox, dy = cars[i].y - oy;
    if (sqrt(rx_dot2_np(dx, dy, dx, dy)) < 0.5) continue; /* np.linalg.norm, :13 */
    double cx[4], cy[4];
    orc_corners(cars[i].x, cars[i].y, cars[i].angle, cx, cy);
    for (int q = 0; q < 4; ++q) {
      double d = orc_ray_seg(ox, oy, rdx, rdy, cx[q], cy[q], cx[(q + 1) & 3], cy[(q + 1) & 3]);
      if (d >= 0 && d < min_car) min_car = d;
    }
  }
  return (min_car < wall) ? min_car : wall;
}

/* MultiCar.rectangles_intersect -- environment/multi_car.py:16-43 (SAT) */
static int orc_rect_intersect(const double ax[4], const double ay[4], const double bx[4], const double by[4]) {
  double axis[4][2];
  for (int i = 0; i < 2; ++i) {
    axis[i][0] = -(ay[i + 1] - ay[i]);
    axis[i][1] = ax[i + 1] - ax[i];
    axis[2 + i][0] = -(by[i + 1] - by[i]);
    axis[2 + i][1] = bx[i + 1] - bx[i];
  }
  for (int q = 0; q < 4; ++q) {
    double amax = 0, amin = 0, bmax = 0, bmin = 0;
    for (int c = 0; c < 4; ++c) {
      double pa = rx_dot2_np(ax[c], ay[c], axis[q][0], axis[q][1]);
      double pb = rx_dot2_np(bx[c], by[c], axis[q][0], axis[q][1]);
      if (c == 0 || pa > amax) amax = pa;
      if (c == 0 || pa < amin) amin = pa;
      if (c == 0 || pb > bmax) bmax = pb;
      if (c == 0 || pb < bmin) bmin = pb;
    }
    if (amax < bmin || bmax < amin) return 0;
  }
  return 1;
}

/* --------------------------------------------------- multi_racing_env.py */

typedef struct {
  /* per agent arrays [n][2] */
  double *x, *y, *angle, *vx, *vy, *progress, *last_progress, *last_steering;
  int32_t* finished_step; /* -1 = None */
  uint8_t* flags;         /* F_* incl. F_HAS_CRASHED */
  /* per env [n] */
  int32_t *steps, *track;
} orc_multi_state;

/* MultiRacingEnv._get_obs -- environment/multi_racing_env.py:60-105 (2 agents) */
static void orc_multi_obs(const orc_tracks* T, int k, const orc_car cars[2], int a, double last_steering,
                          int n_sensors, const double* rel_angles, float* obs) {
  int W = T->wp_off[k + 1] - T->wp_off[k];
  const double* seg = T->seg + 4 * (2 * (size_t)T->wp_off[k]);
  double maxd = T->meta[8 * k + 4];
  const orc_car* car = &cars[a];
  for (int i = 0; i < n_sensors; ++i) {
    double world_angle = car->angle + rel_angles[i];
    float d = (float)orc_raycast_with_cars(seg, 2 * W, car->x, car->y, world_angle, 2, cars);
    obs[i] = d / 50.0f;
  }
  double c = orc_cos(car->angle), s = orc_sin(car->angle);
  double vf = car->vx * c + car->vy * s;
  double vl = (-car->vx) * s + car->vy * c;
  obs[n_sensors + 0] = (float)rx_clip(vf / ORC_MAX_SPEED, -1.0, 1.0);
  obs[n_sensors + 1] = (float)rx_clip(vl / ORC_MAX_SPEED, -1.0, 1.0);
  obs[n_sensors + 2] = (float)rx_clip(0.0 / ORC_STEER_SPEED, -1.0, 1.0);
  obs[n_sensors + 3] = (float)last_steering;
  const orc_car* o = &cars[1 - a];
  double rx = o->x - car->x, ry = o->y - car->y;
  double lrx = rx * c + ry * s;
  double lry = (-rx) * s + ry * c;
  double rvx = o->vx - car->vx, rvy = o->vy - car->vy;
  double lvx = rvx * c + rvy * s;
  double lvy = (-rvx) * s + rvy * c;
  obs[n_sensors + 4] = (float)rx_clip(lrx / maxd, -1.0, 1.0);
  obs[n_sensors + 5] = (float)rx_clip(lry / maxd, -1.0, 1.0);
  obs[n_sensors + 6] = (float)rx_clip(lvx / ORC_MAX_SPEED, -1.0, 1.0);
  obs[n_sensors + 7] = (float)rx_clip(lvy / ORC_MAX_SPEED, -1.0, 1.0);
}

/* MultiRacingEnv.reset -- environment/multi_racing_env.py:118-153.
 * first[e] = agent_order[0] after np.random.shuffle (injected; the reference
 * draws it from the global numpy RNG). */
void orc_multi_reset(int n, const orc_tracks* T, orc_multi_state st, const uint8_t* mask, const uint8_t* first,
                     int n_sensors, const double* rel_angles, float* obs) {
  int D = n_sensors + 8;
  for (int e = 0; e < n; ++e) {
    if (mask && !mask[e]) continue;
    int k = st.track[e];
    const double* m = T->meta + 8 * k;
    orc_car cars[2];
    for (int a = 0; a < 2; ++a) {
      int pos_idx = (first[e] == a) ? 0 : 1; /* agent_order.index(i) */
      double offset = ((double)pos_idx - 0.5) * 3.5;
      cars[a].x = m[0] + m[5] * offset;
      cars[a].y = m[1] + m[6] * offset;
      cars[a].angle = m[2];
      cars[a].vx = cars[a].vy = 0.0;
      cars[a].progress = 0.0;
      cars[a].crashed = 0;
      size_t i = 2 * (size_t)e + a;
      st.x[i] = cars[a].x;
      st.y[i] = cars[a].y;
      st.angle[i] = cars[a].angle;
      st.vx[i] = st.vy[i] = 0.0;
      st.progress[i] = 0.0;
      st.last_progress[i] = 0.0;
      st.last_steering[i] = 0.0;
      st.finished_step[i] = -1;
      st.flags[i] = 0;
    }
    st.steps[e] = 0;
    for (int a = 0; a < 2; ++a)
      orc_multi_obs(T, k, cars, a, 0.0, n_sensors, rel_angles, obs + ((size_t)e * 2 + a) * D);
  }
}

/* MultiRacingEnv.calc_reward -- environment/multi_racing_env.py:155-196 */
static double orc_multi_reward(orc_car* car, uint8_t* fl, int32_t* finished_step, double last_progress, int steps) {
  double p = car->progress;
  double pd = p - last_progress;
  if (last_progress > 0.9 && p < 0.1)
    pd = (1.0 - last_progress) + p;
  else if (last_progress < 0.1 && p > 0.9)
    pd = -((1.0 - p) + last_progress);
  double r = 0.0;
  r += pd * 200;
  if (!car->crashed && pd > 0) {
    double speed = sqrt(orc_pow2(car->vx) + orc_pow2(car->vy));
    double ratio = rx_clip(speed / ORC_MAX_SPEED, 0.0, 1.0);
    r += ratio * 18;
  }
  if (!(*fl & F_CP25) && 0.25 <= p && p < 0.35) { *fl |= F_CP25; r += 25; }
  if ((*fl & F_CP25) && !(*fl & F_CP50) && 0.50 <= p && p < 0.60) { *fl |= F_CP50; r += 25; }
  if ((*fl & F_CP50) && !(*fl & F_CP75) && 0.75 <= p && p < 0.85) { *fl |= F_CP75; r += 25; }
  int all_cp = (*fl & (F_CP25 | F_CP50 | F_CP75)) == (F_CP25 | F_CP50 | F_CP75);
  if (all_cp && last_progress > 0.9 && p < 0.1 && pd > 0) {
    *fl |= F_FINISHED;
    *finished_step = steps;
    double tb = 300 - ((double)steps / 15);
    r += 100 + (tb > 0 ? tb : 0.0);
  }
  if (car->crashed && !(*fl & F_HAS_CRASHED)) {
    r -= 160;
    *fl |= F_HAS_CRASHED;
  }
  return r;
}

/* MultiRacingEnv.step -- environment/multi_racing_env.py:213-269 (2 agents).
 * obs [n][2][D], reward [n][2], done [n] (= terminated), done_all [n],
 * truncated [n], placement [n][2] (0 if not terminal),
 * info [n][2][2] = speed, progress */
void orc_multi_step(int n, const orc_tracks* T, orc_multi_state st, const float* actions, int n_sensors,
                    const double* rel_angles, float* obs, double* reward, uint8_t* done, uint8_t* done_all,
                    uint8_t* truncated, int32_t* placement, double* info) {
  int D = n_sensors + 8;
  for (int e = 0; e < n; ++e) {
    int k = st.track[e];
    int W = T->wp_off[k + 1] - T->wp_off[k];
    const double* wp = T->wp + 2 * (size_t)T->wp_off[k];
    const double* nrm = T->nrm + 2 * (size_t)T->wp_off[k];
    double width = T->meta[8 * k + 3];
    orc_car cars[2];
    uint8_t fl[2];
    for (int a = 0; a < 2; ++a) {
      size_t i = 2 * (size_t)e + a;
      cars[a].x = st.x[i];
      cars[a].y = st.y[i];
      cars[a].angle = st.angle[i];
      cars[a].vx = st.vx[i];
      cars[a].vy = st.vy[i];
      cars[a].progress = st.progress[i];
      fl[a] = st.flags[i];
      cars[a].crashed = (fl[a] & F_CRASHED) != 0;
    }
    double steer[2];
    for (int a = 0; a < 2; ++a) { /* :216-220 */
      float a0 = actions[4 * e + 2 * a], a1 = actions[4 * e + 2 * a + 1];
      steer[a] = (double)orc_clipf(a0, -1.0f, 1.0f);
      float thr = orc_clipf((a1 + 1.0f) / 2.0f, 0.0f, 1.0f);
      orc_car_update(&cars[a], steer[a], (double)thr, wp, nrm, W, width);
    }
    double pen[2] = {0.0, 0.0};
    { /* :222-231 */
      double ax[4], ay[4], bx[4], by[4];
      orc_corners(cars[0].x, cars[0].y, cars[0].angle, ax, ay);
      orc_corners(cars[1].x, cars[1].y, cars[1].angle, bx, by);
      if (orc_rect_intersect(ax, ay, bx, by)) {
        for (int a = 0; a < 2; ++a) {
          cars[a].vx *= 0.92;
          cars[a].vy *= 0.92;
          pen[a] += -5.0;
        }
      }
    }
    int steps = st.steps[e] + 1;
    double r[2];
    for (int a = 0; a < 2; ++a) {
      size_t i = 2 * (size_t)e + a;
      fl[a] = (uint8_t)((fl[a] & ~F_CRASHED) | (cars[a].crashed ? F_CRASHED : 0));
      r[a] = orc_multi_reward(&cars[a], &fl[a], &st.finished_step[i], st.last_progress[i], steps) + pen[a];
    }
    for (int a = 0; a < 2; ++a) {
      size_t i = 2 * (size_t)e + a;
      orc_multi_obs(T, k, cars, a, steer[a], n_sensors, rel_angles, obs + i * D);
      if (info) {
        info[2 * i + 0] = sqrt(orc_pow2(cars[a].vx) + orc_pow2(cars[a].vy));
        info[2 * i + 1] = (fl[a] & F_FINISHED) ? 1.0 : cars[a].progress;
      }
    }
    int any_fin = (fl[0] & F_FINISHED) || (fl[1] & F_FINISHED);
    int all_crash = cars[0].crashed && cars[1].crashed;
    int term = any_fin || all_crash;
    int trunc = steps >= 3000;
    placement[2 * e] = placement[2 * e + 1] = 0;
    if (term || trunc) { /* place(), :198-211 */
      double sc[2];
      for (int a = 0; a < 2; ++a) {
        size_t i = 2 * (size_t)e + a;
        int fs = st.finished_step[i];
        double v = (double)((fl[a] & F_FINISHED) ? 10000 : 0) + cars[a].progress * 100;
        v = v + (double)(cars[a].crashed ? 0 : 10);
        v = v + 1.0 / (double)(fs > 0 ? fs : 10000);
        sc[a] = v;
      }
      /* sorted((score, idx), reverse=True): ties -> larger idx first */
      int firstp = (sc[1] > sc[0] || sc[1] == sc[0]) ? 1 : 0;
      placement[2 * e + firstp] = 1;
      placement[2 * e + (1 - firstp)] = 2;
      r[firstp] += 250;
    }
    for (int a = 0; a < 2; ++a) {
      size_t i = 2 * (size_t)e + a;
      reward[i] = r[a];
      st.x[i] = cars[a].x;
      st.y[i] = cars[a].y;
      st.angle[i] = cars[a].angle;
      st.vx[i] = cars[a].vx;
      st.vy[i] = cars[a].vy;
      st.progress[i] = cars[a].progress;
      st.last_progress[i] = cars[a].progress; /* :267-268 */
      st.last_steering[i] = steer[a];
      st.flags[i] = fl[a];
    }
    st.steps[e] = steps;
    done[e] = (uint8_t)term;
    done_all[e] = (uint8_t)(term || trunc);
    truncated[e] = (uint8_t)trunc;
  }
}

/* ------------------------------------------------------------ agent/ppo.py */

/* PPO.compute_advantages -- agent/ppo.py:134-154 (float32, no FMA).
 * gamma_f = float(gamma); gl_f = float(gamma * gae_lambda) (the Python double
 * product is rounded to f32 once when it multiplies the tensor). */
void orc_gae(int T, int N, const float* rewards, const float* values, const float* dones, const float* next_value,
             const uint8_t* next_done, float gamma_f, float gl_f, float* adv, float* ret) {
  for (int n = 0; n < N; ++n) {
    float run = 0.0f;
    for (int t = T - 1; t >= 0; --t) {
      float nnt, nv;
      if (t == T - 1) {
        nnt = 1.0f - (float)next_done[n];
        nv = next_value[n];
      } else {
        nnt = 1.0f - dones[(size_t)(t + 1) * N + n];
        nv = values[(size_t)(t + 1) * N + n];
      }
      float delta = (rewards[(size_t)t * N + n] + (gamma_f * nnt) * nv) - values[(size_t)t * N + n];
      run = delta + (gl_f * nnt) * run;
      adv[(size_t)t * N + n] = run;
      ret[(size_t)t * N + n] = run + values[(size_t)t * N + n];
    }
  }
}

/* test hook: the libm mode this build was compiled with */
int orc_device_libm(void) {
#ifdef ORC_DEVICE_LIBM
  return 1;
#else
  return 0;
#endif
}

void orc_sincos_dev(int n, const double* x, double* s, double* c) {
  for (int i = 0; i < n; ++i) rx_sincos(x[i], &s[i], &c[i]);
}
