"""NumPy restatement of the reference's single-agent env step -- TEST / BASELINE
INFRASTRUCTURE ONLY.

This is the CPU baseline bench.py times beside the GPU (``cpu_baseline``,
kind "port"): it keeps the reference's execution model -- one Python object
per env, a Python loop over envs (SyncVectorEnv), numpy vectorised over the
track segments inside each of the 11 raycasts -- so its env-steps/s is the
reference's CPU cost structure on the GPU box's own host cores.  The
reference itself cannot travel to the GPU box.  tests/test_oracle_golden.py
pins this restatement bit-for-bit against the reference's golden vectors.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
"""
import numpy as np

MAX_SPEED, ACCEL, STEER, DRAG, LAT, GRIP = 30.0, 10.0, 3.0, 0.985, 0.85, 0.9  # environment/car.py:4-11
TWO_PI = 2 * np.pi


class NpTrack:
    """Track query methods over precomputed geometry (environment/track.py:150-199)."""

    def __init__(self, waypoints, normals, starts, v2, width, start_pose):
        self.waypoints = np.asarray(waypoints, dtype=np.float64)
        self.normals = np.asarray(normals, dtype=np.float64)
        self.starts = np.asarray(starts, dtype=np.float64)
        self.v2 = np.asarray(v2, dtype=np.float64)
        self.track_width = width
        self.start_pose = tuple(start_pose)

    def closest(self, x, y):  # track.py:150-152
        return int(np.sum((self.waypoints - np.array((x, y))) ** 2, axis=1).argmin())

    def collide(self, corners):  # track.py:163-171
        for c in corners:
            i = self.closest(c[0], c[1])
            if abs(np.dot(c - self.waypoints[i], self.normals[i])) > self.track_width:
                return True
        return False

    def raycast(self, origin, direction, max_dist=50.0):  # track.py:173-199
        rd = np.array([np.cos(direction), np.sin(direction)])
        v1 = origin - self.starts
        v3 = np.array([-rd[1], rd[0]])
        dotp = np.sum(self.v2 * v3, axis=1)
        ok = np.abs(dotp) > 1e-10
        if not ok.any():
            return max_dist
        cr = self.v2[:, 0] * v1[:, 1] - self.v2[:, 1] * v1[:, 0]
        t = np.full(len(self.starts), max_dist)
        t[ok] = cr[ok] / dotp[ok]
        dp = np.sum(v1 * v3, axis=1)
        s = np.full(len(self.starts), -1.0)
        s[ok] = dp[ok] / dotp[ok]
        hit = ok & (t >= 0) & (s >= 0) & (s <= 1)
        return float(np.min(t[hit])) if hit.any() else max_dist


_LOCAL = np.array([[2.0, 1.0], [2.0, -1.0], [-2.0, -1.0], [-2.0, 1.0]])


class NpRacingEnv:
    """environment/racing_env.py + car.py, numpy, one env."""

    def __init__(self, track, num_sensors=11, speed_weight=8.0):
        self.track = track
        self.num_sensors = num_sensors
        self.speed_weight = speed_weight
        self.angles = np.linspace(-np.pi / 3, np.pi / 3, num_sensors)
        self.reset()

    def reset(self):
        self.x, self.y, self.angle = self.track.start_pose
        self.vx = self.vy = 0.0
        self.progress = 0.0
        self.crashed = self.finished = False
        self.steps = 0
        self.last_progress = 0.0
        self.last_steering = 0.0
        self.cp = [False, False, False]
        return self.obs()

    def corners(self):  # car.py:26-43
        c, s = np.cos(self.angle), np.sin(self.angle)
        return (np.array([[c, -s], [s, c]]) @ _LOCAL.T).T + np.array([self.x, self.y])

    def update(self, steering, throttle, dt=0.05):  # car.py:45-80
        if self.crashed:
            return
        self.angle = (self.angle + (steering * STEER * dt)) % TWO_PI
        c, s = np.cos(self.angle), np.sin(self.angle)
        vf = self.vx * c + self.vy * s
        vl = self.vx * (-s) + self.vy * c
        vf = (vf + ((throttle * ACCEL) * dt)) * DRAG
        vl = vl * LAT * GRIP
        self.vx = vf * np.cos(self.angle) - vl * np.sin(self.angle)
        self.vy = vf * np.sin(self.angle) + vl * np.cos(self.angle)
        sp = np.sqrt((self.vx ** 2) + (self.vy ** 2))
        if sp > MAX_SPEED:
            k = MAX_SPEED / sp
            self.vx *= k
            self.vy *= k
        self.x = self.x + (self.vx * dt)
        self.y = self.y + (self.vy * dt)
        self.progress = self.track.closest(self.x, self.y) / len(self.track.waypoints)
        self.crashed = self.track.collide(self.corners())

    def obs(self):  # racing_env.py:44-75
        d = np.zeros(self.num_sensors, dtype=np.float32)
        o = np.array([self.x, self.y])
        for i, a in enumerate(self.angles):
            d[i] = self.track.raycast(o, self.angle + a, 50.0)
        d = d / 50.0
        c, s = np.cos(self.angle), np.sin(self.angle)
        vf = np.clip((self.vx * c + self.vy * s) / MAX_SPEED, -1.0, 1.0)
        vl = np.clip((-self.vx * s + self.vy * c) / MAX_SPEED, -1.0, 1.0)
        av = np.clip(0.0 / STEER, -1.0, 1.0)
        return np.concatenate([d, [vf, vl, av, self.last_steering]]).astype(np.float32)

    def step(self, action):  # racing_env.py:104-167
        steering = float(np.clip(action[0], -1.0, 1.0))
        throttle = float(np.clip(action[1], 0.0, 1.0))
        self.last_steering = steering
        self.update(steering, throttle)
        self.steps += 1
        p, lp = self.progress, self.last_progress
        pd = p - lp
        if lp > 0.9 and p < 0.1:
            pd = (1.0 - lp) + p
        elif lp < 0.1 and p > 0.9:
            pd = -((1.0 - p) + lp)
        r = pd * 200
        for k, (lo, hi) in enumerate(((0.25, 0.35), (0.50, 0.60), (0.75, 0.85))):
            if (k == 0 or self.cp[k - 1]) and not self.cp[k] and lo <= p < hi:
                self.cp[k] = True
                r += 20
        if not self.crashed and pd > 0:
            r += np.clip(np.sqrt(self.vx ** 2 + self.vy ** 2) / MAX_SPEED, 0.0, 1.0) * self.speed_weight
        if self.crashed:
            r -= 60
        if all(self.cp) and lp > 0.9 and p < 0.1 and pd > 0:
            self.finished = True
            r += 100
            r += max(0, 200 - (self.steps / 10))
        obs = self.obs()
        term = self.crashed or self.finished
        trunc = self.steps >= 3000
        self.last_progress = p
        return obs, r, term, trunc


class NpSyncVectorEnv:
    """SyncVectorEnv-style sequential loop with NEXT_STEP autoreset."""

    def __init__(self, envs):
        self.envs = envs
        self.pending = np.zeros(len(envs), dtype=bool)

    def reset(self):
        self.pending[:] = False
        return np.stack([e.reset() for e in self.envs])

    def step(self, actions):
        n = len(self.envs)
        obs = np.zeros((n, self.envs[0].num_sensors + 4), np.float32)
        rew = np.zeros(n)
        term = np.zeros(n, bool)
        trunc = np.zeros(n, bool)
        for i, e in enumerate(self.envs):
            if self.pending[i]:
                obs[i] = e.reset()
            else:
                obs[i], rew[i], term[i], trunc[i] = e.step(actions[i])
        self.pending = term | trunc
        return obs, rew, term, trunc


def make_track(geom):
    """NpTrack from a dict with wp, nrm, starts, v2, width, start (golden / TrackGeometry)."""
    return NpTrack(geom["wp"], geom["nrm"], geom["starts"], geom["v2"], geom["width"], geom["start"])
