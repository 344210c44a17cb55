"""ctypes binding for the C oracle (oracle/rx_oracle.c) -- TEST INFRASTRUCTURE ONLY.

Loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
as the checker.  Every function mirrors the reference function named in its
docstring (file:line under the reference root).

All state is struct-of-arrays numpy (float64 / int32 / uint8), the same layout
the device uses (include/rx.h), so a test can hand identical arrays to both.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(HERE, "build")

F_CRASHED, F_FINISHED, F_CP25, F_CP50, F_CP75, F_HAS_CRASHED = 1, 2, 4, 8, 16, 32

_P = ctypes.c_void_p


def build(force=False):
    """Compile liboracle.so / liboracle_dev.so with gcc (oracle/Makefile)."""
    libs = [os.path.join(BUILD, n) for n in ("liboracle.so", "liboracle_dev.so")]
    if force or not all(os.path.exists(p) for p in libs):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return libs


class OrcTracks(ctypes.Structure):
    _fields_ = [("n_tracks", ctypes.c_int), ("wp_off", _P), ("wp", _P), ("nrm", _P), ("seg", _P), ("meta", _P)]


class OrcSingleState(ctypes.Structure):
    _fields_ = [(k, _P) for k in ("x", "y", "angle", "vx", "vy", "progress", "last_progress", "last_steering",
                                  "steps", "track", "flags")]


class OrcMultiState(ctypes.Structure):
    _fields_ = [(k, _P) for k in ("x", "y", "angle", "vx", "vy", "progress", "last_progress", "last_steering",
                                  "finished_step", "flags", "steps", "track")]


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


class TrackTable:
    """Host copy of the device track-table layout (include/rx.h).

    wp_off int32 [n+1]; wp, nrm float64 [Wtot,2]; seg float64 [2*Wtot,4] =
    (start.x, start.y, v2.x, v2.y), left boundary segments then right ones per
    track (environment/track.py:134-148); meta float64 [n,8] = start x, y,
    angle, width, max_track_distance, normals[0].x, normals[0].y, 0.
    """

    def __init__(self, tracks):
        # tracks: list of dicts with wp, nrm, starts, v2, start(3), width, maxd
        W = [len(t["wp"]) for t in tracks]
        self.wp_off = np.concatenate([[0], np.cumsum(W)]).astype(np.int32)
        self.wp = np.ascontiguousarray(np.concatenate([t["wp"] for t in tracks]), dtype=np.float64)
        self.nrm = np.ascontiguousarray(np.concatenate([t["nrm"] for t in tracks]), dtype=np.float64)
        self.seg = np.ascontiguousarray(np.concatenate(
            [np.concatenate([t["starts"], t["v2"]], axis=1) for t in tracks]), dtype=np.float64)
        meta = np.zeros((len(tracks), 8), dtype=np.float64)
        for k, t in enumerate(tracks):
            meta[k, 0:3] = t["start"]
            meta[k, 3] = t["width"]
            meta[k, 4] = t["maxd"]
            meta[k, 5:7] = t["nrm"][0]
        self.meta = meta
        self.n = len(tracks)

    def c(self):
        return OrcTracks(self.n, _ptr(self.wp_off), _ptr(self.wp), _ptr(self.nrm), _ptr(self.seg), _ptr(self.meta))

    def segments(self, k):
        a, b = 2 * self.wp_off[k], 2 * self.wp_off[k + 1]
        return self.seg[a:b]

    def waypoints(self, k):
        return self.wp[self.wp_off[k]:self.wp_off[k + 1]]


def single_state(n):
    d = {k: np.zeros(n, dtype=np.float64) for k in ("x", "y", "angle", "vx", "vy", "progress", "last_progress",
                                                    "last_steering")}
    d["steps"] = np.zeros(n, dtype=np.int32)
    d["track"] = np.zeros(n, dtype=np.int32)
    d["flags"] = np.zeros(n, dtype=np.uint8)
    return d


def multi_state(n):
    d = {k: np.zeros((n, 2), dtype=np.float64) for k in ("x", "y", "angle", "vx", "vy", "progress", "last_progress",
                                                         "last_steering")}
    d["finished_step"] = np.full((n, 2), -1, dtype=np.int32)
    d["flags"] = np.zeros((n, 2), dtype=np.uint8)
    d["steps"] = np.zeros(n, dtype=np.int32)
    d["track"] = np.zeros(n, dtype=np.int32)
    return d


class Oracle:
    """One build of the oracle.  device_libm=False -> glibc numerics (reference)."""

    def __init__(self, device_libm=False):
        glibc, dev = build()
        self.lib = ctypes.CDLL(dev if device_libm else glibc)
        L = self.lib
        L.orc_raycast.restype = ctypes.c_double
        L.orc_raycast.argtypes = [_P, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double]
        L.orc_closest_wp.restype = ctypes.c_int
        L.orc_closest_wp.argtypes = [_P, ctypes.c_int, ctypes.c_double, ctypes.c_double]
        L.orc_single_step.argtypes = [ctypes.c_int, ctypes.POINTER(OrcTracks), OrcSingleState, _P, _P, ctypes.c_int,
                                      _P, _P, _P, _P, _P, _P]
        L.orc_single_reset.argtypes = [ctypes.c_int, ctypes.POINTER(OrcTracks), OrcSingleState, _P, ctypes.c_int, _P,
                                       _P, _P]
        L.orc_multi_step.argtypes = [ctypes.c_int, ctypes.POINTER(OrcTracks), OrcMultiState, _P, ctypes.c_int, _P, _P,
                                     _P, _P, _P, _P, _P, _P]
        L.orc_multi_reset.argtypes = [ctypes.c_int, ctypes.POINTER(OrcTracks), OrcMultiState, _P, _P, ctypes.c_int,
                                      _P, _P]
        L.orc_gae.argtypes = [ctypes.c_int, ctypes.c_int, _P, _P, _P, _P, _P, ctypes.c_float, ctypes.c_float, _P, _P]
        L.orc_sincos_dev.argtypes = [ctypes.c_int, _P, _P, _P]
        L.orc_device_libm.restype = ctypes.c_int
        self.device_libm = bool(L.orc_device_libm())

    # --- environment/track.py
    def raycast(self, seg, ox, oy, direction, max_dist=50.0):
        """Track.raycast -- environment/track.py:173-199"""
        seg = np.ascontiguousarray(seg, dtype=np.float64)
        return self.lib.orc_raycast(_ptr(seg), len(seg), ox, oy, direction, max_dist)

    def closest_wp(self, wp, x, y):
        """Track.closest_waypoint_idx -- environment/track.py:150-152"""
        wp = np.ascontiguousarray(wp, dtype=np.float64)
        return self.lib.orc_closest_wp(_ptr(wp), len(wp), x, y)

    # --- environment/racing_env.py
    @staticmethod
    def _sstate(st):
        for k, v in st.items():
            assert v.flags["C_CONTIGUOUS"], k
        return OrcSingleState(*[_ptr(st[k]) for k, _ in OrcSingleState._fields_])

    def single_reset(self, table, st, rel_angles, mask=None):
        """RacingEnv.reset -- environment/racing_env.py:86-102 (all envs, or where mask)"""
        n = len(st["x"])
        D = len(rel_angles) + 4
        obs = np.zeros((n, D), dtype=np.float32)
        rel = np.ascontiguousarray(rel_angles, dtype=np.float64)
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        tc = table.c()
        self.lib.orc_single_reset(n, ctypes.byref(tc), self._sstate(st), _ptr(m), len(rel), _ptr(rel), _ptr(obs), None)
        return obs

    def single_step(self, table, st, actions, rel_angles, speed_weight=8.0):
        """RacingEnv.step -- environment/racing_env.py:104-167 (batched, in place on st)"""
        n = len(st["x"])
        D = len(rel_angles) + 4
        act = np.ascontiguousarray(actions, dtype=np.float32).reshape(n, 2)
        sw = np.ascontiguousarray(np.broadcast_to(np.asarray(speed_weight, dtype=np.float64), (n,)))
        rel = np.ascontiguousarray(rel_angles, dtype=np.float64)
        obs = np.zeros((n, D), dtype=np.float32)
        rew = np.zeros(n, dtype=np.float64)
        term = np.zeros(n, dtype=np.uint8)
        trunc = np.zeros(n, dtype=np.uint8)
        info = np.zeros((n, 3), dtype=np.float64)
        tc = table.c()
        self.lib.orc_single_step(n, ctypes.byref(tc), self._sstate(st), _ptr(act), _ptr(sw), len(rel), _ptr(rel),
                                 _ptr(obs), _ptr(rew), _ptr(term), _ptr(trunc), _ptr(info))
        return obs, rew, term.astype(bool), trunc.astype(bool), info

    # --- environment/multi_racing_env.py
    @staticmethod
    def _mstate(st):
        for k, v in st.items():
            assert v.flags["C_CONTIGUOUS"], k
        return OrcMultiState(*[_ptr(st[k]) for k, _ in OrcMultiState._fields_])

    def multi_reset(self, table, st, first, rel_angles, mask=None):
        """MultiRacingEnv.reset -- environment/multi_racing_env.py:118-153 (agent order injected)"""
        n = len(st["steps"])
        D = len(rel_angles) + 8
        obs = np.zeros((n, 2, D), dtype=np.float32)
        rel = np.ascontiguousarray(rel_angles, dtype=np.float64)
        f = np.ascontiguousarray(np.broadcast_to(np.asarray(first, dtype=np.uint8), (n,)))
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        tc = table.c()
        self.lib.orc_multi_reset(n, ctypes.byref(tc), self._mstate(st), _ptr(m), _ptr(f), len(rel), _ptr(rel),
                                 _ptr(obs))
        return obs

    def multi_step(self, table, st, actions, rel_angles):
        """MultiRacingEnv.step -- environment/multi_racing_env.py:213-269"""
        n = len(st["steps"])
        D = len(rel_angles) + 8
        act = np.ascontiguousarray(actions, dtype=np.float32).reshape(n, 2, 2)
        rel = np.ascontiguousarray(rel_angles, dtype=np.float64)
        obs = np.zeros((n, 2, D), dtype=np.float32)
        rew = np.zeros((n, 2), dtype=np.float64)
        done = np.zeros(n, dtype=np.uint8)
        done_all = np.zeros(n, dtype=np.uint8)
        trunc = np.zeros(n, dtype=np.uint8)
        place = np.zeros((n, 2), dtype=np.int32)
        info = np.zeros((n, 2, 2), dtype=np.float64)
        tc = table.c()
        self.lib.orc_multi_step(n, ctypes.byref(tc), self._mstate(st), _ptr(act), len(rel), _ptr(rel), _ptr(obs),
                                _ptr(rew), _ptr(done), _ptr(done_all), _ptr(trunc), _ptr(place), _ptr(info))
        return obs, rew, done.astype(bool), done_all.astype(bool), trunc.astype(bool), place, info

    # --- agent/ppo.py
    def gae(self, rewards, values, dones, next_value, next_done, gamma, gae_lambda):
        """PPO.compute_advantages -- agent/ppo.py:134-154"""
        T, N = rewards.shape
        r = np.ascontiguousarray(rewards, dtype=np.float32)
        v = np.ascontiguousarray(values, dtype=np.float32)
        d = np.ascontiguousarray(dones, dtype=np.float32)
        nv = np.ascontiguousarray(next_value, dtype=np.float32)
        nd = np.ascontiguousarray(next_done, dtype=np.uint8)
        adv = np.zeros((T, N), dtype=np.float32)
        ret = np.zeros((T, N), dtype=np.float32)
        self.lib.orc_gae(T, N, _ptr(r), _ptr(v), _ptr(d), _ptr(nv), _ptr(nd), np.float32(gamma),
                         np.float32(gamma * gae_lambda), _ptr(adv), _ptr(ret))
        return adv, ret

    def sincos_dev(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        s = np.empty_like(x)
        c = np.empty_like(x)
        self.lib.orc_sincos_dev(len(x), _ptr(x), _ptr(s), _ptr(c))
        return s, c


def sensor_angles(n_sensors=11, half_cone=np.pi / 3):
    """np.linspace(-cone, cone, n) -- racing_env.py:45 (pi/3), multi_racing_env.py:50 (pi/2)"""
    return np.linspace(-half_cone, half_cone, n_sensors)
