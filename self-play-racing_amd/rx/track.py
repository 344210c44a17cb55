"""Host-side track generation and the device track table.

Restates environment/track.py's generation and geometry (SURVEY.md §8(a) rows
A1, A2, A7) with the same numpy/scipy calls in the same order, so waypoints,
normals and boundary segments are bit-identical to the reference's
(tests/test_track_host.py checks them against the golden vectors).  What is
new is what happens around them:

* ``gen_tracks(..., seed=s)`` reseeds the global RNG inside every track
  (track.py:5-6), so the per-track draws cycle through at most five states;
  the generator memoises that cycle instead of re-drawing 65,536 times, and
  leaves the global RNG exactly where the reference would.
* ``TrackSet`` deduplicates (control points, width) pairs into slots -- seed 1
  gives 7 slots for any number of envs -- and packs them into the flat
  struct-of-arrays table the kernels read (include/rx.h rx_upload_tracks);
  ``TrackSet.save`` / ``TrackSet.load`` keep that table (plus the control
  points and, optionally, the env -> slot assignment) in one ``.npz`` file, so
  a 65,536-env pool is rebuilt without regenerating or re-splining anything
  (format in DESIGN.md).
"""
import numpy as np
from scipy.interpolate import CubicSpline

TWO_PI = 2 * np.pi

DEFAULT_CONTROL_POINTS = np.array([
    [0, 0], [50, 0], [70, 20], [60, 40],
    [70, 50], [50, 70], [20, 70], [10, 50],
    [10, 20], [0, 10],
])  # environment/track.py:70-74 (integer array, as in the reference)
DEFAULT_WIDTH = 6.0  # environment/track.py:77-80


def gen_random_track(num_points=15, base_radius=50, radius_variation=15, angle_jitter=0.2, smoothness=0.5,
                     seed=None):
    """Random closed control polygon -- environment/track.py:4-45.

    Same global-RNG draws in the same order: n jitter offsets, then n radius
    variations (drawn one per point, as the reference's loop does)."""
    rs = np.random
    if seed is not None:
        rs.seed(seed)
    ang = np.linspace(0, TWO_PI, num_points, endpoint=False)
    if angle_jitter > 0:
        half = angle_jitter * (TWO_PI / num_points) / 2
        ang = np.sort((ang + rs.uniform(-half, half, num_points)) % TWO_PI)
    r = np.zeros(num_points)
    for i in range(num_points):
        v = base_radius + rs.uniform(-radius_variation, radius_variation)
        r[i] = v if (smoothness <= 0 or i == 0) else (1 - smoothness) * v + (smoothness * r[i - 1])
    if smoothness > 0:
        r[0] = (r[0] + r[-1]) / 2
    return np.column_stack([r * np.cos(ang), r * np.sin(ang)])


def _draw_params():
    # environment/track.py:50-54, global RNG
    n = np.random.randint(10, 15)
    base = np.random.randint(50, 80)
    var = np.random.randint(10, base // 2 - 10)
    jit = np.random.uniform(0.2, 0.7)
    smooth = np.random.uniform(0.2, 0.7)
    return n, base, var, jit, smooth


def gen_tracks(num_tracks=10, seed=None):
    """environment/track.py:47-56, with the reseed cycle memoised.

    With ``seed`` set, every track's draws start from the RNG state that
    ``np.random.seed(seed)`` plus the previous track's 2*n uniform draws left
    behind, i.e. a function of the previous track's point count only.  The
    loop therefore caches (prev point count) -> (control points, point count,
    RNG state after) and replays it; the returned arrays for equal tracks are
    the same read-only object.  The global RNG ends in the reference's state.
    """
    out = []
    if seed is None or num_tracks <= 0:
        for _ in range(num_tracks):
            out.append(gen_random_track(*_draw_params(), seed))
        return out
    p = _draw_params()
    cp = gen_random_track(*p, seed)
    cp.setflags(write=False)
    out.append(cp)
    prev_n = p[0]
    state_after = None
    memo = {}
    for _ in range(1, num_tracks):
        hit = memo.get(prev_n)
        if hit is None:
            if state_after is not None:  # resync the real RNG before drawing anew
                np.random.set_state(state_after)
            q = _draw_params()
            c = gen_random_track(*q, seed)
            c.setflags(write=False)
            hit = (c, q[0], np.random.get_state())
            memo[prev_n] = hit
        cp, prev_n, state_after = hit
        out.append(cp)
    if state_after is not None:
        np.random.set_state(state_after)
    return out


class TrackGeometry:
    """Track.__init__ geometry -- environment/track.py:61-148, 154-157.

    Attributes mirror the reference's: waypoints [W,2], normals [W,2],
    left_boundary/right_boundary, segment_cache {'starts','ends','v2'} [2W,2],
    track_bounds, max_track_distance, track_width, start pose."""

    def __init__(self, control_points=None, track_width=None, factor=30):
        cp = DEFAULT_CONTROL_POINTS if control_points is None else control_points
        self.control_points = cp
        self.track_width = DEFAULT_WIDTH if track_width is None else track_width
        # gen_waypoints, track.py:100-115 (chord-length periodic cubic spline)
        closed = np.vstack((cp, cp[0]))
        chord = np.sqrt(np.sum(np.diff(closed, axis=0) ** 2, axis=1))
        t = np.concatenate(([0], np.cumsum(chord)))
        sx = CubicSpline(t, closed[:, 0], bc_type="periodic")
        sy = CubicSpline(t, closed[:, 1], bc_type="periodic")
        tw = np.linspace(0, t[-1], len(cp) * factor, endpoint=False)
        self.waypoints = np.column_stack((sx(tw), sy(tw)))
        wp = self.waypoints
        # track_bounds / max_track_distance, track.py:82-91 (np.float64 ** 2 is pow())
        lo_x, hi_x = wp[:, 0].min(), wp[:, 0].max()
        lo_y, hi_y = wp[:, 1].min(), wp[:, 1].max()
        self.track_bounds = {"min_x": lo_x, "max_x": hi_x, "min_y": lo_y, "max_y": hi_y}
        self.max_track_distance = np.sqrt((hi_x - lo_x) ** 2 + (hi_y - lo_y) ** 2)
        # calc_normals, track.py:117-124
        tang = np.diff(wp, axis=0, append=[wp[0]])
        tl = np.linalg.norm(tang, axis=1, keepdims=True)
        tang = tang / np.where(tl == 0, 1, tl)
        self.normals = np.column_stack((-tang[:, 1], tang[:, 0]))
        # boundaries and the segment cache, track.py:93-96, 126-148
        self.left_boundary = wp + self.normals * self.track_width
        self.right_boundary = wp - self.normals * self.track_width
        starts = np.vstack([self.left_boundary, self.right_boundary])
        ends = np.vstack([np.roll(self.left_boundary, -1, axis=0), np.roll(self.right_boundary, -1, axis=0)])
        self.segment_cache = {"starts": starts, "ends": ends, "v2": ends - starts}

    @classmethod
    def from_arrays(cls, control_points, track_width, waypoints, normals, seg, max_track_distance):
        """Rebuild from a stored table slot (no spline): every attribute is an
        exact function of the stored arrays."""
        self = cls.__new__(cls)
        self.control_points = control_points
        self.track_width = track_width
        self.waypoints = waypoints
        wp = waypoints
        self.track_bounds = {"min_x": wp[:, 0].min(), "max_x": wp[:, 0].max(), "min_y": wp[:, 1].min(),
                             "max_y": wp[:, 1].max()}
        self.max_track_distance = np.float64(max_track_distance)
        self.normals = normals
        W = len(wp)
        starts, v2 = seg[:, :2].copy(), seg[:, 2:].copy()
        self.left_boundary, self.right_boundary = starts[:W], starts[W:]
        ends = np.vstack([np.roll(self.left_boundary, -1, axis=0), np.roll(self.right_boundary, -1, axis=0)])
        self.segment_cache = {"starts": starts, "ends": ends, "v2": v2}
        return self

    def get_start_pos(self):
        """track.py:154-157"""
        wp = self.waypoints
        return (wp[0, 0], wp[0, 1], np.arctan2(wp[1, 1] - wp[0, 1], wp[1, 0] - wp[0, 0]))


def _geoms_worker(args):
    """Worker of TrackSet.build (a spawned process: numpy / scipy only): the
    packed table rows of its tracks (TrackSet.arrays layout), not the objects --
    pickling every TrackGeometry back cost more than the splines."""
    items, factor = args
    g = [TrackGeometry(cp, w, factor) for cp, w in items]
    return TrackSet._pack(g)


class TrackSet:
    """Deduplicated (control points, width) slots packed as the device table.

    ``slot(cp, width)`` returns the slot index of a pair, adding it on first
    sight; ``arrays()`` gives the rx_upload_tracks layout (include/rx.h)."""

    def __init__(self, factor=30):
        self.factor = factor
        self.geoms = []
        self._index = {}
        self._packed = None

    @classmethod
    def build(cls, control_points, widths, workers=None, factor=30):
        """The slots of (control_points[i], widths[i]) for every i, in first-sight
        order (as ``slot`` adds them), with the splines of many distinct slots
        computed in ``workers`` spawned processes (each runs TrackGeometry, so the
        geometry is bit-identical to the serial build).  For pools of thousands of
        distinct tracks -- ``gen_tracks(n, seed=None)``, SURVEY.md §8(d)'s stress
        variant -- where the serial spline (~1 ms per track) dominates."""
        ts = cls(factor)
        todo = []
        for cp, w in zip(control_points, widths):
            cp = DEFAULT_CONTROL_POINTS if cp is None else cp
            w = DEFAULT_WIDTH if w is None else w
            key = cls._key(cp, w)
            if key not in ts._index:
                ts._index[key] = len(todo)
                todo.append((cp, w))
        if workers is None:
            import os
            workers = min(16, len(os.sched_getaffinity(0)))
        if workers <= 1 or len(todo) < 256:
            ts.geoms = [TrackGeometry(cp, w, factor) for cp, w in todo]
            return ts
        import multiprocessing as mp
        per = (len(todo) + 4 * workers - 1) // (4 * workers)
        parts = [(todo[i:i + per], factor) for i in range(0, len(todo), per)]
        with mp.get_context("spawn").Pool(workers) as pool:
            packed = list(pool.imap(_geoms_worker, parts))
        W = np.concatenate([np.diff(p["wp_off"]) for p in packed])
        a = dict(wp_off=np.concatenate([[0], np.cumsum(W)]).astype(np.int32),
                 **{k: np.ascontiguousarray(np.concatenate([p[k] for p in packed]))
                    for k in ("wp", "nrm", "seg", "meta")})
        off = a["wp_off"]
        for k, (cp, w) in enumerate(todo):  # views into the packed table (TrackGeometry.from_arrays)
            s, e = off[k], off[k + 1]
            ts.geoms.append(TrackGeometry.from_arrays(cp, w, a["wp"][s:e], a["nrm"][s:e], a["seg"][2 * s:2 * e],
                                                      a["meta"][k, 4]))
        ts._packed = a
        return ts

    @staticmethod
    def _key(cp, width):
        a = np.asarray(cp)
        return (a.dtype.str, a.shape, a.tobytes(), float(width))

    def slot(self, control_points=None, track_width=None):
        cp = DEFAULT_CONTROL_POINTS if control_points is None else control_points
        w = DEFAULT_WIDTH if track_width is None else track_width
        key = self._key(cp, w)
        k = self._index.get(key)
        if k is None:
            k = len(self.geoms)
            self.geoms.append(TrackGeometry(cp, w, self.factor))
            self._index[key] = k
            self._packed = None
        return k

    def __len__(self):
        return len(self.geoms)

    @staticmethod
    def _pack(g):
        W = [len(t.waypoints) for t in g]
        wp_off = np.concatenate([[0], np.cumsum(W)]).astype(np.int32)
        wp = np.ascontiguousarray(np.concatenate([t.waypoints for t in g]), dtype=np.float64)
        nrm = np.ascontiguousarray(np.concatenate([t.normals for t in g]), dtype=np.float64)
        seg = np.ascontiguousarray(np.concatenate(
            [np.concatenate([t.segment_cache["starts"], t.segment_cache["v2"]], axis=1) for t in g]),
            dtype=np.float64)
        meta = np.zeros((len(g), 8), dtype=np.float64)
        for k, t in enumerate(g):
            sx, sy, sa = t.get_start_pos()
            meta[k] = (sx, sy, sa, float(t.track_width), float(t.max_track_distance),
                       t.normals[0, 0], t.normals[0, 1], 0.0)
        return dict(wp_off=wp_off, wp=wp, nrm=nrm, seg=seg, meta=meta)

    def arrays(self):
        if self._packed is None:
            self._packed = self._pack(self.geoms)
        return self._packed

    # ------------------------------------------------------------ on-disk table
    TABLE_VERSION = 1

    def save(self, path, track_of_env=None):
        """Write the table as an uncompressed .npz (loads with allow_pickle=False).

        Keys: version, factor, n_slots; per slot: widths [n], cp_off [n+1] int64,
        cp_is_int [n] bool, control_points [sum P, 2] f64; the device table
        wp_off / wp / nrm / seg / meta exactly as rx_upload_tracks takes it;
        optional track_of_env [N] int32 (the env -> slot assignment)."""
        a = self.arrays()
        cps = [np.asarray(g.control_points) for g in self.geoms]
        cp_off = np.concatenate([[0], np.cumsum([len(c) for c in cps])]).astype(np.int64)
        extra = {}
        if track_of_env is not None:
            toe = np.asarray(track_of_env, dtype=np.int32)
            if toe.size and (toe.min() < 0 or toe.max() >= len(self)):
                raise ValueError("track_of_env refers to a slot outside the table")
            extra["track_of_env"] = toe
        np.savez(path, version=np.int64(self.TABLE_VERSION), factor=np.int64(self.factor),
                 n_slots=np.int64(len(self)), widths=np.array([float(g.track_width) for g in self.geoms]),
                 cp_off=cp_off, cp_is_int=np.array([np.issubdtype(c.dtype, np.integer) for c in cps]),
                 control_points=np.concatenate(cps).astype(np.float64) if cps else np.zeros((0, 2)),
                 **a, **extra)

    @classmethod
    def load(cls, path, verify=False):
        """-> (TrackSet, track_of_env or None).  ``verify`` re-splines every slot
        from its control points and requires the stored geometry bit for bit."""
        with np.load(path, allow_pickle=False) as z:
            if int(z["version"]) != cls.TABLE_VERSION:
                raise ValueError(f"track table version {int(z['version'])} != {cls.TABLE_VERSION}")
            d = {k: z[k] for k in z.files}
        ts = cls(factor=int(d["factor"]))
        n = int(d["n_slots"])
        wp_off, cp_off = d["wp_off"], d["cp_off"]
        if wp_off.shape != (n + 1,) or cp_off.shape != (n + 1,) or d["meta"].shape != (n, 8):
            raise ValueError("inconsistent track table")
        for k in range(n):
            cp = d["control_points"][cp_off[k]:cp_off[k + 1]]
            if d["cp_is_int"][k]:
                cp = cp.astype(np.int64)
            w = float(d["widths"][k])
            a, b = wp_off[k], wp_off[k + 1]
            g = TrackGeometry.from_arrays(cp, w, d["wp"][a:b], d["nrm"][a:b], d["seg"][2 * a:2 * b],
                                          d["meta"][k, 4])
            if verify:
                ref = TrackGeometry(cp, w, ts.factor)
                for x, y in ((ref.waypoints, g.waypoints), (ref.normals, g.normals),
                             (ref.segment_cache["starts"], g.segment_cache["starts"]),
                             (ref.segment_cache["v2"], g.segment_cache["v2"])):
                    if x.shape != y.shape or x.tobytes() != y.tobytes():
                        raise ValueError(f"track table slot {k} does not match its control points")
            ts._index[cls._key(cp, w)] = len(ts.geoms)
            ts.geoms.append(g)
        ts._packed = {k: np.ascontiguousarray(d[k]) for k in ("wp_off", "wp", "nrm", "seg", "meta")}
        return ts, (d["track_of_env"] if "track_of_env" in d else None)
