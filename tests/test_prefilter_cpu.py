"""CPU check of the raycast's float32 segment pre-filter (rx_kernels.hip
seg_may_hit): it must never reject a segment that the exact f64 test
(seg_test, the reference's Track.raycast arithmetic, environment/track.py:
173-199) reports as hit.  Both are emulated here operation by operation in
numpy (float32 ops round like the kernel's; the f64 test mirrors seg_test
with -ffp-contract=off), over random and adversarial rays: segments crossed
near an endpoint, endpoints on the ray line, grazing and far segments, at
track-sized and larger coordinates.  The threshold is the kernel's:
e2 = 2^-17 (|ox| + |oy| + |cx| + |cy| + 2 rad + L + 1) with (cx, cy), rad the
slot's bounding circle and L its longest segment (here: those of the batch)."""
import numpy as np

F = np.float32


def exact_hit(ox, oy, sx, sy, v2x, v2y, v3x, v3y):
    """seg_test's hit predicate (division-free form of track.py:184-196); the
    sign flips are the XOR of dotp's sign bit (np.signbit: -0.0 included)."""
    v1x, v1y = ox - sx, oy - sy
    dotp = v2x * v3x + v2y * v3y
    cross = v2x * v1y - v2y * v1x
    dot = v1x * v3x + v1y * v3y
    D = np.abs(dotp)
    neg = np.signbit(dotp)
    C = np.where(neg, -cross, cross)
    N = np.where(neg, -dot, dot)
    return (D > 1e-10) & (C >= 0.0) & (N >= 0.0) & ((N - D) <= D * 2.0 ** -53)


def fma32(a, b, c):
    """float32 fma: the product of two float32 is exact in float64, the sum is
    taken in extended precision and rounded once to float32."""
    p = np.asarray(a, np.float64) * np.asarray(b, np.float64)
    return (p.astype(np.longdouble) + np.asarray(c, np.longdouble)).astype(F)


def prefilter(ox, oy, sx, sy, v2x, v2y, v3x, v3y, e2):
    """seg_may_hit in float32: a = c0 - sx v3x - sy v3y (c0 = o . v3 per lane),
    p = sz v3x + sw v3y, keep iff |2a - p| - |p| <= e2."""
    of = (ox.astype(F), oy.astype(F))
    sf = (sx.astype(F), sy.astype(F), v2x.astype(F), v2y.astype(F))
    vf = (v3x.astype(F), v3y.astype(F))
    c0 = fma32(of[1], vf[1], of[0] * vf[0])  # __builtin_fmaf(oyf, csf, oxf * -snf)
    aa = fma32(-sf[1], vf[1], fma32(-sf[0], vf[0], c0))
    dp = fma32(sf[3], vf[1], sf[2] * vf[0])
    q = fma32(F(2.0), aa, -dp)  # fma(2, aa, -dp)
    return ~((np.abs(q) - np.abs(dp)) > e2)


def _rays(rng, n, scale):
    ox = rng.uniform(-scale, scale, n)
    oy = rng.uniform(-scale, scale, n)
    th = rng.uniform(-np.pi, np.pi, n)
    return ox, oy, np.cos(th), np.sin(th)  # direction d; v3 = (-sin, cos)


def _e2(ox, oy, sx, sy, v2x, v2y, cx, cy):
    """The kernel's per-lane threshold for a slot with these segments."""
    ex, ey = sx + v2x, sy + v2y
    rad = np.max(np.maximum(np.hypot(sx - cx, sy - cy), np.hypot(ex - cx, ey - cy)))
    L = np.max(np.hypot(v2x, v2y))
    e2 = ((np.abs(ox) + np.abs(oy) + abs(cx) + abs(cy) + 2.0 * rad + L + 1.0) * 2.0 ** -17).astype(F)
    return e2


def test_prefilter_never_rejects_an_exact_hit():
    rng = np.random.default_rng(7)
    total_hits = rejected = 0
    for scale in (150.0, 1000.0):
        n = 400_000
        ox, oy, dx, dy = _rays(rng, n, scale)
        v3x, v3y = -dy, dx
        kind = rng.integers(0, 4, n)
        # a point P on the ray at distance t, then a segment through / near P
        t = rng.uniform(0.0, 60.0, n)
        px, py = ox + t * dx, oy + t * dy
        ang = rng.uniform(-np.pi, np.pi, n)
        ln = rng.uniform(0.2, 6.0, n)
        ux, uy = np.cos(ang), np.sin(ang)
        frac = rng.uniform(0.0, 1.0, n)
        frac = np.where(kind == 1, rng.choice([0.0, 1.0], n) + rng.normal(0, 1e-9, n), frac)  # near an endpoint
        off = np.where(kind == 2, rng.normal(0, 1e-7, n), 0.0)  # the line passes a hair beside
        off = np.where(kind == 3, rng.uniform(-3.0, 3.0, n), off)  # arbitrary nearby segments
        sx = px - frac * ln * ux + off * v3x
        sy = py - frac * ln * uy + off * v3y
        v2x, v2y = ln * ux, ln * uy
        cx, cy = float(np.mean(sx)), float(np.mean(sy))
        e2 = _e2(ox, oy, sx, sy, v2x, v2y, cx, cy)
        hit = exact_hit(ox, oy, sx, sy, v2x, v2y, v3x, v3y)
        keep = prefilter(ox, oy, sx, sy, v2x, v2y, v3x, v3y, e2)
        total_hits += int(hit.sum())
        rejected += int((hit & ~keep).sum())
        # the filter is useful: most non-crossing arbitrary segments are rejected
        far = (kind == 3) & ~hit
        assert (~keep[far]).mean() > 0.5
    assert total_hits > 200_000
    assert rejected == 0


def test_prefilter_endpoint_exactly_on_the_ray():
    """Segments whose start or end point lies exactly on the ray (s = 0 or 1
    exactly representable): the exact test may accept them; the filter must."""
    rng = np.random.default_rng(11)
    n = 200_000
    ox = np.round(rng.uniform(-100, 100, n))
    oy = np.round(rng.uniform(-100, 100, n))
    dx = rng.choice([1.0, -1.0, 0.0], n)
    dy = np.where(dx == 0.0, rng.choice([1.0, -1.0], n), 0.0)  # axis-aligned rays: exact arithmetic
    t = np.round(rng.uniform(0, 50, n))
    sx, sy = ox + t * dx, oy + t * dy  # the start point on the ray
    v2x = np.round(rng.uniform(-5, 5, n))
    v2y = np.round(rng.uniform(-5, 5, n))
    v3x, v3y = -dy, dx
    e2 = _e2(ox, oy, sx, sy, v2x, v2y, 0.0, 0.0)
    hit = exact_hit(ox, oy, sx, sy, v2x, v2y, v3x, v3y)
    keep = prefilter(ox, oy, sx, sy, v2x, v2y, v3x, v3y, e2)
    assert hit.sum() > 10_000
    assert not (hit & ~keep).any()


def test_s_le_1_is_n_le_d():
    """rx_kernels.hip seg_test's division-free s <= 1: with D = |dotp| > 1e-10 and
    N = sgn(dotp) dot (doubles), round(N / D) <= 1 exactly when N <= D -- the
    reference computes s = dot / dotp (environment/track.py:191-196) and tests
    s <= 1.  Checked on 4 M pairs: N within +-4 ulps of D over 16 decades of D,
    random N around D, and D a power of two (the tightest ulp(D) / D)."""
    rng = np.random.default_rng(3)
    n = 1_000_000
    D = np.exp(rng.uniform(np.log(1e-10), np.log(1e6), n))
    k = rng.integers(-4, 5, n)
    N = D.copy()
    for step in range(1, 5):
        N = np.where(k >= step, np.nextafter(N, np.inf), N)
        N = np.where(k <= -step, np.nextafter(N, -np.inf), N)
    P2 = 2.0 ** rng.integers(-33, 20, n).astype(np.float64)
    for NN, DD in ((N, D), (D * rng.uniform(0.5, 1.5, n), D), (np.nextafter(P2, np.inf), P2),
                   (np.nextafter(P2, -np.inf), P2)):
        assert np.array_equal(NN / DD <= 1.0, NN <= DD)
        assert np.array_equal(-NN / DD <= 1.0, -NN <= DD)  # the sign-flipped operand as well
