"""CPU estimate (no GPU): how many of k_step2's box tests would a per-slot
box-distance table skip?  Replays the two-level traversal of cull_scan (as
tools/cull_estimate.py: supers outward from the wave's first car, 8 leaves of 8
segments) for waves of 64 cars and, before each super / leaf box test, applies
    skip X  iff  D(c0, X) >= max over lanes (best_l + r_l)
with D(c0, X) = the distance between box X and the region box of the wave's
first car's chunk c0 (union of its left / right leaf boxes; precomputed per
slot), r_l = the distance of lane l's origin from that region.  Exact: a ray
entering X does so at t >= dist(o, X) >= D(c0, X) - r_l.

    python tools/r06/dtable_estimate.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "self-play-racing_amd"))
import random  # noqa: E402

from rx.track import TrackGeometry, gen_tracks  # noqa: E402

random.seed(1)
np.random.seed(1)
pool = gen_tracks(num_tracks=8, seed=1)
widths = [np.random.randint(6, 10) for _ in range(8)]
G, SG = 8, 8
rng = np.random.default_rng(0)
rel = np.linspace(-np.pi / 3, np.pi / 3, 11)


def bbdist(a, b):
    dx = max(a[0] - b[2], b[0] - a[2], 0.0)
    dy = max(a[1] - b[3], b[1] - a[3], 0.0)
    return np.hypot(dx, dy)


def pdist(O, b):
    dx = np.maximum(np.maximum(b[0] - O[:, 0], O[:, 0] - b[2]), 0)
    dy = np.maximum(np.maximum(b[1] - O[:, 1], O[:, 1] - b[3]), 0)
    return np.hypot(dx, dy)


tot = {m: 0.0 for m in ("box", "scan", "box_skip", "scan_skip", "sup", "sup_skip", "leaf", "leaf_skip", "box3", "scan3",
                        "top3")}
TG = int(os.environ.get("TG", "2"))
nw = 0
for k in range(4):
    tg = TrackGeometry(pool[k], widths[k])
    wp = tg.waypoints
    W = len(wp)
    st = tg.segment_cache["starts"]
    v2 = tg.segment_cache["v2"]
    en = st + v2
    nch = (W + G - 1) // G
    nsup = (nch + SG - 1) // SG
    boxes = {}
    for side in range(2):
        for c in range(nch):
            j0, j1 = side * W + c * G, side * W + min(W, (c + 1) * G)
            P = np.vstack([st[j0:j1], en[j0:j1]])
            boxes[side, c] = (P[:, 0].min(), P[:, 1].min(), P[:, 0].max(), P[:, 1].max())
    sbox = {}
    for side in range(2):
        for s in range(nsup):
            bs = [boxes[side, c] for c in range(s * SG, min(nch, (s + 1) * SG))]
            sbox[side, s] = (min(b[0] for b in bs), min(b[1] for b in bs), max(b[2] for b in bs), max(b[3] for b in bs))
    ntop = (nsup + TG - 1) // TG
    tbox = {}
    for side in range(2):
        for t in range(ntop):
            bs = [sbox[side, u] for u in range(t * TG, min(nsup, (t + 1) * TG))]
            tbox[side, t] = (min(b[0] for b in bs), min(b[1] for b in bs), max(b[2] for b in bs), max(b[3] for b in bs))
    region = {c: (min(boxes[0, c][0], boxes[1, c][0]), min(boxes[0, c][1], boxes[1, c][1]),
                  max(boxes[0, c][2], boxes[1, c][2]), max(boxes[0, c][3], boxes[1, c][3])) for c in range(nch)}
    n = 2048
    wi = np.sort(rng.integers(0, W, n))
    tang = np.roll(wp, -1, 0) - wp
    tang /= np.linalg.norm(tang, axis=1, keepdims=True)
    nrm = np.column_stack([-tang[:, 1], tang[:, 0]])
    off = rng.uniform(-0.8, 0.8, n) * widths[k]
    O = wp[wi] + nrm[wi] * off[:, None]
    head = np.arctan2(tang[wi, 1], tang[wi, 0]) + rng.normal(0, 0.4, n)

    def tint(box, O, D):
        with np.errstate(divide="ignore", invalid="ignore"):
            t1 = (box[0] - O[:, 0]) / D[:, 0]
            t2 = (box[2] - O[:, 0]) / D[:, 0]
            t3 = (box[1] - O[:, 1]) / D[:, 1]
            t4 = (box[3] - O[:, 1]) / D[:, 1]
        lo = np.maximum(np.fmax(np.minimum(t1, t2), np.minimum(t3, t4)), 0)
        hi = np.fmin(np.maximum(t1, t2), np.maximum(t3, t4))
        return lo, hi

    def hits(O, D, j0, j1):
        best = np.full(len(O), np.inf)
        for j in range(j0, j1):
            s, v = st[j], v2[j]
            den = D[:, 0] * v[1] - D[:, 1] * v[0]
            w = s - O
            with np.errstate(divide="ignore", invalid="ignore"):
                t = (w[:, 0] * v[1] - w[:, 1] * v[0]) / den
                uu = (w[:, 0] * D[:, 1] - w[:, 1] * D[:, 0]) / den
            ok = (np.abs(den) > 1e-10) & (t >= 0) & (uu >= 0) & (uu <= 1)
            best = np.where(ok, np.minimum(best, t), best)
        return best

    for g0 in range(0, n, 64):
        Og = O[g0:g0 + 64]
        c0 = wi[g0] // G
        u0 = c0 // SG
        R = region[c0]
        r = pdist(Og, R)
        for ray in range(11):
            th = head[g0:g0 + 64] + rel[ray]
            D = np.column_stack([np.cos(th), np.sin(th)])
            for mode in (0, 1, 2):
                best = np.full(len(Og), np.inf)
                nb = ns = nsup_t = nleaf_t = ntop_t = 0
                topdec = {}
                for s in range(nsup):
                    o_ = (s + 1) >> 1
                    back = s & 1
                    u = (u0 - o_) % nsup if back else (u0 + o_) % nsup
                    l0 = u * SG
                    nl = min(nch, l0 + SG) - l0
                    for side in range(2):
                        Q = np.max(best + r)
                        if mode == 1 and bbdist(sbox[side, u], R) >= Q:
                            continue
                        if mode == 2:
                            key = (side, u // TG)
                            if key not in topdec:
                                nb += 1
                                ntop_t += 1
                                lo, hi = tint(tbox[key], Og, D)
                                topdec[key] = bool(np.any((lo <= hi) & (lo < best)))
                            if not topdec[key]:
                                continue
                        nb += 1
                        nsup_t += 1
                        lo, hi = tint(sbox[side, u], Og, D)
                        if not np.any((lo <= hi) & (lo < best)):
                            continue
                        for q in range(nl):
                            c = l0 + (nl - 1 - q if back else q)
                            Q = np.max(best + r)
                            if mode == 1 and bbdist(boxes[side, c], R) >= Q:
                                continue
                            nb += 1
                            nleaf_t += 1
                            lo, hi = tint(boxes[side, c], Og, D)
                            if np.any((lo <= hi) & (lo < best)):
                                ns += 1
                                j0, j1 = side * W + c * G, side * W + min(W, (c + 1) * G)
                                best = np.minimum(best, hits(Og, D, j0, j1))
                if mode == 0:
                    tot["box"] += nb
                    tot["scan"] += ns
                    tot["sup"] += nsup_t
                    tot["leaf"] += nleaf_t
                elif mode == 2:
                    tot["box3"] += nb
                    tot["scan3"] += ns
                    tot["top3"] += ntop_t
                else:
                    tot["box_skip"] += nb
                    tot["scan_skip"] += ns
                    tot["sup_skip"] += nsup_t
                    tot["leaf_skip"] += nleaf_t
            nw += 1
print({m: round(v / nw, 2) for m, v in tot.items()}, "per ray wave,", nw, "waves")
