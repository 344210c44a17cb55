"""Host track generation/geometry (rx.track) vs the reference's golden geometry.

gen_tracks (environment/track.py:4-56) and Track geometry (track.py:61-157)
must be bit-identical, including the global-RNG state left behind (the
reference draws track widths from it right after, train.py:79)."""
import random

import numpy as np

from rx.track import DEFAULT_CONTROL_POINTS, TrackGeometry, TrackSet, gen_tracks


def _pool(n, seed=1):
    random.seed(seed)
    np.random.seed(seed)
    pool = gen_tracks(num_tracks=n, seed=seed)
    widths = [np.random.randint(6, 10) for _ in range(n)]
    return pool, widths


def test_gen_tracks_seeded_matches_reference(golden):
    g = golden.geo
    for n, key in ((16, None), (64, "pool1x64")):
        pool, widths = _pool(n)
        if key is None:
            for k in range(16):
                assert np.array_equal(pool[k], golden.tracks[k]["cp"])
            assert widths == list(g["pool1_widths"])
        else:
            off = g[key + "_cp_off"]
            for k in range(n):
                assert np.array_equal(pool[k], g[key + "_cp"][off[k]:off[k + 1]]), k
            assert widths == list(g[key + "_widths"])


def test_gen_tracks_unseeded_matches_reference(golden):
    g = golden.geo
    np.random.seed(7)
    free = gen_tracks(num_tracks=8, seed=None)
    off = g["free7x8_cp_off"]
    for k in range(8):
        assert np.array_equal(free[k], g["free7x8_cp"][off[k]:off[k + 1]])


def test_geometry_bit_exact(golden):
    for k, t in enumerate(golden.tracks):
        cp = DEFAULT_CONTROL_POINTS if t["label"] == "default" else t["cp"]
        geo = TrackGeometry(cp, t["width"] if t["label"] != "default" else None)
        assert np.array_equal(geo.waypoints, t["wp"]), k
        assert np.array_equal(geo.normals, t["nrm"]), k
        assert np.array_equal(geo.segment_cache["starts"], t["starts"]), k
        assert np.array_equal(geo.segment_cache["v2"], t["v2"]), k
        assert geo.max_track_distance == t["maxd"], k
        assert np.array_equal(np.array([float(v) for v in geo.get_start_pos()]), t["start"]), k


def test_trackset_dedups_seed1_pool_to_7_slots():
    pool, widths = _pool(4096)
    ts = TrackSet()
    slots = [ts.slot(c, w) for c, w in zip(pool, widths)]
    assert len(ts) == 7
    a = ts.arrays()
    assert a["wp_off"][-1] == sum(len(t.waypoints) for t in ts.geoms)
    assert a["seg"].shape == (2 * a["wp_off"][-1], 4)
    assert max(slots) == 6


def test_eval_pool_matches_reference_protocol(golden):
    """evaluate.py:178-182 pool (the golden set drew it after np.random.seed(12345))."""
    from rx.evaluate import eval_pool
    cps, ws, ids = eval_pool(40, 5, 42, global_seed=12345)
    assert len(cps) == 200 and ids[7] == (1, 2)
    labels = [t["label"] for t in golden.tracks]
    for t in range(4):
        k = labels.index(f"eval42[{t}] w={int(golden.geo['eval42_widths'][t])}")
        assert np.array_equal(cps[5 * t], golden.tracks[k]["cp"])
    assert ws[:5] == list(golden.geo["eval42_widths"][:5])  # widths indexed by RUN (evaluate.py:30)


def test_track_table_file_roundtrip(golden, tmp_path):
    """On-disk table (TrackSet.save/load): the loaded table
    is the saved one byte for byte, its slots are the golden geometry, and the
    stored env assignment comes back."""
    ts = TrackSet()
    want = {}
    for t in golden.tracks:
        cp = DEFAULT_CONTROL_POINTS if t["label"] == "default" else t["cp"]
        w = None if t["label"] == "default" else t["width"]
        want[ts.slot(cp, w)] = t
    pool, widths = _pool(256)
    toe = np.array([ts.slot(c, w) for c, w in zip(pool, widths)], dtype=np.int32)
    p = tmp_path / "tracks.npz"
    ts.save(p, toe)
    ld, toe2 = TrackSet.load(p, verify=True)
    assert np.array_equal(toe, toe2) and len(ld) == len(ts)
    for k in ts.arrays():
        assert ts.arrays()[k].tobytes() == ld.arrays()[k].tobytes(), k
    for k, t in want.items():
        g = ld.geoms[k]
        assert np.array_equal(g.waypoints, t["wp"]) and np.array_equal(g.normals, t["nrm"])
        assert np.array_equal(g.segment_cache["starts"], t["starts"]) and np.array_equal(g.segment_cache["v2"], t["v2"])
        assert g.max_track_distance == t["maxd"]
        assert np.array_equal(np.array([float(v) for v in g.get_start_pos()]), t["start"])
        ref = ts.geoms[k]
        assert np.array_equal(g.segment_cache["ends"], ref.segment_cache["ends"])
        assert g.track_bounds == ref.track_bounds
    # slot lookup by (control points, width) still dedups against loaded slots
    assert ld.slot(pool[0], widths[0]) == toe[0] and len(ld) == len(ts)
    assert ld.slot(DEFAULT_CONTROL_POINTS, None) == ts.slot(DEFAULT_CONTROL_POINTS, None)


def test_track_table_rejects_tampering(tmp_path):
    import pytest
    ts = TrackSet()
    ts.slot(DEFAULT_CONTROL_POINTS, 7)
    p = tmp_path / "t.npz"
    ts.save(p)
    d = dict(np.load(p))
    d["wp"] = d["wp"].copy()
    d["wp"][3, 0] += 1e-9
    np.savez(tmp_path / "bad.npz", **d)
    with pytest.raises(ValueError):
        TrackSet.load(tmp_path / "bad.npz", verify=True)
    assert TrackSet.load(p)[1] is None
