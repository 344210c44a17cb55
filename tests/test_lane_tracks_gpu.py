"""Lane-varying track slots (rx_config.lane_tracks, ABI v23).

A pool of distinct tracks (SURVEY.md §8(d)'s stress variant: gen_tracks(N,
seed=None), environment/track.py:47-56) leaves the slot-grouped waves one env
each; with lane_tracks the single-agent kernels take 64 consecutive envs of any
slots and every lane reads its own slot's tables.  The culling is exact either
way, so the lane-varying kernels must give the slot-uniform kernels' outputs BIT
FOR BIT: observations, f32 rewards, done masks, episode statistics and the f64
state, on the split step, the one-kernel step (same-step autoreset), resets and
the raycast launched on its own.  The stress pool's oracle parity is
tests/test_fullsize_gpu.py::test_stress_distinct_tracks_subset_bit_exact_vs_oracle.
"""
import random

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _pool(n, kind, seed=1):
    from rx.track import gen_tracks
    random.seed(seed)
    np.random.seed(seed)
    if kind == "seed1":  # train.py:67-80: 7 slots
        pool = gen_tracks(num_tracks=n, seed=1)
    elif kind == "distinct":
        pool = gen_tracks(num_tracks=n, seed=None)
    else:  # mixed: every 4th env its own track, the rest on the seed-1 pool's slots
        a = gen_tracks(num_tracks=n, seed=1)
        b = gen_tracks(num_tracks=n // 4 + 1, seed=None)
        pool = [b[i // 4] if i % 4 == 0 else a[i] for i in range(n)]
    widths = [np.random.randint(6, 10) for _ in range(n)]
    return pool, widths


def _pair(n, kind, autoreset="next_step"):
    from rx.track import TrackSet
    from rx.vector_env import RacingVectorEnv
    pool, widths = _pool(n, kind)
    ts = TrackSet.build(pool, widths)
    mk = lambda lt: RacingVectorEnv(pool, widths, device="cuda", autoreset=autoreset, track_set=ts,  # noqa: E731
                                    sched=dict(lane_tracks=lt))
    return mk(-1), mk(1)


def _run(va, vb, steps, seed, state_every=50):
    N = va.num_envs
    assert va.schedule()["lane_tracks"] == 0 and vb.schedule()["lane_tracks"] == 1
    assert torch.equal(va.reset_device(), vb.reset_device())
    g = torch.Generator(device="cuda").manual_seed(seed)
    for t in range(steps):
        a = torch.rand((N, 2), device="cuda", generator=g) * 2 - 1
        a[:, 1].abs_()
        oa, ra, da = va.step_device(a)
        ob, rb, db = vb.step_device(a)
        assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(da, db), t
        if (t + 1) % state_every == 0:
            sa, sb = va.get_state(), vb.get_state()
            for k in ("x", "y", "angle", "vx", "vy", "progress", "last_progress", "last_steering", "steps", "flags",
                      "env_flags", "ep_return", "ep_length"):
                assert np.array_equal(sa[k], sb[k]), (t, k)
    ea, eb = va.episode_stats(), vb.episode_stats()
    assert ea[2] == eb[2] and ea[1] == eb[1] and abs(ea[0] - eb[0]) <= 1e-9 * max(1.0, abs(ea[0])), (ea, eb)
    # the raycast on its own (k_rays<1, true>, rx_step_phases) and an explicit reset of some envs
    z = torch.zeros((N, 2), device="cuda")
    assert torch.equal(va.step_device(z, phases=2)[0], vb.step_device(z, phases=2)[0])
    m = (torch.arange(N, device="cuda") % 3 == 0)
    assert torch.equal(va.reset_device(mask=m), vb.reset_device(mask=m))
    return ea[2]


@pytest.mark.parametrize("N,kind", [(8256, "seed1"), (65536, "seed1"), (4160, "distinct"), (6000, "mixed")])
def test_lane_tracks_equal_slot_uniform_split_step(N, kind):
    """Split step (k_kin1 + k_step2<1, 1, 1, true>) against the slot-uniform
    schedule over 200 steps: on the seed-1 pool (7 slots: lanes of a wave mostly
    share a slot), a distinct-track pool and a mixed pool; ragged sizes leave a
    partial last block."""
    va, vb = _pair(N, kind)
    ended = _run(va, vb, 200, seed=N)
    assert ended > 0
    va.close()
    vb.close()


def test_lane_tracks_equal_slot_uniform_same_step_autoreset():
    """The one-kernel path (k_dyn1<1, FULL, true> + k_rays<1, true>): same-step
    autoreset needs done before the observation, so the split step never runs."""
    va, vb = _pair(5000, "distinct", autoreset="same_step")
    assert _run(va, vb, 150, seed=7) > 0
    va.close()
    vb.close()


def test_lane_tracks_auto_rule():
    """Auto (0): on iff grouping by slot needs more than 2 x ceil(N / 64) dynamics
    waves -- the stress pool (one slot per env) yes, the seed-1 pool no; the
    lane-varying schedule runs one lane per env and per ray, no task sort, no re-sort."""
    from rx.track import TrackSet
    from rx.vector_env import RacingVectorEnv
    for kind, n, want in (("distinct", 4096, 1), ("seed1", 65536, 0), ("seed1", 4096, 0)):
        pool, widths = _pool(n, kind)
        v = RacingVectorEnv(pool, widths, device="cuda", track_set=TrackSet.build(pool, widths))
        s = v.schedule()
        assert s["lane_tracks"] == want, (kind, n, s)
        if want:
            assert s["ray_lpr"] == 1 and s["reward_lpe"] == 1 and s["dyn_waves"] == (n + 63) // 64
            assert s["ray_waves"] == (n + 63) // 64 * 11 and v.env_order()[1] == 0  # no spatial re-sort bins
        v.close()
