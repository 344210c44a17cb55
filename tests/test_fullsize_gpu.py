"""BASELINE.json configurations at their real sizes, under the oracle.

The headline number is measured at 65,536 single-agent envs (configs[2]):
11,264 direction-sorted ray waves placed XCD-aware, the spatial env re-sort
every 16 steps, the split step (k_kin1 + k_step2) and 64 episode-statistic
shards.  Envs are independent, so a fixed random subset of them can be
stepped by the device-libm oracle (oracle/rx_oracle.c: same sin/cos and x*x
as the kernels) beside the full launch geometry and compared BIT FOR BIT
after every step: observations, f32 rewards, done masks, and periodically
the whole f64 state.  Same for the two-car env at configs[3]'s 8,192 envs
(k_kin2 + k_step2<2>, start-slot draws on reset), for one env (configs[0]'s
N = 1 on the HIP path), and for the episode-statistics reduction over all
65,536 envs (every shard summed).

Inputs follow the bench: the reference's seed-1 pool (train.py:67-80),
next-step autoreset, uniform random actions (steer U(-1, 1), throttle
U(0, 1); two-car actions U(-1, 1)^2 per car).
"""
import random

import numpy as np
import pytest
import torch

from oracle.orc import TrackTable, multi_state, sensor_angles, single_state

pytestmark = pytest.mark.gpu

REL1 = sensor_angles(11, np.pi / 3)
REL2 = sensor_angles(11, np.pi / 2)


def _seed1_pool(n):
    from rx.track import gen_tracks
    random.seed(1)
    np.random.seed(1)
    pool = gen_tracks(num_tracks=n, seed=1)
    widths = [np.random.randint(6, 10) for _ in range(n)]
    return pool, widths


def _oracle_table(v):
    """The env's deduplicated device track table as an oracle TrackTable."""
    t = TrackTable.__new__(TrackTable)
    a = v.tracks.arrays()
    t.wp_off, t.wp, t.nrm, t.seg, t.meta = a["wp_off"], a["wp"], a["nrm"], a["seg"], a["meta"]
    t.n = len(a["meta"])
    return t


def _actions(rng, N, A):
    if A == 1:
        return np.stack([rng.uniform(-1, 1, N), rng.uniform(0, 1, N)], 1).astype(np.float32)
    return rng.uniform(-1, 1, (N, 2, 2)).astype(np.float32)


def _single_run(v, idx, oracle_dev, steps, seed, state_every=25):
    """Step every env of v on the device and the envs idx on the oracle; compare."""
    N = v.num_envs
    tab = _oracle_table(v)
    n = len(idx)
    st = single_state(n)
    st["track"][:] = v.track_of_env[idx]
    obs = v.reset_device().cpu().numpy()
    assert np.array_equal(obs[idx], oracle_dev.single_reset(tab, st, REL1))
    rng = np.random.default_rng(seed)
    pending = np.zeros(n, bool)
    ended = 0
    for t in range(steps):
        a = _actions(rng, N, 1)
        obs, rew, done = v.step_device(torch.from_numpy(a).cuda())
        obs, rew, done = obs.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy().astype(bool)
        o_obs, o_rew, o_term, o_trunc, _ = oracle_dev.single_step(tab, st, a[idx], REL1)
        if pending.any():  # gymnasium next-step autoreset
            r_obs = oracle_dev.single_reset(tab, st, REL1, mask=pending)
            o_obs[pending] = r_obs[pending]
            o_rew[pending] = 0.0
            o_term[pending] = False
            o_trunc[pending] = False
        assert np.array_equal(obs[idx], o_obs), t
        assert np.array_equal(rew[idx], o_rew.astype(np.float32)), t
        assert np.array_equal(done[idx], o_term | o_trunc), t
        pending = o_term | o_trunc
        ended += int(pending.sum())
        if (t + 1) % state_every == 0 or t + 1 == steps:
            g = v.get_state()
            for k in ("x", "y", "angle", "vx", "vy", "progress", "last_progress", "last_steering", "steps", "flags"):
                assert np.array_equal(g[k][idx], st[k]), (t, k)
    return ended


def test_65536_envs_subset_bit_exact_vs_oracle(oracle_dev):
    """configs[2] at its real launch geometry: 4,096 random envs of 65,536 ==
    the oracle bit for bit at every one of 200 steps (resets, sorts, crashes)."""
    from rx.vector_env import RacingVectorEnv
    N = 65536
    pool, widths = _seed1_pool(N)
    v = RacingVectorEnv(pool, widths, device="cuda", autoreset="next_step")
    idx = np.sort(np.random.default_rng(3).choice(N, 4096, replace=False))
    ended = _single_run(v, idx, oracle_dev, 200, seed=11)
    assert ended > 500  # the subset saw many episode ends and next-step resets
    v.close()


def test_4096_envs_configs1_geometry_subset_bit_exact_vs_oracle(oracle_dev):
    """configs[1]'s env count on its own default launch geometry (the split step
    with 4 lanes per ray task -- 16 tasks a ray wave -- and the REWARD half at 2
    lanes per env, as rx_assign picks for 4,096 envs): 1,024 random envs == the
    oracle bit for bit at every one of 200 steps (environment/racing_env.py:104-167)."""
    from rx.vector_env import RacingVectorEnv
    N = 4096
    pool, widths = _seed1_pool(N)
    v = RacingVectorEnv(pool, widths, device="cuda", autoreset="next_step")
    sch = v.schedule()
    assert (sch["split"], sch["wide"], sch["dyn_lpe"], sch["ray_lpr"], sch["reward_lpe"]) == (1, 0, 1, 4, 2), sch
    idx = np.sort(np.random.default_rng(17).choice(N, 1024, replace=False))
    ended = _single_run(v, idx, oracle_dev, 200, seed=19)
    assert ended > 100
    v.close()


def test_one_env_hip_step_vs_oracle(oracle_dev):
    """configs[0]'s N = 1 on the HIP path (wide kernels): 1,500 steps, every step exact."""
    from rx.vector_env import RacingVectorEnv
    pool, widths = _seed1_pool(16)
    v = RacingVectorEnv(pool[:1], widths[:1], device="cuda", autoreset="next_step")
    ended = _single_run(v, np.arange(1), oracle_dev, 1500, seed=5, state_every=100)
    assert ended >= 3
    v.close()


def test_episode_statistics_all_shards_at_65536():
    """The 64 sharded episode-statistic rows summed by the reader == returns and
    lengths accumulated from the per-step rewards / dones of all 65,536 envs."""
    from rx.vector_env import RacingVectorEnv
    N = 65536
    pool, widths = _seed1_pool(N)
    v = RacingVectorEnv(pool, widths, device="cuda", autoreset="next_step")
    v.reset_device()
    g = torch.Generator(device="cuda").manual_seed(4)
    scale = torch.tensor([2.0, 1.0], device="cuda")
    shift = torch.tensor([-1.0, 0.0], device="cuda")
    ret = torch.zeros(N, dtype=torch.float64, device="cuda")
    lens = torch.zeros(N, dtype=torch.int64, device="cuda")
    sums = [0.0, 0, 0]
    for t in range(150):
        pend = (v.state["env_flags"] & 1).bool()
        _, _, done = v.step_device(torch.rand((N, 2), device="cuda", generator=g) * scale + shift, full_info=True)
        ret = torch.where(pend, torch.zeros_like(ret), ret + v.buf["reward64"])
        lens = torch.where(pend, torch.zeros_like(lens), lens + 1)
        ended = done.bool() & ~pend
        sums[0] += float(ret[ended].sum())
        sums[1] += int(lens[ended].sum())
        sums[2] += int(ended.sum())
    s = v.episode_stats()
    assert s[2] == sums[2] and s[2] > 20000
    assert s[1] == sums[1]
    assert abs(s[0] - sums[0]) <= 1e-9 * max(1.0, abs(sums[0]))
    v.close()


@pytest.mark.parametrize("N,n_sub,sched", [(8192, 2048, None), (4096, 1024, None), (8192, 1024, {"ray_lpr": 2, "reward_lpe": 1})])
def test_two_car_subset_bit_exact_vs_oracle(oracle_dev, N, n_sub, sched):
    """configs[3]'s env at 8,192 two-car envs (default: a lane per ray task and
    the REWARD half at a lane per car) and at 4,096 (4 lanes per ray task), plus
    8,192 on round 3's schedule (2 lanes per ray, one REWARD lane per env), all
    on the split step k_kin2 + k_step2<2>: a random subset == the oracle bit
    for bit over 200 steps.  On a reset the start-slot order is drawn on the device (the
    reference draws it from the global np.random, multi_racing_env.py:122-138):
    the oracle resets with the order the device chose, which must be one of the
    two slot assignments."""
    from rx.vector_env import RacingVectorEnv
    pool, widths = _seed1_pool(N)
    v = RacingVectorEnv(pool, widths, n_agents=2, device="cuda", autoreset="next_step", seed=9, sched=sched)
    sch = v.schedule()
    want = dict(ray_lpr=4 if 2 * N <= 8192 else 1, reward_lpe=2) if sched is None else sched
    assert sch["split"] == 1 and sch["wide"] == 0 and all(sch[k] == want[k] for k in want), sch
    tab = _oracle_table(v)
    idx = np.sort(np.random.default_rng(5).choice(N, n_sub, replace=False))
    n = len(idx)
    st = multi_state(n)
    st["track"][:] = v.track_of_env[idx]

    def oracle_reset(mask):
        """Reset the masked oracle envs with the device's slot order."""
        g = v.get_state()
        dx = g["x"].reshape(N, 2)[idx]
        keep = {k: val.copy() for k, val in st.items()}
        outs = []
        for first in (0, 1):
            for k in st:
                st[k][...] = keep[k]
            o = oracle_dev.multi_reset(tab, st, first, REL2, mask=mask)
            outs.append((o, {k: val.copy() for k, val in st.items()}))
        pick = np.where(np.all(outs[0][1]["x"] == dx, axis=1), 0, 1)
        ok = np.all(outs[int(1)][1]["x"] == dx, axis=1) | (pick == 0)
        assert ok[mask].all(), "device start slots are neither oracle order"
        obs = np.where(pick[:, None, None] == 0, outs[0][0], outs[1][0])
        for k in st:
            val0, val1 = outs[0][1][k], outs[1][1][k]
            sel = pick.reshape((-1,) + (1,) * (val0.ndim - 1)) == 0
            st[k][...] = np.where(sel, val0, val1)
        return obs

    obs = v.reset_device().cpu().numpy()
    assert np.array_equal(obs[idx], oracle_reset(np.ones(n, bool)))
    rng = np.random.default_rng(13)
    pending = np.zeros(n, bool)
    ended = 0
    for t in range(200):
        a = _actions(rng, N, 2)
        obs, rew, done = v.step_device(torch.from_numpy(a).cuda())
        obs, rew, done = obs.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy().astype(bool)
        o_obs, o_rew, _, o_done_all, _, _, _ = oracle_dev.multi_step(tab, st, a[idx], REL2)
        if pending.any():
            r_obs = oracle_reset(pending)
            o_obs[pending] = r_obs[pending]
            o_rew[pending] = 0.0
            o_done_all[pending] = False
        assert np.array_equal(obs[idx], o_obs), t
        assert np.array_equal(rew[idx], o_rew.astype(np.float32)), t
        assert np.array_equal(done[idx], o_done_all), t
        pending = o_done_all.copy()
        ended += int(pending.sum())
        if (t + 1) % 25 == 0:
            g = v.get_state()
            for k in ("x", "y", "angle", "vx", "vy", "progress", "flags", "finished_step"):
                assert np.array_equal(g[k].reshape(N, 2)[idx], st[k]), (t, k)
    assert ended > 200 * n_sub // 2048
    v.close()


@pytest.mark.parametrize("n_agents,N", [(1, 65536), (2, 8192)])
def test_spatial_sort_orders_envs_by_track_bin(n_agents, N):
    """The hand-written counting sort (rx_sort.hip) at the bench's sizes: right
    after a re-sort step the wave order is a permutation of the envs, every slot
    group keeps exactly its slot's envs, and inside a group the envs ascend by
    sort bin = (closest waypoint of car 0 = trunc(progress * W + 0.5)) >> shift."""
    from rx.vector_env import RacingVectorEnv
    pool, widths = _seed1_pool(N)
    v = RacingVectorEnv(pool, widths, n_agents=n_agents, device="cuda", autoreset="next_step", sort_interval=16)
    v.reset_device()
    rng = np.random.default_rng(21)
    for t in range(32):  # dynamics launches 0 (the reset), 16, 32 re-sort: the order follows step 32's keys
        v.step_device(torch.from_numpy(_actions(rng, N, n_agents)).cuda())
    perm, bins, shift = v.env_order()
    assert bins > 0 and shift == 0
    assert np.array_equal(np.sort(perm), np.arange(N))
    slots = v.track_of_env
    off = v.tracks.arrays()["wp_off"]
    W = (off[1:] - off[:-1]).astype(np.int64)
    prog = v.get_state()["progress"].reshape(N, n_agents)[:, 0]
    w = np.clip(np.trunc(prog * W[slots] + 0.5).astype(np.int64), 0, W[slots]) >> shift
    base = np.concatenate([[0], np.cumsum((W >> shift) + 1)[:-1]])
    key = base[slots] + w
    k_perm = slots[perm]
    assert np.all(np.diff(k_perm) >= 0), "slot groups moved"
    assert np.array_equal(np.bincount(k_perm, minlength=len(W)), np.bincount(slots, minlength=len(W)))
    assert np.all(np.diff(key[perm]) >= 0), "envs not ascending by sort bin"
    assert len(np.unique(key)) > 30  # the cars have started to spread over the tracks
    v.close()


def _stress_pool(n, seed):
    """SURVEY.md §8(d) stress variant: np.random.seed(s); gen_tracks(n, seed=None) --
    every env its own track (no per-track reseed, environment/track.py:47-56)."""
    from rx.track import gen_tracks
    np.random.seed(seed)
    pool = gen_tracks(num_tracks=n, seed=None)
    widths = [np.random.randint(6, 10) for _ in range(n)]
    return pool, widths


def test_stress_distinct_tracks_subset_bit_exact_vs_oracle(oracle_dev):
    """The stress pool at 16,384 envs = 16,384 distinct track slots (P in [10, 14]):
    2,048 random envs == the oracle bit for bit at every one of 200 steps, on the
    schedule rx_assign picks for a pool of distinct tracks."""
    from rx.track import TrackSet
    from rx.vector_env import RacingVectorEnv
    N = 16384
    pool, widths = _stress_pool(N, 5)
    v = RacingVectorEnv(pool, widths, device="cuda", autoreset="next_step", track_set=TrackSet.build(pool, widths))
    assert len(v.tracks) == N
    idx = np.sort(np.random.default_rng(23).choice(N, 2048, replace=False))
    ended = _single_run(v, idx, oracle_dev, 200, seed=29)
    assert ended > 200
    v.close()
