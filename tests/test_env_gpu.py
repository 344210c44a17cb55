"""HIP env kernels vs the reference (golden vectors) and vs the oracle.

Bars (BASELINE.json north_star): integer done/collision masks bit-exact;
float observations/rewards within 1e-5 of the reference.  Against the oracle's
device-libm build (same sin/cos and x*x as the kernels) every output must be
bit-exact -- that isolates the only intended numerical difference from the
reference: glibc's sin/cos/pow(x,2) vs the kernels' correctly rounded ones.
"""
import numpy as np
import pytest
import torch

from oracle.orc import F_CP25, F_CP50, F_CP75, F_CRASHED, F_FINISHED, sensor_angles, single_state
from tests.golden_util import multi_state_from, single_state_from

pytestmark = pytest.mark.gpu

OBS_TOL = 1e-5      # north_star: float observations / rewards
STATE_TOL = 1e-9    # f64 state after one step: ulp-level libm differences only
REL1 = sensor_angles(11, np.pi / 3)
REL2 = sensor_angles(11, np.pi / 2)


@pytest.fixture(scope="module")
def rx():
    if not torch.cuda.is_available():
        pytest.fail("gpu test without a HIP device")
    import rx.vector_env as ve
    return ve


# launch schedule (rx_config ABI v17) the dyn_path fixture imposes on every _venv
_PATH_SCHED = {}


@pytest.fixture(params=["default", "split", "wide"])
def dyn_path(request):
    """Run a test on the default kernel choice for its env count, on the split
    step (k_kin1 + k_step2: REWARD half beside the raycast), which librx uses
    at one lane per env -- forced here via dyn_lpe = 1 -- and on the small-N
    wide kernels (one env per dynamics wave, one ray per raycast wave, brute
    force over the lanes; librx uses them up to 2,048 envs) forced for any N.
    "default" turns the wide kernels off, so small tests run the k_dyn1<4> +
    culled k_rays path that the automatic choice skips below 2,049 envs."""
    if request.param == "split":
        _PATH_SCHED.update(dyn_lpe=1, split=1, wide_n=-1)
    elif request.param == "wide":
        _PATH_SCHED.update(wide_n=1000000)
    else:
        _PATH_SCHED.update(wide_n=-1)
    yield request.param
    _PATH_SCHED.clear()


def _venv(rx, golden, tracks, n_agents=1, sched=None, **kw):
    cps = [golden.tracks[k]["cp"] if golden.tracks[k]["label"] != "default" else None for k in tracks]
    ws = [golden.tracks[k]["width"] for k in tracks]
    from rx.track import DEFAULT_CONTROL_POINTS
    cps = [DEFAULT_CONTROL_POINTS if c is None else c for c in cps]
    return rx.RacingVectorEnv(cps, ws, n_agents=n_agents, sched={**_PATH_SCHED, **(sched or {})}, **kw)


def test_sensor_angles_match_numpy(rx, golden):
    v = _venv(rx, golden, [0])
    assert np.array_equal(v.sensor_angles, REL1)
    v2 = _venv(rx, golden, [0], n_agents=2)
    assert np.array_equal(v2.sensor_angles, REL2)


def _inject(v, st):
    v.set_state(**{k: st[k] for k in ("x", "y", "angle", "vx", "vy", "progress", "last_progress", "last_steering",
                                      "flags", "steps")})
    if "finished_step" in st:
        v.set_state(finished_step=st["finished_step"])
    v.set_state(env_flags=np.zeros(v.num_envs, np.uint8))


def test_single_step_vs_golden_and_oracle(rx, golden, oracle_dev, dyn_path):
    step = golden["step_single"]
    n = len(step["x"])
    v = _venv(rx, golden, step["track"], autoreset="disabled")
    st = single_state_from(step)
    _inject(v, st)
    v.set_speed_weights(step["speed_weight"])
    obs, rew, done = v.step_device(torch.from_numpy(step["action"]).cuda(), full_info=True)
    torch.cuda.synchronize()
    g = v.get_state()
    obs = obs.cpu().numpy()
    rew64 = v.buf["reward64"].cpu().numpy()
    term = v.buf["terminated"].cpu().numpy().astype(bool)
    trunc = v.buf["truncated"].cpu().numpy().astype(bool)
    info = v.buf["info"].cpu().numpy()[:, 0]
    # --- vs reference (golden): masks exact, floats within tolerance
    fl = g["flags"]
    assert np.array_equal((fl & F_CRASHED) != 0, step["o_crashed"])
    assert np.array_equal((fl & F_FINISHED) != 0, step["o_finished"])
    assert np.array_equal(term, step["o_terminated"]) and np.array_equal(trunc, step["o_truncated"])
    cp = np.stack([(fl & F_CP25) != 0, (fl & F_CP50) != 0, (fl & F_CP75) != 0], 1)
    assert np.array_equal(cp, step["o_cp"].astype(bool))
    assert np.array_equal(g["steps"], step["o_steps"])
    assert np.array_equal(g["progress"], step["o_progress"])
    for k in ("x", "y", "angle", "vx", "vy"):
        np.testing.assert_allclose(g[k], step["o_" + k], rtol=0, atol=STATE_TOL, err_msg=k)
    np.testing.assert_allclose(obs, step["o_obs"], rtol=0, atol=OBS_TOL)
    np.testing.assert_allclose(rew64, step["o_reward"], rtol=0, atol=OBS_TOL)
    np.testing.assert_allclose(rew.cpu().numpy(), step["o_reward"].astype(np.float32), rtol=0, atol=OBS_TOL)
    np.testing.assert_allclose(info[:, 0], step["o_info_speed"], atol=1e-9)
    np.testing.assert_allclose(info[:, 1], step["o_info_progress"], atol=0)
    np.testing.assert_allclose(info[:, 2], step["o_progress_delta"], atol=1e-12)
    exact = (obs == step["o_obs"]).all(axis=1).mean()
    print(f"\nobs rows bit-identical to the reference: {exact:.4f} of {n}")
    # --- vs oracle (device libm): everything bit-exact
    st2 = single_state_from(step)
    o_obs, o_rew, o_term, o_trunc, o_info = oracle_dev.single_step(golden.table(), st2, step["action"], REL1,
                                                                    speed_weight=step["speed_weight"])
    assert np.array_equal(obs, o_obs)
    assert np.array_equal(rew64, o_rew)
    assert np.array_equal(term, o_term) and np.array_equal(trunc, o_trunc)
    for k in ("x", "y", "angle", "vx", "vy", "progress", "last_progress", "last_steering", "steps", "flags"):
        assert np.array_equal(g[k], st2[k]), k
    assert np.array_equal(info[:, :3], o_info)


def test_single_trajectories_vs_golden(rx, golden, dyn_path):
    tr = golden["traj_single"]
    tracks = list(tr["track"])
    v = _venv(rx, golden, tracks, autoreset="disabled")
    obs0 = v.reset_device().cpu().numpy()
    assert np.array_equal(obs0, tr["reset_obs"])  # reset obs: bit-exact (no sin/cos ambiguity hit here)
    off = tr["off"]
    L = np.diff(off)
    acts = np.zeros((len(tracks), 2), np.float32)
    worst = 0.0
    for t in range(int(L.max())):
        live = t < L
        for i in range(len(tracks)):
            acts[i] = tr["actions"][off[i] + t] if live[i] else 0.0
        obs, rew, _ = v.step_device(torch.from_numpy(acts).cuda(), full_info=True)
        obs = obs.cpu().numpy()
        rew64 = v.buf["reward64"].cpu().numpy()
        term = v.buf["terminated"].cpu().numpy().astype(bool)
        g = v.get_state()
        for i in np.nonzero(live)[0]:
            j = off[i] + t
            assert bool(term[i]) == bool(tr["terminated"][j]), (i, t)
            assert g["progress"][i] == tr["progress"][j], (i, t)
            worst = max(worst, float(np.abs(obs[i] - tr["obs"][j]).max()), abs(rew64[i] - tr["reward"][j]))
    print(f"\nmax |obs/reward - reference| over {int(L.sum())} trajectory steps: {worst:.3g}")
    assert worst <= OBS_TOL


def test_random_rollout_bit_exact_vs_oracle_dev(rx, golden, oracle_dev, dyn_path):
    """600 steps of random play on 2048 envs over all 21 golden tracks, next-step
    autoreset included: the kernels and the device-libm oracle must stay
    bit-identical at every step (long-horizon exactness)."""
    N = 2048
    tracks = np.arange(N) % golden.n_tracks
    v = _venv(rx, golden, tracks, autoreset="next_step")
    tab = golden.table()
    st = single_state(N)
    st["track"][:] = tracks
    o_obs = oracle_dev.single_reset(tab, st, REL1)
    obs = v.reset_device().cpu().numpy()
    assert np.array_equal(obs, o_obs)
    rng = np.random.default_rng(7)
    pending = np.zeros(N, bool)
    for t in range(600):
        a = np.stack([rng.uniform(-1, 1, N), rng.uniform(0.3, 1.0, N)], 1).astype(np.float32)
        obs, rew, done = v.step_device(torch.from_numpy(a).cuda())
        obs = obs.cpu().numpy()
        rew = rew.cpu().numpy()
        done = done.cpu().numpy()
        # oracle with gymnasium NEXT_STEP autoreset semantics
        o_obs, o_rew, o_term, o_trunc, _ = oracle_dev.single_step(tab, st, a, REL1)
        if pending.any():
            r_obs = oracle_dev.single_reset(tab, st, REL1, mask=pending)
            o_obs[pending] = r_obs[pending]
            o_rew[pending] = 0.0
            o_term[pending] = False
            o_trunc[pending] = False
        # (oracle stepped the pending envs first; their reset overwrote that state)
        assert np.array_equal(obs, o_obs), t
        assert np.array_equal(rew, o_rew.astype(np.float32)), t
        assert np.array_equal(done.astype(bool), o_term | o_trunc), t
        pending = (o_term | o_trunc)
    g = v.get_state()
    for k in ("x", "y", "angle", "vx", "vy", "steps", "flags"):
        assert np.array_equal(g[k], st[k]), k


@pytest.mark.parametrize("split", [-1, 1])
def test_multi_step_vs_golden_and_oracle(rx, golden, oracle_dev, split):
    """Two-car KATs on the one-kernel step (k_dyn2 + k_rays<2>) and on the split
    step (k_kin2 + k_step2<2>)."""
    step = golden["step_multi"]
    v = _venv(rx, golden, step["track"], n_agents=2, autoreset="disabled", sched=dict(split=split))
    st = multi_state_from(step)
    flat = {k: st[k].reshape(-1) for k in ("x", "y", "angle", "vx", "vy", "progress", "last_progress",
                                             "last_steering", "flags", "finished_step")}
    flat["steps"] = st["steps"]
    _inject(v, flat)
    obs, rew, done = v.step_device(torch.from_numpy(step["action"]).cuda(), full_info=True)
    obs = obs.cpu().numpy()
    rew64 = v.buf["reward64"].cpu().numpy()
    term = v.buf["terminated"].cpu().numpy().astype(bool)
    trunc = v.buf["truncated"].cpu().numpy().astype(bool)
    info = v.buf["info"].cpu().numpy()
    g = v.get_state()
    fl = g["flags"].reshape(-1, 2)
    assert np.array_equal((fl & F_CRASHED) != 0, step["o_crashed"])
    assert np.array_equal((fl & F_FINISHED) != 0, step["o_finished"])
    assert np.array_equal(g["finished_step"].reshape(-1, 2), step["o_finished_step"])
    assert np.array_equal(term, step["o_done"]) and np.array_equal(term | trunc, step["o_done_all"])
    assert np.array_equal(trunc, step["o_truncated"])
    assert np.array_equal(info[..., 3].astype(np.int32), step["o_placement"])
    np.testing.assert_allclose(obs, step["o_obs"], rtol=0, atol=OBS_TOL)
    np.testing.assert_allclose(rew64, step["o_reward"], rtol=0, atol=OBS_TOL)
    st2 = multi_state_from(step)
    o = oracle_dev.multi_step(golden.table(), st2, step["action"], REL2)
    assert np.array_equal(obs, o[0]) and np.array_equal(rew64, o[1])
    for k in ("x", "y", "angle", "vx", "vy", "progress", "flags", "finished_step"):
        assert np.array_equal(g[k].reshape(-1, 2), st2[k]), k


def test_multi_reset_slots(rx, golden):
    step = golden["step_multi"]
    n = len(step["reset_track"])
    v = _venv(rx, golden, step["reset_track"], n_agents=2, autoreset="disabled", seed=3)
    obs = v.reset_device().cpu().numpy()
    g = v.get_state()
    x = g["x"].reshape(-1, 2)
    # the start-slot shuffle is drawn on the device (the reference draws it from the
    # global numpy RNG); whichever slot each car got must match the golden reset
    # with the same slot order
    for i in range(n):
        first = 0 if np.isclose(x[i, 0], step["reset_x"][i][0]) and step["reset_order"][i] == 0 else None
        rows = [j for j in range(n) if step["reset_track"][j] == step["reset_track"][i]]
        match = [j for j in rows if np.array_equal(x[i], step["reset_x"][j])]
        assert match, i
        assert np.array_equal(obs[i], step["reset_obs"][match[0]])
        del first


def test_next_step_autoreset_semantics(rx, golden, dyn_path):
    """The step after a terminal one: reset obs, reward 0, terminated = truncated = False."""
    v = _venv(rx, golden, [0] * 64, autoreset="next_step")
    obs0 = v.reset_device().clone()
    acts = torch.tensor([[0.0, 1.0]] * 64, device="cuda")  # straight, full throttle: leaves the track at the first bend
    ended_at = None
    for t in range(400):
        obs, rew, done = v.step_device(acts)
        if done.bool().all():
            ended_at = t
            break
    assert ended_at is not None
    assert (v.state["env_flags"] & 1).bool().all()
    obs, rew, done = v.step_device(acts)
    assert torch.equal(obs, obs0)
    assert (rew == 0).all() and (done == 0).all()
    assert (v.state["steps"] == 0).all()


def test_episode_statistics(rx, golden, dyn_path):
    v = _venv(rx, golden, list(range(8)) * 8, autoreset="next_step")
    v.reset_device()
    ret = torch.zeros(64, dtype=torch.float64, device="cuda")
    acts = torch.tensor([[0.7, 1.0]] * 64, device="cuda")
    sums = [0.0, 0.0, 0]
    lens = torch.zeros(64, dtype=torch.int64, device="cuda")
    for t in range(300):
        pend = (v.state["env_flags"] & 1).bool()
        obs, rew, done = v.step_device(acts, full_info=True)
        r64 = v.buf["reward64"]
        ret = torch.where(pend, torch.zeros_like(ret), ret + r64)
        lens = torch.where(pend, torch.zeros_like(lens), lens + 1)
        ended = done.bool() & ~pend
        sums[0] += float(ret[ended].sum())
        sums[1] += float(lens[ended].sum())
        sums[2] += int(ended.sum())
    s = v.episode_stats()
    assert s[2] == sums[2] and s[2] > 0
    assert abs(s[0] - sums[0]) < 1e-6 * max(1.0, abs(sums[0])) and s[1] == sums[1]


def test_numpy_surface(rx, golden, dyn_path):
    v = _venv(rx, golden, [0, 1, 2, 3], autoreset="next_step")
    obs, infos = v.reset()
    assert obs.shape == (4, 15) and obs.dtype == np.float32
    tot = 0
    for t in range(200):
        obs, rew, term, trunc, infos = v.step(np.tile(np.array([[0.0, 1.0]], np.float32), (4, 1)))
        assert rew.dtype == np.float64 and term.dtype == bool
        if "episode" in infos:
            tot += int(infos["_episode"].sum())
            assert (infos["episode"]["l"][infos["_episode"]] > 0).all()
    assert tot > 0
    v.close()


@pytest.mark.parametrize("chunk,sort,order,sup", [(16, 1, 0, 0), (8, 3, 0, 0), (32, 0, 0, 0), (16, 4, 1, 0),
                                                  (16, 0, 1, 0), (8, 16, 1, 8), (6, 0, 0, 5), (24, 16, 1, 3),
                                                  (12, 16, 2, 6), (16, 3, 2, 0), (12, 0, 2, 6)])
def test_culling_and_sort_are_exact(rx, golden, chunk, sort, order, sup):
    """Chunk culling, spatial re-sorting and the ray-major lane order change
    scheduling only: outputs are bit-identical to the brute-force raycast over
    300 steps of random play."""
    N = 1536
    tracks = np.arange(N) % golden.n_tracks
    vb = _venv(rx, golden, tracks, autoreset="next_step", cull_chunk=0, sort_interval=0)
    vc = _venv(rx, golden, tracks, autoreset="next_step", cull_chunk=chunk, sort_interval=sort, ray_order=order,
              cull_super=sup)
    assert torch.equal(vb.reset_device(), vc.reset_device())
    g = torch.Generator(device="cuda").manual_seed(5)
    for t in range(300):
        a = torch.rand((N, 2), device="cuda", generator=g) * torch.tensor([2.0, 1.0], device="cuda") - torch.tensor(
            [1.0, 0.0], device="cuda")
        ob, rb, db = vb.step_device(a)
        oc, rc, dc = vc.step_device(a)
        assert torch.equal(ob, oc) and torch.equal(rb, rc) and torch.equal(db, dc), t


@pytest.mark.parametrize("n_widths", [1, 5])
def test_resort_both_scan_paths_are_exact(rx, golden, n_widths):
    """The re-sort takes its bin cursors from a scan inside the scatter up to
    8,192 bins (rx_sort.hip kFusedBins) and from k_sort_scan above; widths varied
    per env make 21 x 5 (geometry, width) slots, ~35 k bins, so both paths run.
    Against an unsorted env: outputs bit-identical over 160 steps (10 re-sorts at
    sort_interval 16), the wave order a permutation."""
    N = 4200
    tracks = np.arange(N) % golden.n_tracks
    ws = [golden.tracks[k]["width"] + (i // golden.n_tracks) % n_widths for i, k in enumerate(tracks)]
    from rx.track import DEFAULT_CONTROL_POINTS
    cps = [DEFAULT_CONTROL_POINTS if golden.tracks[k]["label"] == "default" else golden.tracks[k]["cp"] for k in tracks]
    va = rx.RacingVectorEnv(cps, ws, sched=_PATH_SCHED, autoreset="next_step", sort_interval=0)
    vb = rx.RacingVectorEnv(cps, ws, sched=_PATH_SCHED, autoreset="next_step", sort_interval=16)
    bins = vb.env_order()[1]
    assert (bins <= 8192) == (n_widths == 1) and bins > 0, bins
    assert torch.equal(va.reset_device(), vb.reset_device())
    g = torch.Generator(device="cuda").manual_seed(31)
    for t in range(160):
        a = torch.rand((N, 2), device="cuda", generator=g) * 2 - 1
        a[:, 1].abs_()
        oa, ra, da = va.step_device(a)
        ob, rb, db = vb.step_device(a)
        assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(da, db), t
    perm = vb.env_order()[0]
    assert np.array_equal(np.sort(perm), np.arange(N))
    sa, sb = va.get_state(), vb.get_state()
    for k in sa:
        assert np.array_equal(sa[k], sb[k]), k


def test_resort_histogram_survives_split_phase_sequences(rx, golden):
    """The split step's REWARD half counts the re-sort bins as it writes the keys
    (rx_api.cpp sort_hist_done).  Keys requested again before their sort ran --
    rx_step_phases(1) twice with sort_interval = 1, or rx_step_phases(1) then a
    reset -- must not leave a stale or doubled histogram (k_sort_scatter would
    write past N).  Against an unsorted env on the same phase sequence: obs,
    rewards, dones and the state bit-identical, and the wave order a permutation."""
    N = 8256
    tracks = np.arange(N) % golden.n_tracks
    va = _venv(rx, golden, tracks, seed=2, autoreset="next_step", sort_interval=0)
    vb = _venv(rx, golden, tracks, seed=2, autoreset="next_step", sort_interval=1)
    assert vb.schedule()["split"] == 1
    assert torch.equal(va.reset_device(), vb.reset_device())
    g = torch.Generator(device="cuda").manual_seed(23)

    def act():
        a = torch.rand((N, 2), device="cuda", generator=g) * 2 - 1
        a[:, 1].abs_()
        return a

    for t in range(40):
        a1, a2 = act(), act()
        if t % 2 == 0:  # dynamics twice (keys re-requested before the sort), then the raycast (sort)
            for v in (va, vb):
                v.step_device(a1, phases=1)
                v.step_device(a2, phases=1)
            oa, ra, da = va.step_device(a2, phases=2)
            ob, rb, db = vb.step_device(a2, phases=2)
        else:  # dynamics (keys + fused count), then a reset of every env (keys rewritten, not counted)
            for v in (va, vb):
                v.step_device(a1, phases=1)
                v.reset_device()
            oa, ra, da = va.step_device(a2)
            ob, rb, db = vb.step_device(a2)
        assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(da, db), t
        perm = vb.env_order()[0]
        assert np.array_equal(np.sort(perm), np.arange(N)), t
    sa, sb = va.get_state(), vb.get_state()
    for k in sa:
        assert np.array_equal(sa[k], sb[k]), k
    va.close()
    vb.close()


@pytest.mark.parametrize("n_agents,N", [(1, 1536), (1, 8256), (2, 512)])
def test_segment_prefilter_is_exact(rx, golden, n_agents, N):
    """The float32 segment pre-filter (seg_may_hit) only skips exact segment
    tests that cannot report a hit: with (seg_filter on, the default) and
    without it (seg_filter = -1), obs, rewards and dones are bit-identical over
    300 steps of random play (both culled; culled == brute force is checked
    above).  8,256 envs run the split step (k_step2), fewer the one-kernel path
    (k_rays)."""
    tracks = np.arange(N) % golden.n_tracks
    va = _venv(rx, golden, tracks, n_agents=n_agents, seed=3, autoreset="next_step", sched=dict(seg_filter=-1))
    vb = _venv(rx, golden, tracks, n_agents=n_agents, seed=3, autoreset="next_step", sched=dict(seg_filter=1))
    assert torch.equal(va.reset_device(), vb.reset_device())
    g = torch.Generator(device="cuda").manual_seed(12)
    shape = (N, 2) if n_agents == 1 else (N, 2, 2)
    for t in range(300):
        a = torch.rand(shape, device="cuda", generator=g) * 2 - 1
        if n_agents == 1:
            a[:, 1].abs_()
        oa, ra, da = va.step_device(a)
        ob, rb, db = vb.step_device(a)
        assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(da, db), t
    va.close()
    vb.close()


@pytest.mark.parametrize("lpr", [2, 4])
@pytest.mark.parametrize("n_agents,N", [(1, 1536), (1, 8256), (2, 512), (2, 3000)])
def test_lanes_per_ray_are_exact(rx, golden, n_agents, N, lpr):
    """Two or four lanes per ray (ray_lpr: the lanes split each scanned
    leaf and take the minimum of their bests; 4 is the default up to
    RX_RAY_LPR4_N (env, agent) pairs) against one lane per ray: obs, rewards
    and dones are bit-identical over 300 steps of random play.  Ragged sizes
    leave partial ray waves (duplicate-task lanes); 8,256 envs run the split
    step."""
    tracks = np.arange(N) % golden.n_tracks
    va = _venv(rx, golden, tracks, n_agents=n_agents, seed=4, autoreset="next_step", sched=dict(ray_lpr=1))
    vb = _venv(rx, golden, tracks, n_agents=n_agents, seed=4, autoreset="next_step", sched=dict(ray_lpr=lpr))
    assert torch.equal(va.reset_device(), vb.reset_device())
    g = torch.Generator(device="cuda").manual_seed(13)
    shape = (N, 2) if n_agents == 1 else (N, 2, 2)
    for t in range(300):
        a = torch.rand(shape, device="cuda", generator=g) * 2 - 1
        if n_agents == 1:
            a[:, 1].abs_()
        oa, ra, da = va.step_device(a)
        ob, rb, db = vb.step_device(a)
        assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(da, db), t
    va.close()
    vb.close()


@pytest.mark.parametrize("tail,tail_lpr,dispatch", [(3, 2, 0), (11, 4, 0), (5, 2, 1), (2, 4, 2)])
@pytest.mark.parametrize("n_agents,N", [(1, 8256), (2, 3000)])
def test_ray_tail_split_is_exact(rx, golden, n_agents, N, tail, tail_lpr, dispatch):
    """rx_config.ray_tail (ABI v19): the last `tail` ray-wave classes of the
    dispatch order cast at 2 or 4 lanes per ray (each 64-task wave split into
    2 or 4 waves, placed at the end of the table on the group's XCD) against the
    plain one-lane-per-ray table: obs, rewards and dones bit-identical over 300
    steps of random play, on the split step (k_step2) and for two cars; the
    dispatch orders (edges-first auto, centre-first, ascending) likewise."""
    tracks = np.arange(N) % golden.n_tracks
    base = dict(ray_lpr=1, ray_tail=-1)
    va = _venv(rx, golden, tracks, n_agents=n_agents, seed=4, autoreset="next_step", sched=base)
    vb = _venv(rx, golden, tracks, n_agents=n_agents, seed=4, autoreset="next_step",
               sched=dict(ray_lpr=1, ray_tail=tail, ray_tail_lpr=tail_lpr, ray_dispatch=dispatch))
    sb = vb.schedule()
    assert sb["ray_tail"] == tail and sb["ray_tail_lpr"] == tail_lpr and sb["ray_tail_from"] >= 0
    tab = vb.ray_wave_table()
    assert (tab["count"][sb["ray_tail_from"]:] <= 64 // tail_lpr).all()
    assert tab["count"].sum() == N * n_agents * 11  # every task in exactly one wave
    tasks = np.concatenate([np.arange(s, s + c) for s, c in zip(tab["task_start"], tab["count"]) if c > 0])
    assert np.array_equal(np.sort(tasks), np.arange(N * n_agents * 11))
    assert torch.equal(va.reset_device(), vb.reset_device())
    g = torch.Generator(device="cuda").manual_seed(15)
    shape = (N, 2) if n_agents == 1 else (N, 2, 2)
    for t in range(300):
        a = torch.rand(shape, device="cuda", generator=g) * 2 - 1
        if n_agents == 1:
            a[:, 1].abs_()
        oa, ra, da = va.step_device(a)
        ob, rb, db = vb.step_device(a)
        assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(da, db), t
    # the raycast on its own (k_rays, rx_step_phases) reads the same table
    oa = va.step_device(torch.zeros(shape, device="cuda"), phases=2)[0]
    ob = vb.step_device(torch.zeros(shape, device="cuda"), phases=2)[0]
    assert torch.equal(oa, ob)
    va.close()
    vb.close()


@pytest.mark.parametrize("n_agents,N,interval", [(1, 4100, 7), (1, 8256, 16), (2, 3000, 3)])
def test_task_sort_interval_is_exact(rx, golden, n_agents, N, interval):
    """rx_config.task_sort (ABI v20): the ray-task direction sort every `interval`
    dynamics launches (in between the ray waves reuse the previous order; every
    spatial re-sort forces a new one) against a sort every launch: obs, rewards,
    dones and the state bit-identical over 300 steps of random play with
    autoresets, single-agent and two-car."""
    tracks = np.arange(N) % golden.n_tracks
    va = _venv(rx, golden, tracks, n_agents=n_agents, seed=6, autoreset="next_step", sched=dict(task_sort=1))
    vb = _venv(rx, golden, tracks, n_agents=n_agents, seed=6, autoreset="next_step", sched=dict(task_sort=interval))
    assert va.schedule()["task_sort"] == 1 and vb.schedule()["task_sort"] == interval
    assert torch.equal(va.reset_device(), vb.reset_device())
    g = torch.Generator(device="cuda").manual_seed(21)
    shape = (N, 2) if n_agents == 1 else (N, 2, 2)
    for t in range(300):
        a = torch.rand(shape, device="cuda", generator=g) * 2 - 1
        if n_agents == 1:
            a[:, 1].abs_()
        oa, ra, da = va.step_device(a)
        ob, rb, db = vb.step_device(a)
        assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(da, db), t
    sa, sb = va.get_state(), vb.get_state()
    for k in sa:
        assert np.array_equal(sa[k], sb[k]), k
    va.close()
    vb.close()


@pytest.mark.parametrize("lpe", [2, 4])
@pytest.mark.parametrize("N", [4100, 8256])
def test_reward_lanes_per_env_are_exact(rx, golden, N, lpe):
    """The split step's REWARD half at 2 or 4 lanes per env (reward_lpe:
    the five argmin points spread over the env's lanes, the wall test OR-ed
    across them) against one lane per env: obs, rewards and dones
    bit-identical over 300 steps of random play, episode counts exact (ragged last
    dynamics wave at 4,100 envs; the episode-return sums only to f64
    rounding, as their atomic order differs)."""
    tracks = np.arange(N) % golden.n_tracks
    va = _venv(rx, golden, tracks, seed=6, autoreset="next_step", sched=dict(reward_lpe=1))
    vb = _venv(rx, golden, tracks, seed=6, autoreset="next_step", sched=dict(reward_lpe=lpe))
    assert torch.equal(va.reset_device(), vb.reset_device())
    g = torch.Generator(device="cuda").manual_seed(14)
    for t in range(300):
        a = torch.rand((N, 2), device="cuda", generator=g) * 2 - 1
        a[:, 1].abs_()
        oa, ra, da = va.step_device(a)
        ob, rb, db = vb.step_device(a)
        assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(da, db), t
    (ra_, la_, ca_), (rb_, lb_, cb_) = va.episode_stats(), vb.episode_stats()
    assert ca_ == cb_ > 0 and la_ == lb_  # counts and (integer) lengths exact
    assert abs(ra_ - rb_) <= 1e-9 * max(1.0, abs(ra_))  # f64 atomic sums: order differs across shards
    va.close()
    vb.close()


@pytest.mark.parametrize("N,lpr", [(3000, 0), (8192, 0), (2048, 1)])
def test_two_car_reward_lane_per_car_is_exact(rx, golden, N, lpr):
    """k_step2<2>'s REWARD half with a lane per car (reward_lpe = 2 for two cars:
    one closest-waypoint pass per wave instead of two, the pair swapping progress
    and crash flags) against one lane per env: obs, rewards, dones, placement /
    info and the whole state bit-identical over 300 steps of random play; episode
    counts exact.  Ragged last wave at 3,000 envs."""
    tracks = np.arange(N) % golden.n_tracks
    base = dict(ray_lpr=lpr) if lpr else {}
    va = _venv(rx, golden, tracks, n_agents=2, seed=7, autoreset="next_step", sched=dict(base, reward_lpe=1))
    vb = _venv(rx, golden, tracks, n_agents=2, seed=7, autoreset="next_step", sched=dict(base, reward_lpe=2))
    assert vb.schedule()["reward_lpe"] == 2 and vb.schedule()["split"] == 1
    assert torch.equal(va.reset_device(), vb.reset_device())
    g = torch.Generator(device="cuda").manual_seed(19)
    for t in range(300):
        a = torch.rand((N, 2, 2), device="cuda", generator=g) * 2.4 - 1.2
        oa, ra, da = va.step_device(a, full_info=True)
        ob, rb, db = vb.step_device(a, full_info=True)
        assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(da, db), t
        for k in ("reward64", "terminated", "truncated", "info", "ep_done"):
            assert torch.equal(va.buf[k], vb.buf[k]), (t, k)
    sa, sb = va.get_state(), vb.get_state()
    for k in sa:
        assert np.array_equal(sa[k], sb[k]), k
    (ra_, la_, ca_), (rb_, lb_, cb_) = va.episode_stats(), vb.episode_stats()
    assert ca_ == cb_ > 0 and la_ == lb_ and abs(ra_ - rb_) <= 1e-9 * max(1.0, abs(ra_))
    va.close()
    vb.close()


def test_culled_raycast_on_golden_kats(rx, golden):
    """Track.raycast golden KATs (incl. no-hit, > 50 uncapped, grazing, far
    origins) through the culled kernel: sensor 5 (relative angle exactly 0)
    must read float32(t_ref) / 50 exactly, with and without culling."""
    rc = golden["raycast"]
    n = len(rc["t"])
    for chunk in (0, 16):
        v = _venv(rx, golden, rc["track"], autoreset="disabled", cull_chunk=chunk, sort_interval=0)
        v.set_state(x=rc["ox"], y=rc["oy"], angle=rc["dir"], progress=np.zeros(n))
        obs = v.step_device(torch.zeros((n, 2), device="cuda"), phases=2)[0].cpu().numpy()
        want = (rc["t"].astype(np.float32) / np.float32(50.0))
        # the kernels' rx_sincos may differ from glibc's sin/cos by 1 ulp in a few KATs:
        # compare against the oracle (device libm) exactly, against the reference to 1e-5
        np.testing.assert_allclose(obs[:, 5], want, rtol=0, atol=1e-5)
        assert (obs[:, 5] == want).mean() > 0.99


def test_vector_env_from_table_file(tmp_path):
    """RacingVectorEnv.from_table (on-disk track table) == the env built from the pool."""
    import random
    from rx.track import gen_tracks
    from rx.vector_env import RacingVectorEnv
    random.seed(1)
    np.random.seed(1)
    pool = gen_tracks(64, seed=1)
    widths = [np.random.randint(6, 10) for _ in range(64)]
    a = RacingVectorEnv(pool, widths, device="cuda")
    p = tmp_path / "tbl.npz"
    a.save_table(p)
    b = RacingVectorEnv.from_table(p, device="cuda")
    assert np.array_equal(a.track_of_env, b.track_of_env)
    a.reset_device()
    b.reset_device()
    g = torch.Generator(device="cuda").manual_seed(0)
    for _ in range(200):
        act = torch.rand((64, 2), generator=g, device="cuda") * torch.tensor([2.0, 1.0], device="cuda") \
            - torch.tensor([1.0, 0.0], device="cuda")
        oa, ra, da = a.step_device(act)
        ob, rb, db = b.step_device(act)
        assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(da, db)
    a.close()
    b.close()


@pytest.mark.parametrize("order", [1, 2])
def test_ray_major_two_car_is_exact(rx, golden, order):
    """Ray-major (1) and sorted-task (2) lane orders for the two-car kernel (agent, ray) x envs."""
    N = 512
    tracks = np.arange(N) % golden.n_tracks
    va = _venv(rx, golden, tracks, n_agents=2, seed=3)
    vb = _venv(rx, golden, tracks, n_agents=2, seed=3, sort_interval=2, ray_order=order)
    assert torch.equal(va.reset_device(), vb.reset_device())
    g = torch.Generator(device="cuda").manual_seed(8)
    for t in range(200):
        a = torch.rand((N, 2, 2), device="cuda", generator=g) * 2 - 1
        oa, ra, da = va.step_device(a)
        ob, rb, db = vb.step_device(a)
        assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(da, db), t


def test_dyn_lanes_per_env_paths_agree(rx, golden):
    """Small vector envs run the wide kernels (<= 2,048 envs), larger ones the
    split step at one lane per env: envs are independent, so the first envs of
    a large vector env must step exactly like a small one with the same tracks
    and actions."""
    n_small, n_big = 1024, 8256
    tracks = np.arange(n_big) % golden.n_tracks
    big = _venv(rx, golden, tracks, autoreset="next_step")
    small = _venv(rx, golden, tracks[:n_small], autoreset="next_step")
    assert torch.equal(big.reset_device()[:n_small], small.reset_device())
    g = torch.Generator(device="cuda").manual_seed(21)
    for t in range(150):
        a = torch.rand((n_big, 2), device="cuda", generator=g) * torch.tensor([2.0, 1.0], device="cuda") - torch.tensor(
            [1.0, 0.0], device="cuda")
        ob, rb, db = big.step_device(a)
        os_, rs, ds = small.step_device(a[:n_small].contiguous())
        assert torch.equal(ob[:n_small], os_) and torch.equal(rb[:n_small], rs) and torch.equal(db[:n_small], ds), t
    big.close()
    small.close()


@pytest.mark.parametrize("n_agents", [1, 2])
@pytest.mark.parametrize("autoreset", ["next_step", "disabled"])
def test_split_step_equals_one_kernel_step(rx, golden, autoreset, n_agents):
    """The split step (k_kin1 / k_kin2 + fused REWARD/raycast k_step2<A>) == the
    one-kernel step bit for bit: obs, rewards (f32 and f64), masks, placement,
    info, episode statistics and the whole f64 state, over 300 steps of random
    play (two cars: start-slot draws, car-car contact and placement included)."""
    N = 2048
    tracks = np.arange(N) % golden.n_tracks
    kw = dict(autoreset=autoreset, n_agents=n_agents)
    if n_agents == 2:
        kw["seed"] = 5
    one = dict(dyn_lpe=1) if n_agents == 1 else {}
    va = _venv(rx, golden, tracks, sched=dict(one, split=-1), **kw)
    vb = _venv(rx, golden, tracks, sched=dict(one, split=1), **kw)
    assert torch.equal(va.reset_device(), vb.reset_device())
    g = torch.Generator(device="cuda").manual_seed(17)
    for t in range(300):
        if n_agents == 1:
            a = torch.rand((N, 2), device="cuda", generator=g) * torch.tensor([2.4, 1.4], device="cuda") - torch.tensor(
                [1.2, 0.2], device="cuda")
        else:  # both cars often steer into each other: start slots are 3.5 apart
            a = torch.rand((N, 2, 2), device="cuda", generator=g) * 2.4 - 1.2
        oa, ra, da = va.step_device(a, full_info=True)
        ob, rb, db = vb.step_device(a, full_info=True)
        assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(da, db), t
        for k in ("reward64", "terminated", "truncated", "info", "ep_done"):
            assert torch.equal(va.buf[k], vb.buf[k]), (t, k)
    sa, sb = va.get_state(), vb.get_state()
    for k in sa:
        assert np.array_equal(sa[k], sb[k]), k
    ea, eb = va.episode_stats(), vb.episode_stats()  # atomics: the f64 sum order is not fixed
    assert ea[1:] == eb[1:] and ea[0] == pytest.approx(eb[0], rel=1e-12)
