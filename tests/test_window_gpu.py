"""rx_steps' multi-step windows (k_window, ABI v21; DESIGN.md §3 "Multi-step
window") against the per-step launches and against the oracle.

k_window runs the steps between two spatial re-sorts in ONE launch, a
workgroup per 64-env block (phase K: dyn1_env<1, KIN> + the block's ray-task
sort into LDS; phase R: REWARD and the block's ray waves).  It calls the device
functions of k_kin1 / k_step2 on the same rows, so every output must equal K
rx_step calls BIT FOR BIT:

* window on vs window off (rx_steps enqueuing rx_step's launches) on the same
  actions: every step's obs row, f32 reward and done, the terminated /
  truncated masks, the whole f64 state and the episode counts; the episode
  return / length sums only to f64 rounding (their atomic order differs, as
  between any two launch schedules);
* at 65,536 envs (configs[2], the bench) a fixed 2,048-env subset is stepped by
  the device-libm oracle beside the full window launch and compared after every
  step (environment/racing_env.py:104-167, next-step autoreset);
* ragged blocks (slot groups of any size), calls whose K starts mid re-sort
  interval or spans several, windows longer than RX_WIN_MAX_STEPS, and the
  re-sort keys written on exactly the steps the per-step path writes them.
"""
import ctypes
import random

import numpy as np
import pytest
import torch

from oracle.orc import single_state

pytestmark = pytest.mark.gpu


def _seed1_pool(n):
    from rx.track import gen_tracks
    random.seed(1)
    np.random.seed(1)
    pool = gen_tracks(num_tracks=n, seed=1)
    widths = [np.random.randint(6, 10) for _ in range(n)]
    return pool, widths


def _actions(g, K, N):
    a = torch.rand((K, N, 2), device="cuda", generator=g)
    a[..., 0].mul_(2.0).sub_(1.0)
    return a


MODES = [pytest.param(1, id="k_window"), pytest.param(2, id="k_flow")]


def _flow_ok(v):
    """k_flow records a bounded-spin timeout (an incomplete launch) in a device flag."""
    n = ctypes.c_int32(-1)
    from rx import _lib
    _lib.check(v.L.rx_flow_errors(v._h, ctypes.byref(n)), "rx_flow_errors")
    assert n.value == 0, "k_flow: a wave timed out waiting for a task"


def _pair(pool, widths, sched=None, sort_interval=None, mode=1):
    from rx.vector_env import RacingVectorEnv
    kw = dict(device="cuda", autoreset="next_step", sort_interval=sort_interval)
    on = RacingVectorEnv(pool, widths, sched={**(sched or {}), "window": mode}, **kw)
    off = RacingVectorEnv(pool, widths, sched={**(sched or {}), "window": -1}, **kw)
    assert on.schedule()["window"] == mode, on.schedule()
    assert off.schedule()["window"] == 0
    return on, off


def _compare_calls(on, off, Ks, seed):
    """Step both envs through rx_steps with every step's outputs in its own row."""
    N, D = on.num_envs, on.D
    g = torch.Generator(device="cuda").manual_seed(seed)
    assert torch.equal(on.reset_device(), off.reset_device())
    ended = 0
    for K in Ks:
        a = _actions(g, K, N)
        outs = []
        print(f"window parity: N={N} K={K}", flush=True)  # progress (a long GPU test prints as it goes)
        for v in (on, off):
            o = torch.full((K, N, D), float("nan"), device="cuda")
            r = torch.full((K, N), float("nan"), device="cuda")
            d = torch.full((K, N), float("nan"), device="cuda")
            v.steps_device(a, obs_out=o, reward_out=r, done_out=d)
            outs.append((o, r, d, v.buf["terminated"].clone(), v.buf["truncated"].clone()))
        for x, y in zip(*outs):
            assert torch.equal(x, y), K
        ended += int(outs[0][2].sum())
    _flow_ok(on)
    sa, sb = on.get_state(), off.get_state()
    for k in sa:
        assert np.array_equal(sa[k], sb[k]), k
    ea, eb = on.episode_stats(), off.episode_stats()
    assert ea[2] == eb[2] and ea[1] == eb[1]  # counts and lengths are exact (integers in f64)
    assert abs(ea[0] - eb[0]) <= 1e-9 * max(1.0, abs(eb[0]))  # return sums: atomic order only
    return ended


@pytest.mark.parametrize("mode", MODES)
def test_window_equals_per_step_at_65536(mode):
    """configs[2]: the bench's 65,536 envs (1,029 blocks, re-sort every 8 steps);
    calls of 20 (the driver's), 3, 8 and 37 steps -- windows starting anywhere in
    the re-sort interval -- bit-identical to the per-step launches."""
    pool, widths = _seed1_pool(65536)
    on, off = _pair(pool, widths, mode=mode)
    assert on.sort_interval == 8
    ended = _compare_calls(on, off, (20, 3, 8, 37), seed=5)
    assert ended > 5000
    # the reset and the 68 steps were dynamics launches 0 .. 68; launch c writes the re-sort
    # keys when c % 8 == 0, so the next 16 steps (69 .. 84) are windows 69-72, 73-80, 81-84
    on.profile(1)
    on.steps_device(_actions(torch.Generator(device="cuda").manual_seed(2), 16, 65536))
    prof = on.profile_read()
    assert prof.get("k_window", (0, 0))[1] == 3, prof
    on.close()
    off.close()


@pytest.mark.parametrize("mode", MODES)
def test_window_equals_per_step_at_4096(mode):
    """configs[1]'s env count with the window schedule forced (one lane per ray and
    per env, the task sort every launch: what k_window runs) against the per-step
    launches of the same schedule, re-sort every 16 steps."""
    pool, widths = _seed1_pool(4096)
    on, off = _pair(pool, widths, sched=dict(ray_lpr=1, reward_lpe=1, task_sort=1), mode=mode)
    _compare_calls(on, off, (128, 5, 16, 70), seed=9)
    on.close()
    off.close()


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("N,interval", [(4100, 7), (3001, 0), (8256, 3)])
def test_window_ragged_blocks_and_intervals(N, interval, mode):
    """Slot groups of every size (partial blocks), no re-sort at all (one window
    per call, split at RX_WIN_MAX_STEPS = 64 steps), and a re-sort every 3 steps."""
    pool, widths = _seed1_pool(N)
    on, off = _pair(pool, widths, sched=dict(ray_lpr=1, reward_lpe=1, task_sort=1), sort_interval=interval,
                    mode=mode)
    _compare_calls(on, off, (1, 9, 100, 2), seed=N)
    on.close()
    off.close()


@pytest.mark.parametrize("mode", MODES)
def test_window_65536_subset_bit_exact_vs_oracle(oracle_dev, mode):
    """The window path at the bench's launch geometry vs the device-libm oracle: a
    2,048-env subset of 65,536 compared after every one of 120 steps (six calls of
    20 steps, each call's per-step rows kept), whole f64 state after every call."""
    from rx.vector_env import RacingVectorEnv
    from tests.test_fullsize_gpu import REL1, _oracle_table
    N = 65536
    pool, widths = _seed1_pool(N)
    v = RacingVectorEnv(pool, widths, device="cuda", autoreset="next_step", sched=dict(window=mode))
    assert v.schedule()["window"] == mode
    idx = np.sort(np.random.default_rng(23).choice(N, 2048, replace=False))
    tab = _oracle_table(v)
    st = single_state(len(idx))
    st["track"][:] = v.track_of_env[idx]
    obs = v.reset_device().cpu().numpy()
    assert np.array_equal(obs[idx], oracle_dev.single_reset(tab, st, REL1))
    rng = np.random.default_rng(29)
    pending = np.zeros(len(idx), bool)
    ended = 0
    K = 20
    for call in range(6):
        a = np.stack([rng.uniform(-1, 1, (K, N)), rng.uniform(0, 1, (K, N))], -1).astype(np.float32)
        o = torch.empty((K, N, v.D), device="cuda")
        r = torch.empty((K, N), device="cuda")
        d = torch.empty((K, N), device="cuda")
        v.steps_device(torch.from_numpy(a).cuda(), obs_out=o, reward_out=r, done_out=d)
        o, r, d = o.cpu().numpy(), r.cpu().numpy(), d.cpu().numpy().astype(bool)
        for k in range(K):
            o_obs, o_rew, o_term, o_trunc, _ = oracle_dev.single_step(tab, st, a[k][idx], REL1)
            if pending.any():  # gymnasium next-step autoreset
                r_obs = oracle_dev.single_reset(tab, st, REL1, mask=pending)
                o_obs[pending] = r_obs[pending]
                o_rew[pending] = 0.0
                o_term[pending] = False
                o_trunc[pending] = False
            t = call * K + k
            assert np.array_equal(o[k][idx], o_obs), t
            assert np.array_equal(r[k][idx], o_rew.astype(np.float32)), t
            assert np.array_equal(d[k][idx], o_term | o_trunc), t
            pending = o_term | o_trunc
            ended += int(pending.sum())
        g = v.get_state()
        for key in ("x", "y", "angle", "vx", "vy", "progress", "last_progress", "last_steering", "steps", "flags"):
            assert np.array_equal(g[key][idx], st[key]), (call, key)
    assert ended > 100
    _flow_ok(v)
    v.close()


@pytest.mark.parametrize("mode", MODES)
def test_window_graph_replay_equals_eager(mode):
    """The bench captures its timed steps in a HIP graph: a captured rx_steps call
    (k_window_args + k_window + the re-sorts) replayed == the same call eager."""
    pool, widths = _seed1_pool(16384)
    from rx.vector_env import RacingVectorEnv
    va = RacingVectorEnv(pool, widths, device="cuda", autoreset="next_step", sched=dict(ray_lpr=1, reward_lpe=1,
                                                                                          task_sort=1, window=mode))
    vb = RacingVectorEnv(pool, widths, device="cuda", autoreset="next_step", sched=dict(ray_lpr=1, reward_lpe=1,
                                                                                          task_sort=1, window=mode))
    assert va.schedule()["window"] == mode
    va.reset_device()
    vb.reset_device()
    a = _actions(torch.Generator(device="cuda").manual_seed(4), 24, 16384)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=torch.cuda.Stream()):
        va.steps_device(a)
    torch.cuda.synchronize()
    gr.replay()
    vb.steps_device(a)  # the capture executed nothing: vb's one eager call == va's one replay
    torch.cuda.synchronize()
    assert torch.equal(va.buf["obs"], vb.buf["obs"]) and torch.equal(va.buf["reward"], vb.buf["reward"])
    sa, sb = va.get_state(), vb.get_state()
    for k in sa:
        assert np.array_equal(sa[k], sb[k]), k
    va.close()
    vb.close()
