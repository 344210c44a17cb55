"""Pin the oracle (oracle/rx_oracle.c) against the reference's own outputs.

The golden vectors were produced by importing the reference unmodified
(tests/golden/gen_golden.py).  With glibc numerics the oracle must reproduce
every one of them BIT FOR BIT -- that is what makes it a trustworthy checker
for the HIP kernels.  The device-libm build (correctly rounded sin/cos, x*x for
pow(x,2)) must match the integer masks exactly and the floats within the
north-star tolerance.
"""
import numpy as np
import pytest

from oracle.orc import F_CP25, F_CP50, F_CP75, F_CRASHED, F_FINISHED, F_HAS_CRASHED, sensor_angles
from tests.golden_util import multi_state_from, single_state_from

REL_SINGLE = sensor_angles(11, np.pi / 3)
REL_MULTI = sensor_angles(11, np.pi / 2)


def test_raycast_bit_exact(golden, oracle):
    rc = golden["raycast"]
    tab = golden.table()
    got = np.array([oracle.raycast(tab.segments(int(k)), ox, oy, d)
                    for k, ox, oy, d in zip(rc["track"], rc["ox"], rc["oy"], rc["dir"])])
    assert np.array_equal(got, rc["t"])
    # the set exercises the uncapped (>50) and no-hit (==50) branches
    assert (rc["t"] > 50).sum() > 10 and (rc["t"] == 50).sum() > 10


def test_closest_waypoint(golden, oracle):
    rng = np.random.default_rng(0)
    for k in (0, 16, 17):
        wp = golden.tracks[k]["wp"]
        for _ in range(200):
            x, y = rng.uniform(-80, 120, 2)
            ref = int(np.sum((wp - np.array((x, y))) ** 2, axis=1).argmin())
            assert oracle.closest_wp(wp, x, y) == ref


def _check_single(step, st, obs, rew, term, trunc, info, exact=True):
    fl = st["flags"]
    assert np.array_equal((fl & F_CRASHED) != 0, step["o_crashed"])
    assert np.array_equal((fl & F_FINISHED) != 0, step["o_finished"])
    assert np.array_equal(term, step["o_terminated"])
    assert np.array_equal(trunc, step["o_truncated"])
    cp = np.stack([(fl & F_CP25) != 0, (fl & F_CP50) != 0, (fl & F_CP75) != 0], axis=1)
    assert np.array_equal(cp, step["o_cp"].astype(bool))
    assert np.array_equal(st["steps"], step["o_steps"])
    assert np.array_equal(st["progress"], step["o_progress"])  # idx/W: exact whenever argmin agrees
    if exact:
        for k in ("x", "y", "angle", "vx", "vy", "last_progress", "last_steering"):
            assert np.array_equal(st[k], step["o_" + k]), k
        assert np.array_equal(obs, step["o_obs"])
        assert np.array_equal(rew, step["o_reward"])
        assert np.array_equal(info[:, 0], step["o_info_speed"])
        assert np.array_equal(info[:, 1], step["o_info_progress"])
        assert np.array_equal(info[:, 2], step["o_progress_delta"])
    else:
        for k in ("x", "y", "angle", "vx", "vy"):
            np.testing.assert_allclose(st[k], step["o_" + k], rtol=0, atol=1e-9, err_msg=k)
        np.testing.assert_allclose(obs, step["o_obs"], rtol=0, atol=1e-5)
        np.testing.assert_allclose(rew, step["o_reward"], rtol=0, atol=1e-5)


def test_single_step_bit_exact(golden, oracle):
    step = golden["step_single"]
    st = single_state_from(step)
    obs, rew, term, trunc, info = oracle.single_step(golden.table(), st, step["action"], REL_SINGLE,
                                                      speed_weight=step["speed_weight"])
    _check_single(step, st, obs, rew, term, trunc, info, exact=True)


def test_single_step_device_libm_within_tolerance(golden, oracle_dev):
    """The HIP kernels' numerics (CR sin/cos, x*x) vs the reference: masks exact, floats <= 1e-5."""
    step = golden["step_single"]
    st = single_state_from(step)
    obs, rew, term, trunc, info = oracle_dev.single_step(golden.table(), st, step["action"], REL_SINGLE,
                                                          speed_weight=step["speed_weight"])
    _check_single(step, st, obs, rew, term, trunc, info, exact=False)


@pytest.mark.parametrize("dev", [False, True])
def test_single_trajectories(golden, oracle, oracle_dev, dev):
    orc = oracle_dev if dev else oracle
    tr = golden["traj_single"]
    tab = golden.table()
    from oracle.orc import single_state
    for i, k in enumerate(tr["track"]):
        a, b = tr["off"][i], tr["off"][i + 1]
        st = single_state(1)
        st["track"][:] = k
        obs0 = orc.single_reset(tab, st, REL_SINGLE)
        assert np.array_equal(obs0[0], tr["reset_obs"][i])
        for t in range(a, b):
            obs, rew, term, trunc, info = orc.single_step(tab, st, tr["actions"][t][None], REL_SINGLE)
            assert bool(term[0]) == bool(tr["terminated"][t]) and bool(trunc[0]) == bool(tr["truncated"][t])
            if not dev:
                assert np.array_equal(obs[0], tr["obs"][t]), (i, t)
                assert rew[0] == tr["reward"][t]
                assert st["x"][0] == tr["x"][t] and st["y"][0] == tr["y"][t] and st["angle"][0] == tr["angle"][t]
                assert st["vx"][0] == tr["vx"][t] and st["vy"][0] == tr["vy"][t]
            else:
                np.testing.assert_allclose(obs[0], tr["obs"][t], atol=1e-5)
                np.testing.assert_allclose(rew[0], tr["reward"][t], atol=1e-5)
            assert st["progress"][0] == tr["progress"][t]


def _check_multi(step, st, obs, rew, done, done_all, trunc, place, info, exact):
    fl = st["flags"]
    assert np.array_equal((fl & F_CRASHED) != 0, step["o_crashed"])
    assert np.array_equal((fl & F_FINISHED) != 0, step["o_finished"])
    assert np.array_equal((fl & F_HAS_CRASHED) != 0, step["o_has_crashed"])
    assert np.array_equal(st["finished_step"], step["o_finished_step"])
    assert np.array_equal(done, step["o_done"])
    assert np.array_equal(done_all, step["o_done_all"])
    assert np.array_equal(trunc, step["o_truncated"])
    assert np.array_equal(place, step["o_placement"])
    assert np.array_equal(st["steps"], step["o_steps"])
    assert np.array_equal(st["progress"], step["o_progress"])
    cp = np.stack([(fl & F_CP25) != 0, (fl & F_CP50) != 0, (fl & F_CP75) != 0], axis=2)
    assert np.array_equal(cp, step["o_cp"].astype(bool))
    if exact:
        for k in ("x", "y", "angle", "vx", "vy", "last_progress", "last_steering"):
            assert np.array_equal(st[k], step["o_" + k]), k
        assert np.array_equal(obs, step["o_obs"])
        assert np.array_equal(rew, step["o_reward"])
        assert np.array_equal(info[..., 0], step["o_info_speed"])
        assert np.array_equal(info[..., 1], step["o_info_progress"])
    else:
        np.testing.assert_allclose(obs, step["o_obs"], rtol=0, atol=1e-5)
        np.testing.assert_allclose(rew, step["o_reward"], rtol=0, atol=1e-5)


@pytest.mark.parametrize("dev", [False, True])
def test_multi_step(golden, oracle, oracle_dev, dev):
    orc = oracle_dev if dev else oracle
    step = golden["step_multi"]
    st = multi_state_from(step)
    out = orc.multi_step(golden.table(), st, step["action"], REL_MULTI)
    _check_multi(step, st, *out, exact=not dev)


def test_multi_reset(golden, oracle):
    step = golden["step_multi"]
    from oracle.orc import multi_state
    n = len(step["reset_track"])
    st = multi_state(n)
    st["track"][:] = step["reset_track"]
    obs = oracle.multi_reset(golden.table(), st, step["reset_order"].astype(np.uint8), REL_MULTI)
    assert np.array_equal(obs, step["reset_obs"])
    assert np.array_equal(st["x"], step["reset_x"]) and np.array_equal(st["y"], step["reset_y"])


def test_gae_bit_exact(golden, oracle):
    g = golden["gae"]
    for tag in ("a", "b", "c"):
        adv, ret = oracle.gae(g[f"{tag}_rewards"], g[f"{tag}_values"], g[f"{tag}_dones"], g[f"{tag}_next_value"],
                              g[f"{tag}_next_done"], float(g[f"{tag}_gamma"]), float(g[f"{tag}_lambda"]))
        assert np.array_equal(adv, g[f"{tag}_adv"]), tag
        assert np.array_equal(ret, g[f"{tag}_ret"]), tag


def test_device_sincos_is_correctly_rounded(oracle):
    import math
    rng = np.random.default_rng(3)
    x = rng.uniform(-2.0, 9.0, 2000)
    s, c = oracle.sincos_dev(x)
    try:
        import mpmath
    except ImportError:  # pragma: no cover
        pytest.skip("mpmath not importable")
    mpmath.mp.prec = 160
    for xi, si, ci in zip(x, s, c):
        assert float(mpmath.sin(mpmath.mpf(float(xi)))) == si
        assert float(mpmath.cos(mpmath.mpf(float(xi)))) == ci
    # and it agrees with glibc almost always (glibc is not CR: ~0.15% differ by 1 ulp)
    assert (s != np.sin(x)).mean() < 0.01 and (c != np.cos(x)).mean() < 0.01
    assert math.copysign(1.0, oracle.sincos_dev(np.array([-0.0]))[0][0]) == -1.0


def test_numpy_restatement_bit_exact(golden):
    """oracle/np_env.py (bench.py's cpu_baseline) reproduces the reference exactly."""
    from oracle.np_env import NpRacingEnv, make_track
    step = golden["step_single"]
    tracks = {}
    for i in range(0, len(step["x"]), 7):  # every 7th KAT (the full set is the C oracle's job)
        k = int(step["track"][i])
        if k not in tracks:
            tracks[k] = make_track(golden.tracks[k])
        e = NpRacingEnv(tracks[k], 11, float(step["speed_weight"][i]))
        e.x, e.y, e.angle, e.vx, e.vy = (float(step[c][i]) for c in ("x", "y", "angle", "vx", "vy"))
        e.progress, e.crashed, e.finished = float(step["progress"][i]), bool(step["crashed"][i]), bool(step["finished"][i])
        e.steps, e.last_progress, e.last_steering = int(step["steps"][i]), float(step["last_progress"][i]), float(step["last_steering"][i])
        e.cp = [bool(c) for c in step["cp"][i]]
        obs, r, term, trunc = e.step(step["action"][i])
        assert np.array_equal(obs, step["o_obs"][i]), i
        assert r == step["o_reward"][i] and term == step["o_terminated"][i] and trunc == step["o_truncated"][i], i
        assert (e.x, e.y, e.vx, e.vy) == tuple(step[c][i] for c in ("o_x", "o_y", "o_vx", "o_vy")), i
