"""Generate the golden vectors that pin the oracle (and through it the HIP path).

Runs ONLY in the build container, where the reference is mounted read-only at
/root/reference.  It imports the reference's own modules unmodified, with the
test-only gymnasium stand-in in ``_gym_stub/`` first on sys.path (gymnasium
1.2.3 is not installed).  No reference source is copied: the
outputs are data only (inputs and the reference's outputs), written as
compressed ``.npz`` files next to this script.

    python tests/golden/gen_golden.py            # all sets
    python tests/golden/gen_golden.py geometry   # one set

Sets:
  geometry.npz    G1  seed-1 train pool (16 tracks, widths), default Track(),
                      eval pool (seed 42) tracks 0..3 -- control points,
                      waypoints, normals, segment starts/v2, start pose,
                      max_track_distance; plus gen_tracks() RNG outputs.
  raycast.npz     G4  Track.raycast KATs (no-hit, uncapped >50, grazing).
  step_single.npz G2  state-injected RacingEnv.step KATs.
  traj_single.npz G3  reset + scripted-controller trajectories.
  step_multi.npz  G5  state-injected MultiRacingEnv.step KATs (+ reset order).
  gae.npz         G6  PPO.compute_advantages.
  agent.npz       G7  Agent init state_dict + forward on a fixed batch.
  ppo_update.npz  G8  PPO.ppo_update run unbound (full, obs-19, KL early stop).
  schedules.npz   A21 PPO.train / SelfPlayPPO.train per-update schedules
                      (lr, log_std, speed weight, snapshot pool, opponent
                      draws, checkpoint cadence).
  eval_metrics.npz (f)#3 utils/metrics.py:39-78 eval_single_agent on the
                      evaluate.py pool (seed 42, widths by run), driven by a
                      scripted agent; the actions it issued are recorded so
                      the device evaluator can replay them open loop.

Metadata (numpy/scipy/torch versions, libm behaviour notes, CPU model) is stored
in every file under ``meta_*`` keys.
"""
import os
import platform
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("RX_REFERENCE", "/root/reference")


def _import_reference():
    if not os.path.isdir(REF):
        raise SystemExit(f"reference not found at {REF}; golden vectors can only be regenerated in the build container")
    sys.path.insert(0, REF)
    sys.path.insert(0, os.path.join(HERE, "_gym_stub"))
    import environment.track as track  # noqa: E402
    import environment.car as car  # noqa: E402
    import environment.racing_env as racing_env  # noqa: E402
    import environment.multi_racing_env as multi_racing_env  # noqa: E402
    return track, car, racing_env, multi_racing_env


def _meta():
    import scipy
    cpu = platform.processor()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {
        "meta_numpy": np.array(np.__version__),
        "meta_scipy": np.array(scipy.__version__),
        "meta_python": np.array(platform.python_version()),
        "meta_cpu": np.array(cpu),
        "meta_glibc": np.array(" ".join(platform.libc_ver())),
        "meta_generator": np.array("tests/golden/gen_golden.py"),
    }


def _save(name, **arrays):
    arrays.update(_meta())
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    sz = os.path.getsize(path)
    print(f"wrote {path} ({sz / 1024:.1f} KiB)")


def _train_pool(track, n=16, seed=1):
    """train.py:67-80 sequence: seeds, gen_tracks, widths."""
    random.seed(seed)
    np.random.seed(seed)
    pool = track.gen_tracks(num_tracks=n, seed=seed)
    widths = [np.random.randint(6, 10) for _ in range(n)]
    return pool, widths


def _pack_ragged(arrs):
    lens = np.array([len(a) for a in arrs], dtype=np.int64)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    cat = np.concatenate([np.asarray(a, dtype=np.float64) for a in arrs], axis=0)
    return cat, off


def _track_record(T):
    st = T.get_start_pos()
    return dict(
        cp=np.asarray(T.control_points, dtype=np.float64),
        wp=np.asarray(T.waypoints, dtype=np.float64),
        nrm=np.asarray(T.normals, dtype=np.float64),
        starts=np.asarray(T.segment_cache["starts"], dtype=np.float64),
        v2=np.asarray(T.segment_cache["v2"], dtype=np.float64),
        start=np.array([float(st[0]), float(st[1]), float(st[2])]),
        maxd=float(T.max_track_distance),
        width=float(T.track_width),
    )


def _tracks_set(track):
    """The tracks every other set is built on: seed-1 pool (16), default, eval (seed 42) 0..3."""
    pool, widths = _train_pool(track, 16, 1)
    recs, labels = [], []
    for i in range(16):
        T = track.Track(track_pool=pool, track_id=i, track_width=widths[i])
        recs.append(_track_record(T))
        labels.append(f"pool1[{i}] w={widths[i]}")
    recs.append(_track_record(track.Track()))
    labels.append("default")
    np.random.seed(12345)  # evaluate.py does not seed the global RNG before gen_tracks(seed=42)
    eval_pool = track.gen_tracks(num_tracks=40, seed=42)
    eval_w = [np.random.RandomState(42 + i).randint(4, 10) for i in range(40)]
    for i in range(4):
        T = track.Track(track_pool=eval_pool, track_id=i, track_width=eval_w[i])
        recs.append(_track_record(T))
        labels.append(f"eval42[{i}] w={eval_w[i]}")
    return recs, labels, pool, widths, eval_pool, eval_w


def gen_geometry(track):
    recs, labels, pool, widths, eval_pool, eval_w = _tracks_set(track)
    out = {}
    for key in ("cp", "wp", "nrm", "starts", "v2"):
        cat, off = _pack_ragged([r[key] for r in recs])
        out[key] = cat
        out[key + "_off"] = off
    out["start"] = np.stack([r["start"] for r in recs])
    out["maxd"] = np.array([r["maxd"] for r in recs])
    out["width"] = np.array([r["width"] for r in recs])
    out["labels"] = np.array(labels)
    out["pool1_widths"] = np.array(widths, dtype=np.int64)
    out["eval42_widths"] = np.array(eval_w, dtype=np.int64)
    # gen_tracks RNG pins: a larger seed-1 pool (as train.py draws it) and the
    # global-RNG state that follows it (widths).
    pool64, widths64 = _train_pool(track, 64, 1)
    cat, off = _pack_ragged(pool64)
    out["pool1x64_cp"] = cat
    out["pool1x64_cp_off"] = off
    out["pool1x64_widths"] = np.array(widths64, dtype=np.int64)
    # unseeded-per-track generation (seed=None) after a global seed: all distinct
    np.random.seed(7)
    free = track.gen_tracks(num_tracks=8, seed=None)
    cat, off = _pack_ragged(free)
    out["free7x8_cp"] = cat
    out["free7x8_cp_off"] = off
    _save("geometry.npz", **out)
    return recs


def gen_raycast(track, recs_tracks):
    rng = np.random.default_rng(101)
    rows = []
    for ti in (0, 1, 16, 17):
        T = track.Track() if ti == DEFAULT_TRACK else track.Track(control_points=recs_tracks[ti]["cp"], track_width=recs_tracks[ti]["width"])
        wp, nrm, w = T.waypoints, T.normals, T.track_width
        W = len(wp)
        for k in range(600):
            kind = k % 6
            i = rng.integers(W)
            if kind == 0:       # inside the track
                o = wp[i] + nrm[i] * rng.uniform(-0.95 * w, 0.95 * w)
            elif kind == 1:     # near a wall
                o = wp[i] + nrm[i] * (w * rng.choice([-1, 1]) + rng.uniform(-0.3, 0.3))
            elif kind == 2:     # far outside -> often no hit
                o = rng.uniform(-300, 300, 2)
            elif kind == 3:     # centre of the loop (hits far away, > 50 uncapped)
                o = wp.mean(axis=0) + rng.uniform(-5, 5, 2)
            elif kind == 4:     # on a boundary vertex
                o = (wp[i] + nrm[i] * w) if rng.random() < 0.5 else (wp[i] - nrm[i] * w)
            else:               # anywhere near the track
                o = wp[i] + rng.uniform(-20, 20, 2)
            if kind == 4 and rng.random() < 0.5:
                # grazing: aim along the wall segment direction
                j = rng.integers(len(T.segment_cache["v2"]))
                v = T.segment_cache["v2"][j]
                d = float(np.arctan2(v[1], v[0]))
                o = T.segment_cache["starts"][j] - v * rng.uniform(0.5, 3.0)
            else:
                d = float(rng.uniform(-np.pi, 3 * np.pi))
            origin = np.array([float(o[0]), float(o[1])])
            t = T.raycast(origin, d, 50.0)
            rows.append((ti, origin[0], origin[1], d, float(t)))
    a = np.array(rows, dtype=np.float64)
    _save("raycast.npz", track=a[:, 0].astype(np.int64), ox=a[:, 1], oy=a[:, 2], dir=a[:, 3], t=a[:, 4])


def _sample_single_state(rng, T, W):
    """One injected RacingEnv state + action (SURVEY.md §8(c) G2 sampling)."""
    wp, nrm, w = T.waypoints, T.normals, T.track_width
    mode = rng.integers(8)
    if mode == 0:    # near the finish line, all checkpoints, last_progress > 0.9
        i = int(rng.integers(W - 12, W + 6)) % W
    else:
        i = int(rng.integers(W))
    lat = rng.uniform(-1.25 * w, 1.25 * w) if rng.random() < 0.7 else rng.uniform(-0.5 * w, 0.5 * w)
    pos = wp[i] + nrm[i] * lat
    tang = wp[(i + 1) % W] - wp[i]
    head = float(np.arctan2(tang[1], tang[0]))
    ang = head + rng.normal(0, 0.35) + (np.pi if rng.random() < 0.05 else 0.0)
    if rng.random() < 0.5:
        ang = ang % (2 * np.pi)
    spd = rng.choice([rng.uniform(0, 35), rng.uniform(28, 31), 30.0 * (1 + rng.normal(0, 1e-9))])
    vdir = ang + rng.normal(0, 0.2)
    vx, vy = spd * np.cos(vdir), spd * np.sin(vdir)
    prog_i = int(np.sum((wp - pos) ** 2, axis=1).argmin())
    if mode == 0:
        last_p = rng.choice([0.9 + rng.uniform(0.0005, 0.099), prog_i / W])
        cps = (True, True, True)
    else:
        last_p = rng.choice([prog_i / W, rng.uniform(0, 1), rng.choice([0.05, 0.95, 0.24, 0.26, 0.49, 0.51, 0.74, 0.76])])
        r = rng.integers(8)
        cps = (bool(r & 1), bool(r & 2), bool(r & 4))
    steps = int(rng.choice([rng.integers(0, 2990), 2998, 2999, 3000, 3005]))
    crashed = bool(rng.random() < 0.05)
    finished = bool(rng.random() < 0.03)
    last_steer = float(rng.uniform(-1, 1))
    act = np.array([rng.uniform(-1.6, 1.6), rng.uniform(-0.6, 1.6)], dtype=np.float32)
    if rng.random() < 0.3:
        act[0] = np.float32(rng.choice([-1.0, 1.0, 0.0]))
    if rng.random() < 0.3:
        act[1] = np.float32(rng.choice([0.0, 1.0]))
    return dict(x=float(pos[0]), y=float(pos[1]), angle=float(ang), vx=float(vx), vy=float(vy),
                progress=float(prog_i / W) if not crashed else float(rng.choice([prog_i / W, last_p])),
                crashed=crashed, finished=finished, steps=steps, last_progress=float(last_p),
                last_steering=last_steer, cp=cps, action=act)


def _inject_single(env, s):
    env.car.x, env.car.y, env.car.angle = s["x"], s["y"], s["angle"]
    env.car.vx, env.car.vy = s["vx"], s["vy"]
    env.car.progress, env.car.crashed, env.car.finished = s["progress"], s["crashed"], s["finished"]
    env.steps, env.last_progress, env.last_steering = s["steps"], s["last_progress"], s["last_steering"]
    env.checkpoints = {0.25: s["cp"][0], 0.50: s["cp"][1], 0.75: s["cp"][2]}


DEFAULT_TRACK = 16  # index of Track() (integer control points, width 6.0) in the track set


def _single_env(racing_env, recs_tracks, ti):
    if ti == DEFAULT_TRACK:
        return racing_env.RacingEnv(num_sensors=11)
    rec = recs_tracks[ti]
    return racing_env.RacingEnv(num_sensors=11, track_pool=[rec["cp"]], track_id=0, track_width=rec["width"])


def gen_step_single(track, racing_env, recs_tracks, per_track=700):
    rng = np.random.default_rng(202)
    cols = {k: [] for k in ("track", "x", "y", "angle", "vx", "vy", "progress", "crashed", "finished", "steps",
                            "last_progress", "last_steering", "cp", "action", "speed_weight",
                            "o_x", "o_y", "o_angle", "o_vx", "o_vy", "o_progress", "o_crashed", "o_finished",
                            "o_steps", "o_last_progress", "o_last_steering", "o_cp", "o_obs", "o_reward",
                            "o_terminated", "o_truncated", "o_info_speed", "o_info_progress", "o_progress_delta")}
    for ti in (0, 1, 2, 5, 16, 17, 18):
        env = _single_env(racing_env, recs_tracks, ti)
        env.reset(seed=0)
        W = len(env.track.waypoints)
        for k in range(per_track):
            s = _sample_single_state(rng, env.track, W)
            sw = 8.0 if rng.random() < 0.8 else float(rng.uniform(8.0, 14.0))
            env.speed_weight = sw
            _inject_single(env, s)
            obs, rew, term, trunc, info = env.step(s["action"])
            for key in ("x", "y", "angle", "vx", "vy", "progress", "crashed", "finished", "steps",
                        "last_progress", "last_steering", "action"):
                cols[key].append(s[key])
            cols["track"].append(ti)
            cols["cp"].append(s["cp"])
            cols["speed_weight"].append(sw)
            c = env.car
            cols["o_x"].append(float(c.x)); cols["o_y"].append(float(c.y)); cols["o_angle"].append(float(c.angle))
            cols["o_vx"].append(float(c.vx)); cols["o_vy"].append(float(c.vy)); cols["o_progress"].append(float(c.progress))
            cols["o_crashed"].append(bool(c.crashed)); cols["o_finished"].append(bool(c.finished))
            cols["o_steps"].append(env.steps); cols["o_last_progress"].append(float(env.last_progress))
            cols["o_last_steering"].append(float(env.last_steering))
            cols["o_cp"].append((env.checkpoints[0.25], env.checkpoints[0.50], env.checkpoints[0.75]))
            cols["o_obs"].append(obs); cols["o_reward"].append(float(rew))
            cols["o_terminated"].append(bool(term)); cols["o_truncated"].append(bool(trunc))
            cols["o_info_speed"].append(float(info["speed"])); cols["o_info_progress"].append(float(info["progress"]))
            cols["o_progress_delta"].append(float(info["progress_delta"]))
    out = {}
    for k, v in cols.items():
        a = np.array(v)
        if a.dtype == object:
            raise TypeError(k)
        out[k] = a
    out["cp"] = out["cp"].astype(np.uint8)
    out["o_cp"] = out["o_cp"].astype(np.uint8)
    print("step_single: crashes", int(out["o_crashed"].sum()), "finishes", int(out["o_finished"].sum()),
          "term", int(out["o_terminated"].sum()), "trunc", int(out["o_truncated"].sum()), "of", len(out["x"]))
    _save("step_single.npz", **out)


def _controller(env, rng, gain, speed_cap, noise):
    """Pure-pursuit driver so golden trajectories reach checkpoints and finishes."""
    c, T = env.car, env.track
    W = len(T.waypoints)
    i = T.closest_waypoint_idx(c.x, c.y)
    tgt = T.waypoints[(i + 8) % W]
    desired = np.arctan2(tgt[1] - c.y, tgt[0] - c.x)
    err = (desired - c.angle + np.pi) % (2 * np.pi) - np.pi
    steer = np.clip(gain * err + rng.normal(0, noise), -1.2, 1.2)
    spd = np.hypot(c.vx, c.vy)
    thr = 1.0 if spd < speed_cap else 0.0
    if rng.random() < 0.05:
        thr = rng.uniform(-0.2, 1.2)
    return np.array([steer, thr], dtype=np.float32)


def gen_traj_single(track, racing_env, recs_tracks):
    rng = np.random.default_rng(303)
    out = {"track": [], "start": [], "len": [], "actions": [], "obs": [], "reward": [], "terminated": [],
           "truncated": [], "x": [], "y": [], "angle": [], "vx": [], "vy": [], "progress": [], "reset_obs": []}
    off = [0]
    plans = [(0, 3.0, 18.0, 0.05), (1, 3.0, 22.0, 0.05), (2, 2.5, 14.0, 0.02), (16, 3.0, 20.0, 0.05),
             (17, 3.0, 16.0, 0.02), (5, 6.0, 30.0, 0.3), (18, 3.0, 12.0, 0.01), (0, 3.0, 12.0, 0.0)]
    for ti, gain, cap, noise in plans:
        env = _single_env(racing_env, recs_tracks, ti)
        obs0, _ = env.reset(seed=0)
        out["reset_obs"].append(obs0)
        n = 0
        for t in range(3100):
            a = _controller(env, rng, gain, cap, noise)
            obs, rew, term, trunc, info = env.step(a)
            c = env.car
            out["actions"].append(a); out["obs"].append(obs); out["reward"].append(float(rew))
            out["terminated"].append(bool(term)); out["truncated"].append(bool(trunc))
            out["x"].append(float(c.x)); out["y"].append(float(c.y)); out["angle"].append(float(c.angle))
            out["vx"].append(float(c.vx)); out["vy"].append(float(c.vy)); out["progress"].append(float(c.progress))
            n += 1
            if term or trunc:
                break
        out["track"].append(ti)
        off.append(off[-1] + n)
        print(f"traj track {ti}: {n} steps, finished={env.car.finished} crashed={env.car.crashed} trunc={trunc}")
    res = {k: np.array(v) for k, v in out.items() if k not in ("start", "len")}
    res["off"] = np.array(off, dtype=np.int64)
    _save("traj_single.npz", **res)


def gen_step_multi(track, multi_racing_env, recs_tracks, per_track=500):
    rng = np.random.default_rng(404)
    keys = ("track", "order", "x", "y", "angle", "vx", "vy", "progress", "crashed", "finished", "has_crashed",
            "finished_step", "last_progress", "last_steering", "cp", "steps", "action",
            "o_x", "o_y", "o_angle", "o_vx", "o_vy", "o_progress", "o_crashed", "o_finished", "o_has_crashed",
            "o_finished_step", "o_last_progress", "o_last_steering", "o_cp", "o_steps", "o_obs", "o_reward",
            "o_done", "o_done_all", "o_truncated", "o_placement", "o_info_speed", "o_info_progress")
    cols = {k: [] for k in keys}
    reset_rows = {"track": [], "order": [], "obs": [], "x": [], "y": [], "angle": []}
    for ti in (0, 1, 2, 16, 17):
        rec = recs_tracks[ti]
        if ti == DEFAULT_TRACK:
            env = multi_racing_env.MultiRacingEnv(num_agents=2, num_sensors=11)
        else:
            env = multi_racing_env.MultiRacingEnv(num_agents=2, num_sensors=11, track_pool=[rec["cp"]], track_id=0,
                                                  track_width=[rec["width"]])
        T = env.track
        W = len(T.waypoints)
        # reset KATs: both shuffle outcomes
        for first in (0, 1):
            seq = iter([[first, 1 - first]])
            orig = np.random.shuffle
            np.random.shuffle = lambda lst, _s=seq: lst.__setitem__(slice(None), next(_s))
            try:
                obs, _ = env.reset(seed=0)
            finally:
                np.random.shuffle = orig
            reset_rows["track"].append(ti); reset_rows["order"].append(first)
            reset_rows["obs"].append(np.stack([obs["0"], obs["1"]]))
            reset_rows["x"].append([c.x for c in env.cars]); reset_rows["y"].append([c.y for c in env.cars])
            reset_rows["angle"].append([c.angle for c in env.cars])
        for k in range(per_track):
            env.reset(seed=0)
            ss = [_sample_single_state(rng, T, W) for _ in range(2)]
            if rng.random() < 0.5:   # put the second car close to the first: contact / car rays
                base = ss[0]
                ang = base["angle"]
                d = rng.uniform(1.0, 6.0)
                off_a = ang + rng.uniform(-np.pi, np.pi)
                ss[1]["x"] = base["x"] + d * np.cos(off_a)
                ss[1]["y"] = base["y"] + d * np.sin(off_a)
                ss[1]["angle"] = ang + rng.normal(0, 0.6)
            steps = int(rng.choice([rng.integers(0, 2990), 2999, 3000]))
            for i, (c, s) in enumerate(zip(env.cars, ss)):
                c.x, c.y, c.angle, c.vx, c.vy = s["x"], s["y"], s["angle"], s["vx"], s["vy"]
                c.progress, c.crashed, c.finished = s["progress"], s["crashed"], s["finished"]
                d = env.agents_data[i]
                d["last_progress"], d["last_steering"] = s["last_progress"], s["last_steering"]
                d["checkpoints"] = {0.25: s["cp"][0], 0.50: s["cp"][1], 0.75: s["cp"][2]}
                d["has_crashed"] = bool(s["crashed"] and rng.random() < 0.7)
                d["finished_step"] = (int(rng.integers(100, 2900)) if (s["finished"] and rng.random() < 0.8) else None)
            env.steps = steps
            acts = {f"{i}": np.array([rng.uniform(-1.5, 1.5), rng.uniform(-1.5, 1.5)], dtype=np.float32) for i in range(2)}
            pre = [dict(d) for d in env.agents_data]
            obs, rew, dones, trunc, infos = env.step(acts)
            cols["track"].append(ti); cols["order"].append(-1)
            for key in ("x", "y", "angle", "vx", "vy", "progress", "crashed", "finished", "last_progress", "last_steering"):
                cols[key].append([s[key] for s in ss])
            cols["has_crashed"].append([p["has_crashed"] for p in pre])
            cols["finished_step"].append([(-1 if p["finished_step"] is None else p["finished_step"]) for p in pre])
            cols["cp"].append([s["cp"] for s in ss])
            cols["steps"].append(steps)
            cols["action"].append(np.stack([acts["0"], acts["1"]]))
            cs = env.cars
            cols["o_x"].append([float(c.x) for c in cs]); cols["o_y"].append([float(c.y) for c in cs])
            cols["o_angle"].append([float(c.angle) for c in cs]); cols["o_vx"].append([float(c.vx) for c in cs])
            cols["o_vy"].append([float(c.vy) for c in cs]); cols["o_progress"].append([float(c.progress) for c in cs])
            cols["o_crashed"].append([bool(c.crashed) for c in cs]); cols["o_finished"].append([bool(c.finished) for c in cs])
            ad = env.agents_data
            cols["o_has_crashed"].append([bool(d["has_crashed"]) for d in ad])
            cols["o_finished_step"].append([(-1 if d["finished_step"] is None else d["finished_step"]) for d in ad])
            cols["o_last_progress"].append([float(d["last_progress"]) for d in ad])
            cols["o_last_steering"].append([float(d["last_steering"]) for d in ad])
            cols["o_cp"].append([(d["checkpoints"][0.25], d["checkpoints"][0.50], d["checkpoints"][0.75]) for d in ad])
            cols["o_steps"].append(env.steps)
            cols["o_obs"].append(np.stack([obs["0"], obs["1"]]))
            cols["o_reward"].append([float(rew["0"]), float(rew["1"])])
            cols["o_done"].append(bool(dones["0"])); cols["o_done_all"].append(bool(dones["__all__"]))
            cols["o_truncated"].append(bool(trunc))
            cols["o_placement"].append([int(infos[f"{i}"].get("placement", 0)) for i in range(2)])
            cols["o_info_speed"].append([float(infos[f"{i}"]["speed"]) for i in range(2)])
            cols["o_info_progress"].append([float(infos[f"{i}"]["progress"]) for i in range(2)])
    out = {k: np.array(v) for k, v in cols.items()}
    out["cp"] = out["cp"].astype(np.uint8)
    out["o_cp"] = out["o_cp"].astype(np.uint8)
    for k, v in reset_rows.items():
        out["reset_" + k] = np.array(v)
    print("step_multi: contacts/crash/finish/done:", int((out["o_reward"] < -4).sum()), int(out["o_crashed"].sum()),
          int(out["o_finished"].sum()), int(out["o_done_all"].sum()))
    _save("step_multi.npz", **out)


def gen_gae():
    sys.path.insert(0, REF)
    import torch
    from agent.ppo import PPO

    class _Self:
        pass

    out = {}
    for tag, (T, N, gamma, lam) in {"a": (2048, 16, 0.99, 0.95), "b": (256, 64, 0.99, 0.97), "c": (64, 512, 0.99, 0.95)}.items():
        g = torch.Generator().manual_seed(T * 7 + N)
        rewards = (torch.randn(T, N, generator=g) * 10).float()
        values = (torch.randn(T, N, generator=g) * 30).float()
        dones = (torch.rand(T, N, generator=g) < 0.03).float()
        next_value = (torch.randn(N, generator=g) * 30).float()
        next_done = torch.rand(N, generator=g) < 0.05
        s = _Self()
        s.config = {"num_steps": T, "gamma": gamma, "gae_lambda": lam}
        s.device = torch.device("cpu")
        adv, ret = PPO.compute_advantages(s, rewards, dones, values, next_value, next_done)
        for k, v in dict(rewards=rewards, values=values, dones=dones, next_value=next_value,
                         next_done=next_done, adv=adv, ret=ret).items():
            out[f"{tag}_{k}"] = v.numpy()
        out[f"{tag}_gamma"] = np.array(gamma)
        out[f"{tag}_lambda"] = np.array(lam)
    out["meta_torch"] = np.array(torch.__version__)
    _save("gae.npz", **out)


def gen_agent():
    sys.path.insert(0, REF)
    import torch
    from agent.ppo import Agent
    from gymnasium import spaces
    out = {}
    for obs_dim in (15, 19):
        torch.manual_seed(1)
        ag = Agent(spaces.Box(-1.0, 1.0, shape=(obs_dim,), dtype=np.float32),
                   spaces.Box(np.array([-1.0, 0.0]), np.array([1.0, 1.0]), shape=(2,), dtype=np.float32))
        ag.log_std.fill_(-0.5)
        g = torch.Generator().manual_seed(obs_dim)
        obs = (torch.rand(64, obs_dim, generator=g) * 2 - 1).float()
        act = (torch.rand(64, 2, generator=g) * 2.4 - 1.2).clamp(-1, 1).float()
        with torch.no_grad():
            _, logp, ent, val = ag.get_action_and_value(obs, act)
            mu = ag.actor_mu(obs)
        for k, v in ag.state_dict().items():
            out[f"d{obs_dim}_sd_{k}"] = v.numpy()
        out[f"d{obs_dim}_obs"] = obs.numpy(); out[f"d{obs_dim}_act"] = act.numpy()
        out[f"d{obs_dim}_mu"] = mu.numpy(); out[f"d{obs_dim}_logp"] = logp.numpy()
        out[f"d{obs_dim}_ent"] = ent.numpy(); out[f"d{obs_dim}_val"] = val.numpy()
    out["meta_torch"] = np.array(torch.__version__)
    _save("agent.npz", **out)


def _np_state(prefix, out):
    st = np.random.get_state()
    out[prefix + "_keys"] = np.asarray(st[1], dtype=np.uint32)
    out[prefix + "_pos"] = np.array(st[2], dtype=np.int64)


def _ppo_cfg(**over):
    c = {"learning_rate": 3e-4, "gamma": 0.99, "gae_lambda": 0.95, "clip_coef": 0.2, "ent_coef": 0.01,
         "vf_coef": 0.5, "update_epochs": 2, "num_minibatches": 4, "max_grad_norm": 0.5, "kl_target": 0.015}
    c.update(over)
    c["batch_size"] = c["num_steps"] * c["num_envs"]
    c["minibatch_size"] = c["batch_size"] // c["num_minibatches"]
    return c


def _ppo_batch(torch, Agent, spaces, obs_dim, T, N, seed, log_std, adv_scale):
    """A realistic rollout batch: actions sampled from the policy itself (some
    clamped to the box edge, agent/ppo.py:44-53 Q7), its own log-probs and
    values, random advantages, returns = advantages + values."""
    torch.manual_seed(seed)
    ag = Agent(spaces.Box(-1.0, 1.0, shape=(obs_dim,), dtype=np.float32),
               spaces.Box(np.array([-1.0, 0.0]), np.array([1.0, 1.0]), shape=(2,), dtype=np.float32))
    ag.log_std.fill_(log_std)
    g = torch.Generator().manual_seed(seed + 1)
    obs = (torch.rand(T, N, obs_dim, generator=g) * 2 - 1).float()
    with torch.no_grad():
        act, logp, _, val = ag.get_action_and_value(obs.reshape(-1, obs_dim))
    act = act.reshape(T, N, 2)
    logp = logp.reshape(T, N)
    val = val.reshape(T, N)
    adv = (torch.randn(T, N, generator=g) * adv_scale + 0.2).float()
    ret = adv + val
    return ag, dict(obs=obs, actions=act, logprobs=logp, values=val, advantages=adv, returns=ret)


def gen_ppo_update(big=False):
    """G8: PPO.ppo_update (agent/ppo.py:156-209) run unbound on CPU torch.

    Cases: 'full' (2 epochs x 4 minibatches, no KL stop, obs 15), 'd19' (obs
    19, 3 x 2, larger lr), 'stop' (KL early stop inside epoch 2, at a
    minibatch chosen from the KLs the unstopped run sees) -> ppo_update.npz;
    with ``big``: 'mb32k' (configs[1]'s minibatch size: 4,096 envs x 8 steps
    in ONE 32,768-row minibatch, 2 epochs) -> ppo_update_mb32k.npz.  Recorded: the
    initial state_dict and batch, np.random state before/after, every
    optimizer step's gradient as Adam sees it (flat, parameter order,
    after clip_grad_norm_; the first two steps), the
    post-update parameters and Adam state, the number of optimizer steps,
    the KL per minibatch and the stop point."""
    sys.path.insert(0, REF)
    import contextlib
    import io
    import torch
    from torch import optim
    from agent.ppo import Agent, PPO
    from gymnasium import spaces

    class _Self:
        pass

    def run(ag0, batch, cfg, np_seed, record_kl=False):
        ag = Agent(spaces.Box(-1.0, 1.0, shape=(batch["obs"].shape[-1],), dtype=np.float32),
                   spaces.Box(np.array([-1.0, 0.0]), np.array([1.0, 1.0]), shape=(2,), dtype=np.float32))
        ag.load_state_dict(ag0.state_dict())
        opt = optim.Adam(ag.parameters(), lr=cfg["learning_rate"], eps=1e-5)
        grads, kls = [], []
        orig_step = opt.step

        def step(*a, **k):
            grads.append(torch.cat([p.grad.reshape(-1) for p in ag.parameters()]).clone())
            return orig_step(*a, **k)
        opt.step = step
        if record_kl:  # the KL the reference tests at each minibatch (agent/ppo.py:178-180)
            orig_gav = ag.get_action_and_value
            b_lp = batch["logprobs"].reshape(-1)
            inds_seen = []

            def gav(x, action=None):
                r = orig_gav(x, action)
                inds_seen.append(r[1].detach().clone())
                return r
            ag.get_action_and_value = gav
        s = _Self()
        s.config, s.agent, s.optimizer, s.device = cfg, ag, opt, torch.device("cpu")
        np.random.seed(np_seed)
        st0 = {}
        _np_state("rng_before", st0)
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            PPO.ppo_update(s, batch["advantages"], batch["returns"], batch["values"], batch["logprobs"],
                           batch["actions"], batch["obs"])
        st1 = {}
        _np_state("rng_after", st1)
        if record_kl:
            # replay the shuffles from the same seed to recover mb_inds
            rs = np.random.RandomState(np_seed)
            b_inds = np.arange(cfg["batch_size"])
            k = 0
            for _ in range(cfg["update_epochs"]):
                rs.shuffle(b_inds)
                for s0 in range(0, cfg["batch_size"], cfg["minibatch_size"]):
                    if k >= len(inds_seen):
                        break
                    mb = b_inds[s0:s0 + cfg["minibatch_size"]]
                    kls.append(float((b_lp[mb] - inds_seen[k]).mean()))
                    k += 1
        return ag, opt, grads, kls, st0, st1, buf.getvalue()

    out = {}
    cases = {
        "mb32k": dict(obs_dim=15, T=8, N=4096, seed=14, log_std=-0.7, adv_scale=4.0, np_seed=8,
                      cfg=dict(num_steps=8, num_envs=4096, update_epochs=2, num_minibatches=1, kl_target=1e9)),
    } if big else {
        "full": dict(obs_dim=15, T=64, N=16, seed=11, log_std=-0.5, adv_scale=3.0, np_seed=5,
                     cfg=dict(num_steps=64, num_envs=16, update_epochs=2, num_minibatches=4, kl_target=1e9)),
        "d19": dict(obs_dim=19, T=32, N=16, seed=12, log_std=-0.9, adv_scale=8.0, np_seed=6,
                    cfg=dict(num_steps=32, num_envs=16, update_epochs=3, num_minibatches=2, kl_target=1e9,
                             learning_rate=1e-3, ent_coef=0.02, gae_lambda=0.97)),
        "stop": dict(obs_dim=15, T=64, N=16, seed=13, log_std=-1.2, adv_scale=5.0, np_seed=7,
                     cfg=dict(num_steps=64, num_envs=16, update_epochs=3, num_minibatches=4, kl_target=None,
                              learning_rate=3e-3)),
    }
    for tag, cs in cases.items():
        ag0, batch = _ppo_batch(torch, Agent, spaces, cs["obs_dim"], cs["T"], cs["N"], cs["seed"], cs["log_std"],
                                cs["adv_scale"])
        cfg = dict(cs["cfg"])
        kl_stop_at = -1
        if cfg["kl_target"] is None:
            # KLs of an unstopped run; the target sits just below the first KL of
            # epoch 2 that exceeds every earlier one -> the update returns there
            probe = _ppo_cfg(**dict(cfg, kl_target=1e9))
            _, _, _, kls, _, _, _ = run(ag0, batch, probe, cs["np_seed"], record_kl=True)
            per_epoch = probe["num_minibatches"]
            j = next(k for k in range(per_epoch + 1, len(kls)) if kls[k] > max(kls[:k]))
            cfg["kl_target"] = 0.5 * (kls[j] + max(kls[:j]))
            kl_stop_at = j
        c = _ppo_cfg(**cfg)
        ag, opt, grads, kls, st0, st1, text = run(ag0, batch, c, cs["np_seed"], record_kl=True)
        if kl_stop_at >= 0:
            assert len(grads) == kl_stop_at and "Early stopping" in text, (len(grads), kl_stop_at, text)
        for k, v in ag0.state_dict().items():
            out[f"{tag}_sd0_{k}"] = v.numpy()
        for k, v in batch.items():
            out[f"{tag}_{k}"] = v.numpy()
        for k, v in ag.state_dict().items():
            out[f"{tag}_sd1_{k}"] = v.numpy()
        st = opt.state_dict()["state"]
        out[f"{tag}_adam_exp_avg"] = torch.cat([st[i]["exp_avg"].reshape(-1) for i in sorted(st)]).numpy()
        out[f"{tag}_adam_exp_avg_sq"] = torch.cat([st[i]["exp_avg_sq"].reshape(-1) for i in sorted(st)]).numpy()
        out[f"{tag}_adam_step"] = np.array([float(st[i]["step"]) for i in sorted(st)])
        out[f"{tag}_grads"] = torch.stack(grads[:2]).numpy()  # first two optimizer steps
        out[f"{tag}_n_steps"] = np.array(len(grads))
        out[f"{tag}_kls"] = np.array(kls)
        out[f"{tag}_kl_stop_at"] = np.array(kl_stop_at)
        out[f"{tag}_np_seed"] = np.array(cs["np_seed"])
        for k, v in c.items():
            out[f"{tag}_cfg_{k}"] = np.array(v)
        for d in (st0, st1):
            for k, v in d.items():
                out[f"{tag}_{k}"] = v
        print(f"ppo_update {tag}: {len(grads)} optimizer steps, stop_at={kl_stop_at}, kl_target={c['kl_target']:.6g}")
    out["meta_torch"] = np.array(torch.__version__)
    _save("ppo_update_mb32k.npz" if big else "ppo_update.npz", **out)


def gen_schedules():
    """A21: the per-update schedules of PPO.train (agent/ppo.py:235-258) and
    SelfPlayPPO.train (agent/self_play_ppo.py:113-139, 154-167), recorded by
    running the reference's own train loops with the rollout / advantage /
    update phases replaced by recorders (no envs exist here).  Recorded per
    update: lr, log_std, the speed_weight the loop setattr's on envs.envs[i];
    self-play: pool membership after the snapshot step (ids = the update a
    snapshot was taken at), the opponent np.random.choice draws, the updates
    that write a checkpoint."""
    sys.path.insert(0, REF)
    import tempfile
    import contextlib
    import io
    import types
    import torch
    from torch import optim
    from agent.ppo import Agent, PPO
    from agent.self_play_ppo import SelfPlayPPO
    from gymnasium import spaces

    out = {}
    obs_sp = spaces.Box(-1.0, 1.0, shape=(15,), dtype=np.float32)
    act_sp = spaces.Box(np.array([-1.0, 0.0]), np.array([1.0, 1.0]), shape=(2,), dtype=np.float32)

    def stub(cfg, sp_obs):
        s = types.SimpleNamespace()
        s.config, s.device = cfg, torch.device("cpu")
        N, D = cfg["num_envs"], sp_obs.shape[0]
        s.envs = types.SimpleNamespace(single_observation_space=sp_obs, single_action_space=act_sp,
                                       envs=[types.SimpleNamespace() for _ in range(N)],
                                       reset=lambda: (np.zeros((N, D), np.float32), {}), close=lambda: None)
        torch.manual_seed(cfg["seed"])
        s.agent = Agent(sp_obs, act_sp)
        s.optimizer = optim.Adam(s.agent.parameters(), lr=cfg["learning_rate"], eps=1e-5)
        s.rec = {"lr": [], "log_std": [], "speed_weight": [], "opponent": [], "pool": []}
        s.update_idx = [0]

        def collect(*bufs):
            s.rec["lr"].append(s.optimizer.param_groups[0]["lr"])
            s.rec["log_std"].append(s.agent.log_std.detach().clone().numpy())
            s.rec["speed_weight"].append(getattr(s.envs.envs[0], "speed_weight", np.nan))
            return bufs + ([],)
        s.collect_rollout = collect
        s.compute_advantages = lambda r, d, v, nv, nd: (r, r)

        def upd(*a):  # tag the weights with the update index: snapshots become identifiable
            with torch.no_grad():
                s.agent.critic[4].bias.fill_(float(s.update_idx[0]))
            s.update_idx[0] += 1
        s.ppo_update = upd
        return s

    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp:
        os.chdir(tmp)
        os.makedirs("models")  # SelfPlayPPO.train torch.save's checkpoints there unguarded
        try:
            # single-agent: base_config values, 37 updates
            cfg = _ppo_cfg(num_steps=4, num_envs=2, update_epochs=10, num_minibatches=2)
            cfg.update(seed=1, total_timesteps=8 * 37 + 5)
            s = stub(cfg, obs_sp)
            with contextlib.redirect_stdout(io.StringIO()):
                PPO.train(s)
            out["single_num_updates"] = np.array(len(s.rec["lr"]))
            out["single_lr"] = np.array(s.rec["lr"])
            out["single_log_std"] = np.stack(s.rec["log_std"])
            out["single_speed_weight"] = np.array(s.rec["speed_weight"])
            out["single_learning_rate"] = np.array(cfg["learning_rate"])
            # self-play: self_play_config values, 64 updates (snapshots at 15, 30, 45, 60)
            cfg = _ppo_cfg(num_steps=4, num_envs=2, update_epochs=10, num_minibatches=2, learning_rate=3e-4,
                           gae_lambda=0.97, ent_coef=0.02)
            cfg.update(seed=1, total_timesteps=8 * 64, snapshot_freq=15, pool_size=3)
            sp_obs = spaces.Box(-1.0, 1.0, shape=(19,), dtype=np.float32)
            s = stub(cfg, sp_obs)
            s.opponent_pool, s.curr_opponent = [], None
            s.snapshot_freq, s.pool_size = cfg["snapshot_freq"], cfg["pool_size"]
            s.snapshot_agent = lambda: SelfPlayPPO.snapshot_agent(s)
            s.select_opponent = lambda: SelfPlayPPO.select_opponent(s)

            def update_opponent():  # agent/self_play_ppo.py:46-50 minus the env rebuild
                s.curr_opponent = s.select_opponent()
                s.rec["opponent"].append(-1 if s.curr_opponent is None else int(s.curr_opponent.critic[4].bias.item()))
                s.rec["pool"].append([int(o.critic[4].bias.item()) for o in s.opponent_pool]
                                     + [-2] * (cfg["pool_size"] - len(s.opponent_pool)))
            s.update_opponent = update_opponent
            np.random.seed(1)
            with contextlib.redirect_stdout(io.StringIO()):
                SelfPlayPPO.train(s)
            out["selfplay_num_updates"] = np.array(len(s.rec["lr"]))
            out["selfplay_lr"] = np.array(s.rec["lr"])
            out["selfplay_log_std"] = np.stack(s.rec["log_std"])
            out["selfplay_opponent"] = np.array(s.rec["opponent"], dtype=np.int64)
            out["selfplay_pool"] = np.array(s.rec["pool"], dtype=np.int64)
            out["selfplay_np_seed"] = np.array(1)
            out["selfplay_snapshot_freq"] = np.array(cfg["snapshot_freq"])
            out["selfplay_pool_size"] = np.array(cfg["pool_size"])
            out["selfplay_checkpoints"] = np.array(sorted(int(f.split("_")[-1].split(".")[0])
                                                          for f in os.listdir("models")), dtype=np.int64)
        finally:
            os.chdir(cwd)
    out["meta_torch"] = np.array(torch.__version__)
    _save("schedules.npz", **out)


def gen_eval_metrics(track, racing_env):
    """(f)#3: the reference's per-episode evaluation metrics.  Episodes follow
    rx.evaluate.eval_pool(4, 2): np.random.seed(0), gen_tracks(4, seed=42),
    run r uses width RandomState(42 + r).randint(4, 10) (evaluate.py:26-31
    indexes widths by run).  The agent is a scripted pure-pursuit driver
    (varied gains / caps / noise so episodes finish, crash and time out)."""
    import torch
    sys.path.insert(0, REF)
    from utils.metrics import eval_single_agent
    np.random.seed(0)
    pool = track.gen_tracks(num_tracks=4, seed=42)
    widths = [np.random.RandomState(42 + i).randint(4, 10) for i in range(4)]
    plans = {(0, 0): (3.0, 18.0, 0.05), (0, 1): (3.0, 22.0, 0.05), (1, 0): (2.5, 14.0, 0.02),
             (1, 1): (12.0, 40.0, 0.6), (2, 0): (3.0, 16.0, 0.02), (2, 1): (3.0, 2.5, 0.0),
             (3, 0): (3.0, 12.0, 0.01), (3, 1): (0.0, 2.0, 0.0)}
    rng = np.random.default_rng(909)
    keys = ("total_reward", "steps", "progress", "finished", "crashed", "speed", "total_distance", "distance_per_step")
    out = {k: [] for k in keys}
    acts, off = [], [0]

    class Scripted:
        def __init__(self, env, plan):
            self.env, self.plan, self.log = env, plan, []

        def get_action_and_value(self, obs_tensor):
            a = _controller(self.env, rng, *self.plan)
            self.log.append(a)
            return torch.from_numpy(a[None]), None, None, None

    for t in range(4):
        for r in range(2):
            env = racing_env.RacingEnv(num_sensors=11, track_pool=pool, track_id=t, track_width=widths[r])
            agent = Scripted(env, plans[(t, r)])
            m = eval_single_agent(env, agent, "cpu", max_steps=2000)
            for k in keys:
                out[k].append(m[k])
            acts.extend(agent.log)
            off.append(len(acts))
            print(f"eval track {t} run {r}: steps {m['steps']} finished {m['finished']} crashed {m['crashed']}")
    res = {k: np.array(v, dtype=np.float64 if k not in ("steps", "finished", "crashed") else
                       (np.int64 if k == "steps" else np.uint8)) for k, v in out.items()}
    res["actions"] = np.array(acts, dtype=np.float32)
    res["off"] = np.array(off, dtype=np.int64)
    res["widths"] = np.array(widths, dtype=np.int64)
    _save("eval_metrics.npz", **res)


def main(argv):
    want = set(argv[1:]) or {"geometry", "raycast", "step_single", "traj_single", "step_multi", "gae", "agent",
                             "ppo_update", "ppo_update_mb32k", "schedules", "eval_metrics"}
    if want <= {"ppo_update", "ppo_update_mb32k", "schedules"}:
        sys.path.insert(0, os.path.join(HERE, "_gym_stub"))
        if "ppo_update" in want:
            gen_ppo_update()
        if "ppo_update_mb32k" in want:
            gen_ppo_update(big=True)
        if "schedules" in want:
            gen_schedules()
        return
    track, car, racing_env, multi_racing_env = _import_reference()
    recs = None
    if want & {"geometry", "raycast", "step_single", "traj_single", "step_multi"}:
        recs = gen_geometry(track) if "geometry" in want else _tracks_set(track)[0]
    if "raycast" in want:
        gen_raycast(track, recs)
    if "step_single" in want:
        gen_step_single(track, racing_env, recs)
    if "traj_single" in want:
        gen_traj_single(track, racing_env, recs)
    if "step_multi" in want:
        gen_step_multi(track, multi_racing_env, recs)
    if "gae" in want:
        gen_gae()
    if "agent" in want:
        gen_agent()
    if "ppo_update" in want:
        gen_ppo_update()
    if "ppo_update_mb32k" in want:
        gen_ppo_update(big=True)
    if "schedules" in want:
        gen_schedules()
    if "eval_metrics" in want:
        gen_eval_metrics(track, racing_env)


if __name__ == "__main__":
    main(sys.argv)
