"""bench.py's cpu_baseline leg, Mode B workers -- BASELINE INFRASTRUCTURE ONLY.

Each worker is a fresh ``python -m oracle.cpu_baseline`` child process that
imports numpy / scipy and this repository's oracle/np_env.py restatement, and
nothing else: no torch, no HIP runtime.  (Round 3 ran them as a
multiprocessing "spawn" pool, whose workers re-imported bench.py -- and with
it torch -- and were then SIGTERM-ed by Pool.__exit__: 16 "Aborted" dumps per
run.)  A worker steps ONE env (SyncVectorEnv of 1, the reference's plumbing,
agent/ppo.py:70 + environment/racing_env.py:104-167 restated) with uniform
random actions for a time budget, prints one JSON line {"steps", "seconds"} and
exits 0.

Only bench.py's cpu_baseline leg (and tests/) use this module.
"""
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def np_envs(pool, widths, n_envs, first=0):
    """NpRacingEnv objects over the reference geometry (rx.track.TrackGeometry ==
    environment/track.py:61-148, bit-exact), one geometry per (control points, width)."""
    from oracle.np_env import NpRacingEnv, NpTrack
    from rx.track import TrackGeometry
    envs, geo = [], {}
    for i in range(first, first + n_envs):
        key = (id(pool[i]), widths[i])
        if key not in geo:
            g = TrackGeometry(pool[i], widths[i])
            geo[key] = NpTrack(g.waypoints, g.normals, g.segment_cache["starts"], g.segment_cache["v2"],
                               g.track_width, g.get_start_pos())
        envs.append(NpRacingEnv(geo[key], 11))
    return envs


def worker(cp, width, budget_s, seed):
    """Mode B worker body: ONE env on one core, random actions, bounded time."""
    from oracle.np_env import NpSyncVectorEnv
    venv = NpSyncVectorEnv(np_envs([cp], [width], 1))
    venv.reset()
    rng = np.random.default_rng(seed)
    steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        venv.step(np.array([[rng.uniform(-1, 1), rng.uniform(0, 1)]], dtype=np.float32))
        steps += 1
    return steps, time.perf_counter() - t0


def run_workers(jobs, timeout_s):
    """Start one child per job [(control points, width, budget_s, seed)], all at
    once, and collect their (steps, seconds).  Children run with
    OPENBLAS_NUM_THREADS=1; a failing child raises (its stderr is kept)."""
    env = dict(os.environ, OPENBLAS_NUM_THREADS="1", OMP_NUM_THREADS="1")
    env["PYTHONPATH"] = os.pathsep.join([ROOT, os.path.join(ROOT, "self-play-racing_amd"),
                                         env.get("PYTHONPATH", "")]).rstrip(os.pathsep)
    # stdout / stderr go to temporary files, not pipes: a child that writes more than a
    # pipe buffer (repeated warnings) cannot block against the parent, and every wait
    # below has a real deadline
    procs = []
    deadline = time.monotonic() + timeout_s
    try:
        for cp, width, budget, seed in jobs:
            arg = json.dumps({"cp": np.asarray(cp, dtype=np.float64).tolist(), "width": float(width),
                              "budget_s": float(budget), "seed": int(seed)})
            fo, fe = tempfile.TemporaryFile("w+"), tempfile.TemporaryFile("w+")
            p = subprocess.Popen([sys.executable, "-m", "oracle.cpu_baseline"], cwd=ROOT, env=env,
                                 stdin=subprocess.PIPE, stdout=fo, stderr=fe, text=True)
            procs.append((p, fo, fe))
            p.stdin.write(arg)
            p.stdin.close()
        out = []
        for p, fo, fe in procs:
            try:
                rc = p.wait(timeout=max(0.1, deadline - time.monotonic()))
            except subprocess.TimeoutExpired:
                raise RuntimeError(f"cpu_baseline worker still running after {timeout_s} s") from None
            fo.seek(0)
            fe.seek(0)
            o, e = fo.read(), fe.read()
            if rc != 0:
                raise RuntimeError(f"cpu_baseline worker exited with {rc}: {e[-2000:]}")
            r = json.loads(o.strip().splitlines()[-1])
            out.append((int(r["steps"]), float(r["seconds"])))
    finally:
        for p, fo, fe in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
            fo.close()
            fe.close()
    return out


def _main():
    a = json.loads(sys.stdin.read())
    cp = np.asarray(a["cp"], dtype=np.float64)
    # widths are Python ints in train.py's pool (np.random.randint): keep an integral width integral
    w = a["width"]
    w = int(w) if float(w).is_integer() else w
    steps, sec = worker(cp, w, a["budget_s"], a["seed"])
    print(json.dumps({"steps": steps, "seconds": sec, "torch_loaded": "torch" in sys.modules}), flush=True)


if __name__ == "__main__":
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    pkg = os.path.join(ROOT, "self-play-racing_amd")
    if pkg not in sys.path:
        sys.path.insert(0, pkg)
    _main()
