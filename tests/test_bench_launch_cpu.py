"""bench.py's own N-rank launcher, on CPU.

`python bench.py --gpus N` with no WORLD_SIZE in the environment must start the
N ranks itself (fresh child processes, rendezvous on 127.0.0.1) -- the form the
driver's SCALE run uses -- and relay exactly one JSON line from rank 0.
--launch-selftest stops each rank after the process-group plumbing (gloo), so
this runs without a GPU.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, timeout=240):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + list(args), cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_bench_self_launches_two_ranks_without_torchrun():
    r = _run("--gpus", "2", "--dist-backend", "gloo", "--launch-selftest", "--steps", "3", "--warmup", "1")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout  # rank 0 only, one line
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 3 and out["warmup"] == 1
    d = out["dist"]
    assert d["backend"] == "gloo" and d["world_size"] == 2
    assert [i["rank"] for i in d["ranks"]] == [0, 1]
    assert [i["local_rank"] for i in d["ranks"]] == [0, 1]
    assert out["max_over_ranks"] == 2.0  # the MAX all-reduce the timed region uses


def test_bench_launcher_propagates_a_rank_failure():
    # an unknown backend makes every rank fail at init_process_group: the parent must
    # return non-zero (and not hang waiting for the survivors)
    r = _run("--gpus", "2", "--dist-backend", "no-such-backend", "--launch-selftest", timeout=120)
    assert r.returncode != 0
    assert r.stdout.strip() == ""


def test_bench_rejects_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-selftest"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_cpu_baseline_workers_are_torch_free_and_exit_cleanly():
    """bench.py's Mode B CPU-baseline workers (oracle/cpu_baseline.py, VERDICT r03
    #6): fresh child processes that never import torch (so no HIP runtime and no
    torch signal handlers), exit 0 on their own, and step the oracle env."""
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))
    from rx.track import gen_tracks
    from oracle.cpu_baseline import run_workers
    import numpy as np
    np.random.seed(1)
    pool = gen_tracks(2, seed=1)
    res = run_workers([(pool[0], 7, 0.3, 0), (pool[1], 8, 0.3, 1)], timeout_s=120)
    assert len(res) == 2 and all(s > 0 and sec >= 0.3 for s, sec in res)
    arg = json.dumps({"cp": np.asarray(pool[0]).tolist(), "width": 6, "budget_s": 0.1, "seed": 0})
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([ROOT, os.path.join(ROOT, "self-play-racing_amd")]))
    r = subprocess.run([sys.executable, "-m", "oracle.cpu_baseline"], input=arg, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["torch_loaded"] is False and out["steps"] > 0


def test_cpu_baseline_worker_timeout_is_enforced():
    """A worker that outlives the deadline is killed and reported (ADVICE r04:
    the waits used to come after blocking pipe reads, so the timeout never applied)."""
    import time
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))
    from rx.track import gen_tracks
    from oracle.cpu_baseline import run_workers
    import numpy as np
    import pytest
    np.random.seed(1)
    pool = gen_tracks(1, seed=1)
    t0 = time.monotonic()
    with pytest.raises(RuntimeError, match="still running"):
        run_workers([(pool[0], 7, 60.0, 0)], timeout_s=3)
    assert time.monotonic() - t0 < 30
