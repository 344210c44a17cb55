"""Latency breakdown of the production raycast waves (k_step2's ray half) from
in-kernel s_memtime stamps.

    python tools/ray_stamps.py build      # here: rx/lib/librx_raystamps.so (-DRX_RAY_STAMPS)
    python tools/ray_stamps.py [N]        # on the GPU box: one JSON object

Phases per ray wave (stamps after a full s_waitcnt): 0->1 task id, state
loads; 1->2 sincos; 2->3 culling setup; 3->4 box traversal + leaf scans;
4->5 obs store.  Also per wave: wall-clock start / end (100 MHz), box tests,
leaf scans, segments through the float32 pre-filter (4-segment groups), exact
segment tests run (some lane passed the pre-filter) and those that lowered
some lane's best.  Reported for all waves, by dispatch rank (ray-wave class run,
RX_RAY_DISPATCH 3) and for the waves that end in the last 25 % of the launch
(the tail).  Profiling variant only; the product library has no stamps.
Reference: environment/track.py:173-199 (the raycast these waves compute).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))
sys.path.insert(0, ROOT)
LIB = os.path.join(ROOT, "self-play-racing_amd", "rx", "lib", "librx_raystamps.so")

if len(sys.argv) > 1 and sys.argv[1] == "build":
    from rx import _build
    print(_build.build(out=LIB, defines=("RX_RAY_STAMPS",)))
    sys.exit(0)

os.environ.setdefault("RX_LIB_PATH", LIB)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import seed1_pool  # noqa: E402
from rx.vector_env import RacingVectorEnv  # noqa: E402


def stats(d, sel):
    if not np.any(sel):
        return None
    x = d[sel]
    return {"waves": int(sel.sum()), "phase_cycles_median": np.median(x[:, :5], axis=0).round(0).tolist(),
            "phase_cycles_mean": x[:, :5].mean(axis=0).round(0).tolist(),
            "wall_us_mean": round(float(x[:, 5].mean()), 2), "box_tests_mean": round(float(x[:, 6].mean()), 1),
            "leaf_scans_mean": round(float(x[:, 7].mean()), 2),
            "segments_prefiltered_mean": round(float(x[:, 10].mean()), 1),
            "exact_tests_mean": round(float(x[:, 8].mean()), 1), "exact_tests_lowering_best_mean": round(float(x[:, 9].mean()), 1)}


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    pool, widths = seed1_pool(N)
    env = RacingVectorEnv(pool, widths, device="cuda")
    env.reset_device()
    g = torch.Generator(device="cuda").manual_seed(0)
    scale = torch.tensor([2.0, 1.0], device="cuda")
    shift = torch.tensor([-1.0, 0.0], device="cuda")

    def act():
        return torch.rand((N, 2), generator=g, device="cuda") * scale + shift
    for _ in range(150):
        env.step_device(act())
    sched = env.schedule()
    nrw = sched["ray_waves"]
    maxw = -(-64 * sched["ray_lpr"] * env.n_sensors // 64)
    env.counters = torch.zeros(16 + 12 * nrw, dtype=torch.int64, device="cuda")
    env._io_cache.clear()  # the cached io structs hold the counters pointer
    out = {"n_envs": N, "schedule": sched, "runs": []}
    for rep in range(3):
        env.counters.zero_()
        env.step_device(act())
        torch.cuda.synchronize()
        raw = env.counters[16:].view(nrw, 12).cpu().numpy()
        st = raw[:, :10].astype(np.float64)
        ok = st[:, 0] > 0
        d = np.zeros((nrw, 11))
        d[:, 8] = (raw[:, 10] & 0xFFFFFFFF).astype(np.float64)  # exact segment tests (some lane passed the pre-filter)
        d[:, 9] = (raw[:, 10] >> 32).astype(np.float64)  # of them: a lane's best lowered
        d[:, 10] = raw[:, 11].astype(np.float64)  # segments through the pre-filter (4-segment groups)
        d[:, :5] = np.diff(st[:, :6], axis=1)
        d[:, 5] = (st[:, 7] - st[:, 6]) / 100.0  # 100 MHz ticks -> us
        d[:, 6:8] = st[:, 8:10]
        t0 = st[ok, 6].min()
        end = (st[:, 7] - t0) / 100.0
        span = float(end[ok].max())
        rank = (np.arange(nrw) // 8) // max(1, nrw // maxw // 8)
        run = {"span_us": round(span, 2), "all": stats(d, ok),
               "by_dispatch_rank": [stats(d, ok & (rank == r)) for r in range(maxw)],
               "tail_last_25pct": stats(d, ok & (end >= 0.75 * span)),
               "corr_wall_us_vs_box_tests": round(float(np.corrcoef(d[ok, 5], d[ok, 6])[0, 1]), 3),
               "corr_wall_us_vs_leaf_scans": round(float(np.corrcoef(d[ok, 5], d[ok, 7])[0, 1]), 3)}
        out["runs"].append(run)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
