"""Stress pool (gen_tracks(N, seed=None), a slot per env) --
per-kernel durations of the step under several schedules (rx_profile wave stamps),
each after the same burn-in.  Phases: 'step' = k_kin1 + k_step2 (REWARD beside the
raycast); 'split' = k_kin1 + k_step2 (REWARD only) + k_rays alone.

    python tools/r06/stress_probe.py [N] [sched ...]   (sched: 'lane_tracks=1,...'; default set below)
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))
sys.path.insert(0, ROOT)


def main():
    from bench import stress_pool
    from rx.track import TrackSet
    from rx.vector_env import RacingVectorEnv
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    workers = int(os.environ.get("RX_PROBE_WORKERS", "0")) or None  # 1: serial table build (under a profiler)
    scheds = sys.argv[2:] or ["lane_tracks=1", "lane_tracks=-1", "lane_tracks=-1,ray_lpr=4,reward_lpe=4",
                              "lane_tracks=-1,ray_lpr=4"]
    t0 = time.perf_counter()
    pool, widths = stress_pool(n)
    ts = TrackSet.build(pool, widths, workers=workers)
    print(f"table {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    acts = torch.rand((64, n, 2), device=dev, generator=g) * torch.tensor([2.0, 1.0], device=dev) + \
        torch.tensor([-1.0, 0.0], device=dev)
    for sc in scheds:
        sched = {k: int(v) for k, v in (kv.split("=") for kv in sc.split(",") if kv)}
        # cull_chunk / cull_super are table-build parameters (rx_config), not schedule fields
        geo = {k: sched.pop(k) for k in ("cull_chunk", "cull_super") if k in sched}
        env = RacingVectorEnv(pool, widths, device=dev, autoreset="next_step", track_set=ts, sched=sched, **geo)
        env.reset_device()
        for k in range(100):
            env.step_device(acts[k % 64])
        torch.cuda.synchronize()
        env.profile(1)
        for k in range(16):
            env.step_device(acts[k % 64])
        env.profile(0)
        step = env.profile_read()
        env.profile(1)
        for k in range(16):
            env.step_device(acts[k % 64], phases=1)
            env.step_device(acts[k % 64], phases=2)
        env.profile(0)
        split = env.profile_read()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for k in range(50):
            env.step_device(acts[k % 64])
        torch.cuda.synchronize()
        el = (time.perf_counter() - t1) / 50
        out = {"sched": sc, "n": n, "lib": os.path.basename(os.environ.get("RX_LIB_PATH", "librx.so")), "schedule": {k: v for k, v in env.schedule().items() if k in (
            "lane_tracks", "ray_lpr", "reward_lpe", "dyn_waves", "ray_waves")},
               "step_ms": {k: round(v[0], 4) for k, v in step.items()},
               "split_ms": {k: round(v[0], 4) for k, v in split.items()},
               "eager_ms_per_step": round(el * 1e3, 4), "env_steps_per_s": round(n / el / 1e6, 1)}
        print(json.dumps(out), flush=True)
        env.close()


if __name__ == "__main__":
    main()
