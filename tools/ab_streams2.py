"""Concurrency probe: G independent env groups, each stepping on its own
stream with its own action draws and NO per-step cross-stream sync (joined
once at the end), vs one group on one stream."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))
sys.path.insert(0, ROOT)


def run(groups, steps=300, warmup=20, E=65536):
    from bench import seed1_pool
    from rx.vector_env import RacingVectorEnv
    dev = torch.device("cuda", 0)
    pool, widths = seed1_pool(E)
    n = E // groups
    envs = [RacingVectorEnv(pool[g * n:(g + 1) * n], widths[g * n:(g + 1) * n], device=dev) for g in range(groups)]
    streams = [torch.cuda.Stream(device=dev) for _ in range(groups)]
    acts = [torch.empty((n, 2), device=dev) for _ in range(groups)]
    us = [torch.empty((n, 2), device=dev) for _ in range(groups)]
    scale = torch.tensor([2.0, 1.0], device=dev)
    shift = torch.tensor([-1.0, 0.0], device=dev)
    gens = [torch.Generator(device=dev).manual_seed(g) for g in range(groups)]
    for e in envs:
        e.reset_device()
    torch.cuda.synchronize()

    def loop(k):
        for _ in range(k):
            for g in range(groups):
                with torch.cuda.stream(streams[g]):
                    torch.rand((n, 2), generator=gens[g], device=dev, out=us[g])
                    torch.addcmul(shift, us[g], scale, out=acts[g])  # steer U(-1,1), throttle U(0,1)
                    envs[g].step_device(acts[g])

    loop(warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    loop(steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    for e in envs:
        e.close()
    return E * steps / dt


if __name__ == "__main__":
    print(json.dumps({f"groups={g}": round(run(g) / 1e6, 1) for g in (1, 2, 4, 8)}))
