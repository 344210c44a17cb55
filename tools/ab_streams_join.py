"""Concurrency probe at steady state: the 65,536 envs as G groups on G streams,
with (join=1: fork from / join to one main stream every step, what a
synchronous rollout needs) or without (join=0) a per-step cross-stream sync.
    python tools/ab_streams_join.py"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))
sys.path.insert(0, ROOT)


def run(groups, join, steps=600, warmup=150, E=65536):
    from bench import seed1_pool
    from rx.vector_env import RacingVectorEnv
    dev = torch.device("cuda", 0)
    pool, widths = seed1_pool(E)
    n = E // groups
    envs = [RacingVectorEnv(pool[g * n:(g + 1) * n], widths[g * n:(g + 1) * n], device=dev) for g in range(groups)]
    main = torch.cuda.current_stream(dev)
    streams = [torch.cuda.Stream(device=dev) for _ in range(groups)]
    bank = torch.rand((32, E, 2), device=dev) * torch.tensor([2.0, 1.0], device=dev) - torch.tensor([1.0, 0.0], device=dev)
    fork = [torch.cuda.Event() for _ in range(groups)]
    done = [torch.cuda.Event() for _ in range(groups)]
    for e in envs:
        e.reset_device()
    torch.cuda.synchronize()

    def loop(k, t0=0):
        for t in range(k):
            a = bank[(t0 + t) % 32]
            if join:
                ev = torch.cuda.Event()
                ev.record(main)
            for g in range(groups):
                s = streams[g]
                if join:
                    s.wait_event(ev)
                with torch.cuda.stream(s):
                    envs[g].step_device(a[g * n:(g + 1) * n])
                if join:
                    done[g].record(s)
            if join:
                for g in range(groups):
                    main.wait_event(done[g])

    loop(warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    loop(steps, warmup)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    for e in envs:
        e.close()
    return E * steps / dt


if __name__ == "__main__":
    res = {}
    for rep in range(2):
        for g, j in ((1, 0), (2, 1), (2, 0), (4, 1), (4, 0)):
            res.setdefault(f"groups={g},join={j}", []).append(round(run(g, j) / 1e6, 1))
    print(json.dumps(res))
