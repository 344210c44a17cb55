"""A/B: one 65,536-env handle on one stream vs the same envs split into G
handles on G streams (fork/join per step).  Measures whether concurrent
kernels fill the tails of k_dyn1 / k_rays."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))
sys.path.insert(0, ROOT)


def run(groups, steps=200, warmup=20, E=65536, graph_steps=0):
    from bench import seed1_pool
    from rx.vector_env import RacingVectorEnv
    dev = torch.device("cuda", 0)
    pool, widths = seed1_pool(E)
    n = E // groups
    envs = [RacingVectorEnv(pool[g * n:(g + 1) * n], widths[g * n:(g + 1) * n], device=dev) for g in range(groups)]
    streams = [torch.cuda.Stream(device=dev) for _ in range(groups)]
    torch.manual_seed(0)
    acts = torch.empty((E, 2), device=dev)
    for e in envs:
        e.reset_device()
    def step():
        main = torch.cuda.current_stream(dev)
        torch.rand((E, 2), device=dev, out=acts)
        if groups == 1:
            envs[0].step_device(acts)
            return
        for g, (e, s) in enumerate(zip(envs, streams)):
            s.wait_stream(main)
            with torch.cuda.stream(s):
                e.step_device(acts[g * n:(g + 1) * n])
        for s in streams:
            main.wait_stream(s)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if graph_steps:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(graph_steps):
                step()
        runs = steps // graph_steps
        steps = runs * graph_steps
        g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(runs):
            g.replay()
        torch.cuda.synchronize()
        return E * steps / (time.perf_counter() - t0)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return E * steps / dt


if __name__ == "__main__":
    out = {f"groups={g}": round(run(g) / 1e6, 1) for g in (1, 2, 4)}
    for gs in (1, 10):
        for g in (1, 2, 4):
            out[f"graph{gs} groups={g}"] = round(run(g, graph_steps=gs) / 1e6, 1)
    print(json.dumps({"env_steps_per_s_M": out}))
