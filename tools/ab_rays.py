"""Interleaved A/B of env-step variants in ONE process (cdna guide §5.4 rule 24).

    python tools/ab_rays.py [--envs 65536] [--rounds 5] [--steps 50]

Variants: brute-force raycast vs chunk culling (G = 8/16/32) with/without
the spatial re-sort.  Every variant steps the same seed-1 pool with the same
random action stream; per round each variant runs --steps steps; reports
median/min ms per step and per kernel phase (HIP events).
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--variants", default="0:0,16:0,16:1,8:1,32:1,16:4")
    args = ap.parse_args()
    from bench import seed1_pool
    from rx.vector_env import RacingVectorEnv
    pool, widths = seed1_pool(args.envs)
    dev = torch.device("cuda", 0)
    variants = [tuple(int(x) for x in v.split(":")) for v in args.variants.split(",")]
    envs = {v: RacingVectorEnv(pool, widths, device=dev, cull_chunk=v[0], sort_interval=v[1]) for v in variants}
    g = torch.Generator(device=dev)
    res = {v: {"step": [], "dyn": [], "rays": []} for v in variants}
    for v, e in envs.items():
        e.reset_device()
        g.manual_seed(0)
        for _ in range(20):  # warm up + spread the cars out
            a = torch.rand((args.envs, 2), generator=g, device=dev) * 2 - 1
            e.step_device(a)
    torch.cuda.synchronize()
    for r in range(args.rounds):
        for v, e in envs.items():
            g.manual_seed(100 + r)
            ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
            for k in range(args.steps):
                a = torch.rand((args.envs, 2), generator=g, device=dev) * 2 - 1
                a[:, 1].abs_()
                ev[k][0].record()
                e.step_device(a, phases=1)
                ev[k][1].record()
                e.step_device(a, phases=2)
                ev[k][2].record()
            torch.cuda.synchronize()
            res[v]["dyn"].append(np.mean([x[0].elapsed_time(x[1]) for x in ev]))
            res[v]["rays"].append(np.mean([x[1].elapsed_time(x[2]) for x in ev]))
            res[v]["step"].append(np.mean([x[0].elapsed_time(x[2]) for x in ev]))
    out = {}
    for v in variants:
        out[f"cull{v[0]}_sort{v[1]}"] = {k: {"median_ms": float(np.median(x)), "min_ms": float(np.min(x))}
                                         for k, x in res[v].items()}
    print(json.dumps({"envs": args.envs, "rounds": args.rounds, "steps": args.steps, "results": out}, indent=1))


if __name__ == "__main__":
    main()
