"""Same-session A/B of launch schedules on the bench workload (GPU box).

    python tools/ab_sched.py OUT.jsonl [--envs 65536] [--agents 1] [--steps 300] [--rounds 3]
                             --variant name:k=v,k=v [--variant ...]

One process, one track pool: for every round, each variant builds its own
RacingVectorEnv (rx_config schedule fields, include/rx.h; scheduling only --
results are identical), runs a 150-step burn-in of the bench's uniform random
actions, times --steps production steps (one rx_step each, queue-drain sync at
both edges, exactly bench.py's timed region), then records 16 instrumented steps
for the k_step2 wave-slot view (tools/wave_profile.py summarize).  Rounds
interleave the variants so box drift hits all of them alike.  One JSON line per
(round, variant) plus a summary line per variant (median env-steps/s).
"""
import argparse
import gc
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))
sys.path.insert(0, ROOT)


def parse_variant(v):
    name, _, kv = v.partition(":")
    return name, {k: int(x) for k, x in (p.split("=") for p in kv.split(",") if p)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--agents", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--burn", type=int, default=150)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variant", action="append", required=True)
    args = ap.parse_args()
    from bench import seed1_pool, wave_slots
    from rx.vector_env import RacingVectorEnv
    N, A = args.envs, args.agents
    pool, widths = seed1_pool(N)
    variants = [parse_variant(v) for v in args.variant]
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    scale = torch.tensor([2.0, 1.0], device=dev) if A == 1 else torch.tensor(2.0, device=dev)
    shift = torch.tensor([-1.0, 0.0], device=dev) if A == 1 else torch.tensor(-1.0, device=dev)
    shape = (N, 2) if A == 1 else (N, 2, 2)
    bank_n = 64
    bank = torch.addcmul(shift, torch.rand((bank_n,) + shape, device=dev), scale)
    res = {name: [] for name, _ in variants}
    out = open(args.out, "a")
    for rnd in range(args.rounds):
        for name, sched in variants:
            env = RacingVectorEnv(pool, widths, n_agents=A, device=dev, autoreset="next_step", sched=sched)
            env.reset_device()
            for k in range(args.burn):
                env.step_device(bank[k % bank_n])
            torch.cuda.synchronize()
            gc.collect()
            gc.disable()
            s = torch.cuda.current_stream(dev)
            while not s.query():
                pass
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(args.steps):
                env.step_device(bank[k % bank_n])
            while not s.query():
                pass
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            gc.enable()
            env.profile(1)
            for k in range(16):
                env.step_device(bank[k % bank_n])
            env.profile(0)
            prof = env.profile_read()
            ws = wave_slots(env, 32) if A == 1 else None
            rate = N * args.steps / el
            line = {"round": rnd, "variant": name, "sched": sched, "schedule": env.schedule(), "envs": N, "agents": A,
                    "steps": args.steps, "env_steps_per_s": round(rate, 1), "ms_per_step": round(el / args.steps * 1e3, 4),
                    "kernels_ms": {k: round(v[0], 5) for k, v in prof.items()}, "wave_slots": ws}
            res[name].append(rate)
            out.write(json.dumps(line) + "\n")
            out.flush()
            print(f"round {rnd} {name}: {rate / 1e6:.1f} M env-steps/s  k_step2 "
                  f"{prof.get('k_step2', (float('nan'),))[0] * 1e3:.1f} us  util "
                  f"{(ws or {}).get('wave_slot_utilisation')}", flush=True)
            env.close()
            del env
    for name, _ in variants:
        v = sorted(res[name])
        line = {"summary": name, "median_env_steps_per_s": round(v[len(v) // 2], 1), "all": [round(x, 1) for x in v]}
        out.write(json.dumps(line) + "\n")
        print(json.dumps(line), flush=True)
    out.close()


if __name__ == "__main__":
    main()
