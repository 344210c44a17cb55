"""Rollout groups probe (GPU box): is a T-step rollout of N single-agent envs
faster as G independent env groups, each with its own handle and HIP stream,
than as one handle?  Each group runs rx_rollout_steps (policy + env kernels)
over its own [T, N/G] buffers; the groups never wait for each other until the
rollout ends.  Per env the trajectory is the same either way (each env's step
depends only on its own obs and its noise), so only the time can differ.

    python tools/group_probe.py OUT.jsonl [--envs 4096] [--T 128] [--groups 1,2,4] [--rounds 3]
                                [--sched k=v,...] [--prec fp32|bf16]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))
sys.path.insert(0, ROOT)
from bench import seed1_pool  # noqa: E402
from rx import _lib, ppo_fused  # noqa: E402
from rx.agent import Agent  # noqa: E402
from rx.optim import FlatParams  # noqa: E402
from rx.vector_env import RacingVectorEnv  # noqa: E402


class Group:
    def __init__(self, pool, widths, agent, flat, T, prec, sched):
        self.env = RacingVectorEnv(pool, widths, device="cuda", sched=sched)
        self.env.reset_device()
        n, D = self.env.num_envs, self.env.D
        z = dict(dtype=torch.float32, device="cuda")
        self.bufs = (torch.zeros((T, n, D), **z), torch.zeros((T, n, 2), **z), torch.zeros((T, n), **z),
                     torch.zeros((T, n), **z), torch.zeros((T, n), **z), torch.zeros((T, n), **z),
                     self.env.buf["obs"].clone(), torch.zeros(n, **z))
        self.ro = ppo_fused.StepRollout(agent, flat, self.env, T, prec)
        self.stream = torch.cuda.Stream()

    def rollout(self):
        obs, actions, logprobs, dones, rewards, values, next_obs, next_done = self.bufs
        with torch.cuda.stream(self.stream):
            obs[0].copy_(next_obs)
            dones[0].copy_(next_done)
            self.ro(*self.bufs, stream=self.stream)


def run(groups, cur):
    ev = []
    for g in groups:
        g.stream.wait_stream(cur)
        g.rollout()
        e = torch.cuda.Event()
        e.record(g.stream)
        ev.append(e)
    for e in ev:
        cur.wait_event(e)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--T", type=int, default=128)
    ap.add_argument("--groups", default="1,2,4")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--sched", default="")
    ap.add_argument("--prec", default="fp32")
    args = ap.parse_args()
    N, T = args.envs, args.T
    sched = {k: int(v) for k, v in (p.split("=") for p in args.sched.split(",") if p)}
    prec = _lib.RX_PREC_BF16 if args.prec == "bf16" else _lib.RX_PREC_FP32
    pool, widths = seed1_pool(N)
    torch.manual_seed(1)
    probe = RacingVectorEnv(pool[:64], widths[:64], device="cuda")
    agent = Agent(probe.single_observation_space, probe.single_action_space).cuda()
    probe.close()
    flat = FlatParams(agent)
    cur = torch.cuda.current_stream()
    configs = {}
    for G in (int(x) for x in args.groups.split(",")):
        n = N // G
        configs[G] = [Group(pool[i * n:(i + 1) * n], widths[i * n:(i + 1) * n], agent, flat, T, prec, sched)
                      for i in range(G)]
    out = open(args.out, "a")
    res = {G: [] for G in configs}
    for rnd in range(args.rounds):
        for G, groups in configs.items():
            for _ in range(2):  # warm-up rollouts (also moves the envs off their start lines)
                run(groups, cur)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.reps):
                run(groups, cur)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / args.reps
            res[G].append(N * T / dt)
            rec = {"round": rnd, "groups": G, "envs": N, "T": T, "prec": args.prec, "sched": sched,
                   "schedule": groups[0].env.schedule(), "ms_per_rollout": round(dt * 1e3, 3),
                   "us_per_step": round(dt / T * 1e6, 2), "env_steps_per_s": round(N * T / dt, 1)}
            out.write(json.dumps(rec) + "\n")
            out.flush()
            print(json.dumps(rec), flush=True)
    for G, v in res.items():
        s = {"summary": G, "envs": N, "median_env_steps_per_s": sorted(v)[len(v) // 2], "all": [round(x, 1) for x in v]}
        out.write(json.dumps(s) + "\n")
        print(json.dumps(s), flush=True)


if __name__ == "__main__":
    main()
