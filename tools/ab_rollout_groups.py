"""Probe: a configs[1] rollout (4,096 envs x 128 steps, fused policy) as G
independent env groups, each running policy + env step on its own HIP stream
with no per-step join (one join at the end).  Envs are independent, so every
group's trajectory is what the one-stream rollout computes for those envs.
    python tools/ab_rollout_groups.py [N] [T]"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))
sys.path.insert(0, ROOT)


def main():
    from rx import ppo_fused
    from rx.configs import base_config
    from rx.envs import RacingEnv
    from rx.ppo import PPO
    from rx.track import gen_tracks
    from rx.vector_env import RacingVectorEnv
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    np.random.seed(1)
    pool = gen_tracks(N, seed=1)
    widths = [np.random.randint(6, 10) for _ in range(N)]
    cfg = base_config(num_envs=N, num_steps=T)
    p = PPO(lambda i: RacingEnv(11, pool, i, widths[i]), cfg)
    D = p.envs.buf["obs"].shape[-1]
    dev = p.device
    obs = torch.zeros((T, N, D), device=dev)
    act = torch.zeros((T, N, 2), device=dev)
    lp = torch.zeros((T, N), device=dev)
    val = torch.zeros((T, N), device=dev)
    rew = torch.zeros((T, N), device=dev)
    don = torch.zeros((T, N), device=dev)
    nobs = torch.zeros((N, D), device=dev)
    ndone = torch.zeros(N, device=dev)
    res = {}
    for G in (1, 2, 4):
        n = N // G
        envs = [RacingVectorEnv(pool[g * n:(g + 1) * n], widths[g * n:(g + 1) * n], device=dev) for g in range(G)]
        pas = [ppo_fused.PolicyAct(p.agent, p._flat, n, D) for _ in range(G)]
        streams = [torch.cuda.Stream(device=dev) for _ in range(G)]
        main = torch.cuda.current_stream(dev)
        for g, e in enumerate(envs):
            obs[0, g * n:(g + 1) * n].copy_(e.reset_device())
        torch.cuda.synchronize()

        noise = torch.empty((T, N, 2), device=dev)

        def rollout():
            noise.normal_()  # all steps' N(0, 1) draws up front, on the main (capture) stream
            ev = torch.cuda.Event()
            ev.record(main)
            for s in streams:
                s.wait_event(ev)
            for t in range(T):
                last = t + 1 == T
                for g in range(G):
                    lo, hi = g * n, (g + 1) * n
                    with torch.cuda.stream(streams[g]):
                        a = pas[g](obs[t, lo:hi], act[t, lo:hi], lp[t, lo:hi], val[t, lo:hi], eps=noise[t, lo:hi])
                        envs[g].step_device(a, obs_out=nobs[lo:hi] if last else obs[t + 1, lo:hi],
                                            reward_out=rew[t, lo:hi], done_out=ndone[lo:hi] if last else don[t + 1, lo:hi])
            for s in streams:
                main.wait_stream(s)

        def timed(fn):
            ts = []
            for rep in range(4):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            return float(np.median(ts[1:]))
        te = timed(rollout)
        rollout()  # warm every path once more before the capture
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            rollout()
        tg = timed(gr.replay)
        res[f"G={G}"] = {"eager_ms": round(1e3 * te, 2), "graph_ms": round(1e3 * tg, 2),
                         "graph_env_steps_per_s_M": round(N * T / tg / 1e6, 1)}
        for e in envs:
            e.close()
    print(json.dumps({"N": N, "T": T, **res}))


if __name__ == "__main__":
    main()
