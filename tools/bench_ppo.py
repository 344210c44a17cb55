"""PPO training throughput on the device engine (BASELINE.json configs[1], [3]).

    python tools/bench_ppo.py --mode single --envs 4096 --steps 128 [--bf16] [--no-graph]
    python tools/bench_ppo.py --mode selfplay --envs 8192 --steps 128

Times complete PPO updates (rollout with the policy in the loop + GAE + 10 x
16-minibatch update) after one warm-up update, and reports env-steps/s of
training, the rollout-only rate, and the per-phase split.
"""
import argparse
import json
import os
import random
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["single", "selfplay"], default="single")
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=128)
    ap.add_argument("--updates", type=int, default=3)
    ap.add_argument("--bf16", action="store_true")
    ap.add_argument("--no-graph", action="store_true", help="eager rollout (no captured rollout graph)")
    ap.add_argument("--no-graph-update", action="store_true", help="eager fused update (no captured epoch graphs)")
    ap.add_argument("--device-shuffle", action="store_true")
    args = ap.parse_args()
    from rx.configs import base_config, self_play_config
    from rx.envs import MultiRacingEnv, RacingEnv
    from rx.ppo import PPO
    from rx.selfplay import SelfPlayPPO
    from rx.track import gen_tracks
    mk = base_config if args.mode == "single" else self_play_config
    cfg = mk(num_envs=args.envs, num_steps=args.steps, policy_dtype="bf16" if args.bf16 else "fp32",
             graph_rollout=False if args.no_graph else "auto", graph_update=False if args.no_graph_update else "auto",
             kl_target=1e9,
             shuffle="device" if args.device_shuffle else "numpy")  # no early stop: time the full update
    cfg["total_timesteps"] = (args.updates + 1) * cfg["batch_size"]
    if os.environ.get("EPOCH_SYNC") is not None:  # A/B: host KL check after every epoch (1) or one per update (0)
        cfg["epoch_sync"] = os.environ["EPOCH_SYNC"] == "1"
    if os.environ.get("GRAPH_ROLLOUT") is not None:  # A/B: rollout as one captured HIP graph (1) or eager (0)
        cfg["graph_rollout"] = os.environ["GRAPH_ROLLOUT"] == "1"
    random.seed(1)
    np.random.seed(1)
    torch.manual_seed(1)
    pool = gen_tracks(args.envs, seed=1)
    widths = [np.random.randint(6, 10) for _ in range(args.envs)]
    if args.mode == "single":
        t = PPO(lambda i: RacingEnv(11, pool, i, widths[i]), cfg)
    else:
        t = SelfPlayPPO(lambda i: MultiRacingEnv(2, 11, pool, i, widths), cfg)
        t.opponent_pool.append(t.snapshot_agent())  # time the frozen-opponent path
    bufs = t._buffers()
    next_obs = t.envs.buf["obs"].clone()
    next_done = torch.zeros(t.num_local_envs, device=t.device)
    rows = []
    for u in range(args.updates + 1):
        if args.mode == "selfplay":
            t.update_opponent()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = t.collect_rollout(*bufs, next_obs, next_done)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        obs, actions, logprobs, dones, rewards, values, next_obs, next_done, ep = out
        with torch.no_grad():
            nv = t.agent.get_value(next_obs).flatten()
        adv, ret = t.compute_advantages(rewards, dones, values, nv, next_done)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        t.ppo_update(adv, ret, values, logprobs, actions, obs)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        rows.append((t1 - t0, t2 - t1, t3 - t2))
    r = np.array(rows[1:])  # drop the warm-up / capture update
    B = cfg["batch_size"]
    res = {"mode": args.mode, "envs": args.envs, "num_steps": args.steps, "batch": B,
           "policy_dtype": cfg["policy_dtype"], "graph_rollout": cfg["graph_rollout"],
           "graph_update": cfg["graph_update"], "shuffle": cfg["shuffle"],
           "first_rollout_s": rows[0][0], "first_update_only_s": rows[0][2],
           "rollout_s": float(r[:, 0].mean()), "gae_s": float(r[:, 1].mean()), "update_s": float(r[:, 2].mean()),
           "rollout_env_steps_per_s": B / float(r[:, 0].mean()),
           "train_env_steps_per_s": B / float(r.sum(axis=1).mean()),
           "first_update_s": float(sum(rows[0]))}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
