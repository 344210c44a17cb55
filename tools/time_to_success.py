"""PPO wall-clock to 90% success (second half of BASELINE.json's metric).

Trains the reference's single-agent PPO through the drop-in API (train.py's
train_single with rx imports: seed-1 pool, widths randint(6, 10), base
hyperparameters) and, every ``--eval-every`` updates, runs the evaluate.py
protocol (rx.evaluate: 40 tracks x 5 runs, seed 42, <= 2,000 steps,
stochastic policy).  Reports the training wall-clock (evaluations excluded)
at the first evaluation with success_rate >= target.

    python tools/time_to_success.py --num-envs 16 --num-steps 2048       # reference config
    python tools/time_to_success.py --num-envs 4096 --num-steps 128      # configs[1]
"""
import argparse
import contextlib
import io
import json
import os
import random
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))


def run(num_envs=16, num_steps=2048, total_timesteps=5_000_000, eval_every=5, target=0.9, max_minutes=15.0, seed=1,
        device_shuffle=False, quiet=False, policy_dtype="fp32"):
    """Train (train.py train_single through rx) and evaluate every ``eval_every``
    updates; returns the result dict (value_s = training seconds to target)."""
    from rx.configs import base_config
    from rx.envs import RacingEnv
    from rx.evaluate import Evaluator
    from rx.ppo import PPO
    from rx.track import gen_tracks

    config = base_config(num_envs=num_envs, num_steps=num_steps, total_timesteps=total_timesteps,
                         seed=seed, shuffle="device" if device_shuffle else "numpy", policy_dtype=policy_dtype)
    random.seed(config["seed"])
    np.random.seed(config["seed"])
    torch.manual_seed(config["seed"])
    pool = gen_tracks(num_tracks=config["num_envs"], seed=config["seed"])
    widths = [np.random.randint(6, 10) for _ in range(config["num_envs"])]

    def env_fn(i):
        return RacingEnv(num_sensors=11, track_pool=pool, track_id=i, track_width=widths[i])

    t_build = time.perf_counter()
    trainer = PPO(env_fn, config, device="cuda")
    evaluator = Evaluator(device=trainer.device)
    build_s = time.perf_counter() - t_build
    train_s = 0.0
    curve = []
    reached = None
    ctx = contextlib.redirect_stdout(io.StringIO()) if quiet else contextlib.nullcontext()
    with ctx:
        t0 = time.perf_counter()
        for update, num_updates, global_step, ep in trainer.train_iter():
            torch.cuda.synchronize()
            now = time.perf_counter()
            train_s += now - t0
            row = {"update": update + 1, "global_step": global_step, "train_s": round(train_s, 3),
                   "episodes": len(ep), "mean_reward": float(ep.mean_reward) if ep else None}
            if (update + 1) % eval_every == 0 or update + 1 == num_updates:
                te = time.perf_counter()
                res = evaluator.run(trainer.agent)
                row.update(success_rate=res["success_rate"], crash_rate=res["crash_rate"],
                           eval_s=round(time.perf_counter() - te, 3))
                if not quiet:
                    print(json.dumps(row), flush=True)
                if reached is None and res["success_rate"] >= target:
                    reached = dict(row)
                    curve.append(row)
                    break
            curve.append(row)
            if train_s > max_minutes * 60:
                break
            t0 = time.perf_counter()
    trainer.envs.close()
    evaluator.close()
    return {"metric": "PPO wall-clock to 90% success rate", "target": target,
            "value_s": reached["train_s"] if reached else None,
            "reached_at_step": reached["global_step"] if reached else None,
            "config": {"num_envs": num_envs, "num_steps": num_steps, "total_timesteps": total_timesteps,
                       "shuffle": config.get("shuffle", "numpy"), "policy_dtype": policy_dtype,
                       "eval": "evaluate.py protocol: 40 tracks (seed 42) x 5 runs, widths by run, max 2000 steps, "
                               "stochastic policy", "eval_every_updates": eval_every},
            "build_s": round(build_s, 3), "curve": curve}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--num-envs", type=int, default=16)
    ap.add_argument("--num-steps", type=int, default=2048)
    ap.add_argument("--total-timesteps", type=int, default=5_000_000)
    ap.add_argument("--eval-every", type=int, default=5)
    ap.add_argument("--target", type=float, default=0.9)
    ap.add_argument("--max-minutes", type=float, default=15.0)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default=None)
    ap.add_argument("--device-shuffle", action="store_true", help="config shuffle='device' (rx_random_permutation)")
    ap.add_argument("--policy-dtype", choices=("fp32", "bf16"), default="fp32",
                    help="config policy_dtype: bf16 runs the policy / PPO kernels on bf16 MFMA operands")
    args = ap.parse_args()
    out = run(args.num_envs, args.num_steps, args.total_timesteps, args.eval_every, args.target, args.max_minutes,
              args.seed, args.device_shuffle, policy_dtype=args.policy_dtype)
    print(json.dumps(out), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
