"""A/B probe of rx_steps' multi-step windows (k_window) against the per-step
launches on the bench's workload (seed-1 pool, uniform random actions resident
in HBM, next-step autoreset): env-steps/s of one rx_steps call of --steps steps,
window on vs off, interleaved --reps times, plus the k_window / k_step2 launch
durations from the per-wave stamps (rx_profile).

    python tools/window_probe.py --envs 65536 --steps 1000 --reps 3
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
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--burn", type=int, default=200)
    ap.add_argument("--sched", default="", help="extra schedule overrides key=value,...")
    ap.add_argument("--label", default="")
    ap.add_argument("--mode", type=int, default=1, help="rx_config.window of the 'on' env: 1 k_window, 2 k_flow")
    ap.add_argument("--sort-interval", type=int, default=None)
    args = ap.parse_args()
    from rx.track import gen_tracks
    from rx.vector_env import RacingVectorEnv
    N = args.envs
    random.seed(1)
    np.random.seed(1)
    pool = gen_tracks(num_tracks=N, seed=1)
    widths = [np.random.randint(6, 10) for _ in range(N)]
    extra = {k: int(v) for k, v in (kv.split("=") for kv in args.sched.split(",") if kv)}
    envs = {w: RacingVectorEnv(pool, widths, device="cuda", autoreset="next_step", sort_interval=args.sort_interval,
                               sched={**extra, "window": args.mode if w == 1 else -1})
            for w in (1, -1)}
    torch.manual_seed(1234)
    K = args.steps
    bank = torch.rand((K + args.burn, N, 2), device="cuda")
    bank[..., 0].mul_(2.0).sub_(1.0)
    for v in envs.values():
        v.reset_device()
        v.steps_device(bank[:args.burn])
    torch.cuda.synchronize()
    res = {1: [], -1: []}
    for _ in range(args.reps):
        for w, v in envs.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            v.steps_device(bank[args.burn:args.burn + K])
            torch.cuda.synchronize()
            res[w].append(N * K / (time.perf_counter() - t0))
    prof = {}
    wg = None
    for w, v in envs.items():
        v.profile(1)
        v.steps_device(bank[args.burn:args.burn + 64])
        prof[w] = {k: [round(x[0] * 1e3, 2), x[1]] for k, x in v.profile_read().items()}
        v.profile(0)
        if w == 1 and "k_window" in prof[w]:
            durs, ends = [], []
            for k in range(prof[w]["k_window"][1]):
                st, en, kind, _ = v.profile_waves(k)
                live = np.isfinite(st) & np.isfinite(en)
                durs.append(en[live] - st[live])
                ends.append(en[live])
            d = np.concatenate(durs)
            e = np.concatenate(ends)
            wg = {"wg_dur_us_percentiles": [round(float(np.percentile(d, q)), 1) for q in (0, 10, 25, 50, 75, 90, 99, 100)],
                  "wg_end_us_percentiles": [round(float(np.percentile(e, q)), 1) for q in (0, 10, 25, 50, 75, 90, 99, 100)],
                  "hist_dur_us": np.histogram(d, bins=12)[0].tolist(),
                  "hist_edges_us": [round(float(x), 1) for x in np.histogram(d, bins=12)[1]]}
    out = {"label": args.label, "envs": N, "steps": K, "schedule_on": envs[1].schedule(),
           "window_on_Msteps": [round(x / 1e6, 1) for x in res[1]],
           "window_off_Msteps": [round(x / 1e6, 1) for x in res[-1]],
           "sort_interval": envs[1].sort_interval,
           "kernel_us_on": prof[1], "kernel_us_off": prof[-1], "window_workgroups": wg,
           "lib": os.environ.get("RX_LIB_PATH", "default")}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
