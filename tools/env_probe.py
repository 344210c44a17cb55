"""Env-only throughput and per-kernel durations (rx_profile) for a vector env
configuration: python tools/env_probe.py N AGENTS [steps]."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))
sys.path.insert(0, ROOT)
from bench import seed1_pool  # noqa: E402
from rx.vector_env import RacingVectorEnv  # noqa: E402

N, A = int(sys.argv[1]), int(sys.argv[2])
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 400
pool, widths = seed1_pool(N)
if os.environ.get("PROBE_CONTIG") == "1":  # envs of one slot contiguous: the wave order is the env order
    key = [hash((pool[i].tobytes(), int(widths[i]))) for i in range(N)]
    order = sorted(range(N), key=lambda i: key[i])
    pool, widths = [pool[i] for i in order], [widths[i] for i in order]
env = RacingVectorEnv(pool, widths, n_agents=A, device="cuda",
                      sort_interval=int(os.environ.get("PROBE_SORT", "16")))
env.reset_device()
lo = torch.tensor([-1.0, 0.0] if A == 1 else [-1.0, -1.0], device="cuda")
bank = torch.rand((64, N, A, 2) if A == 2 else (64, N, 2), device="cuda") * 2 - 1
if A == 1:
    bank[..., 1] = bank[..., 1].abs()
for k in range(100):
    env.step_device(bank[k % 64])
torch.cuda.synchronize()
env.profile(1)
t0 = time.perf_counter()
for k in range(steps):
    rec = k % 8 == 0
    if rec:
        env.profile(2)
    env.step_device(bank[k % 64])
    if rec:
        env.profile(0)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
prof = env.profile_read()
split = None
if os.environ.get("PROBE_SPLIT") == "1":  # REWARD half alone + the raycast alone (rx_step_phases 1, 2)
    env.profile(1)
    for k in range(16):
        env.step_device(bank[k % 64], phases=1)
        env.step_device(bank[k % 64], phases=2)
    env.profile(0)
    split = {k: round(v[0] * 1e3, 1) for k, v in env.profile_read().items()}
print(json.dumps({"contig": os.environ.get("PROBE_CONTIG", "0"), "sort": os.environ.get("PROBE_SORT", "16"), "N": N, "agents": A, "env_steps_per_s": round(N * steps / dt), "us_per_step": round(dt / steps * 1e6, 1),
                  "kernels_us": {k: round(v[0] * 1e3, 1) for k, v in prof.items()}, "split_us": split}))
