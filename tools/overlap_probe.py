"""Timing probe (results are NOT meaningful, only kernel overlap): does k_dyn1
run concurrently with k_rays on a second stream?  (a) one stream: dyn then
rays; (b) dyn on stream 2 concurrently with rays on stream 1, joined per step."""
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

N = 65536
pool, widths = seed1_pool(N)
env = RacingVectorEnv(pool, widths, device="cuda")
env.reset_device()
a = torch.rand((N, 2), device="cuda") * torch.tensor([2.0, 1.0], device="cuda") - torch.tensor([1.0, 0.0], device="cuda")
s1 = torch.cuda.current_stream()
s2 = torch.cuda.Stream()
res = {}
for mode in ("seq", "conc", "seq", "conc"):
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(200):
            if mode == "seq":
                env.step_device(a)
            else:
                e0 = torch.cuda.Event()
                e0.record(s1)
                s2.wait_event(e0)
                env.step_device(a, phases=1, stream=s2)
                env.step_device(a, phases=2, stream=s1)
                e1 = torch.cuda.Event()
                e1.record(s2)
                s1.wait_event(e1)
        torch.cuda.synchronize()
        res[mode] = round((time.perf_counter() - t0) / 200 * 1e6, 1)
    print(mode, res[mode], "us/step", flush=True)
print(json.dumps(res))
