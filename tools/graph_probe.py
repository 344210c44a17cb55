"""Host/launch overhead probe: the bench's env step (65,536 envs, resident action
bank) issued eagerly vs replayed from a HIP graph of 16 steps (one sort period)."""
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

N, K = 65536, 16
pool, widths = seed1_pool(N)
env = RacingVectorEnv(pool, widths, device="cuda")
env.reset_device()
acts = torch.rand((K, N, 2), device="cuda") * torch.tensor([2.0, 1.0], device="cuda") - torch.tensor([1.0, 0.0],
                                                                                                    device="cuda")
for k in range(32):
    env.step_device(acts[k % K])
torch.cuda.synchronize()
res = {}
t0 = time.perf_counter()
for r in range(20):
    for k in range(K):
        env.step_device(acts[k])
t_host = time.perf_counter() - t0
torch.cuda.synchronize()
res["eager_us_per_step"] = (time.perf_counter() - t0) / (20 * K) * 1e6
res["eager_host_us_per_step"] = t_host / (20 * K) * 1e6
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    with torch.cuda.graph(g, stream=s):
        for k in range(K):
            env.step_device(acts[k])
torch.cuda.current_stream().wait_stream(s)
for _ in range(3):
    g.replay()
torch.cuda.synchronize()
t0 = time.perf_counter()
for r in range(20):
    g.replay()
torch.cuda.synchronize()
res["graph_us_per_step"] = (time.perf_counter() - t0) / (20 * K) * 1e6
print(json.dumps({k: round(v, 2) for k, v in res.items()}))
