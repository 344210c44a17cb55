"""k_kin1's ray-task sort split into its phases (profiling build librx_kstamps.so,
tools/dyn_stamps.py kin build): stamp 8 (before the sort) -> 10 (ranks: the LDS
atomics) -> 11 (scan + LDS scatter) -> 9 (row copy + task-id stores, after a full
s_waitcnt).  python tools/kin_sort_stamps.py [N]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))
sys.path.insert(0, ROOT)
os.environ["RX_LIB_PATH"] = os.path.join(ROOT, "self-play-racing_amd", "rx", "lib", "librx_kstamps.so")
from bench import seed1_pool  # noqa: E402
from rx.vector_env import RacingVectorEnv  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
pool, widths = seed1_pool(N)
env = RacingVectorEnv(pool, widths, device="cuda")
env.reset_device()
g = torch.Generator(device="cuda").manual_seed(0)
scale = torch.tensor([2.0, 1.0], device="cuda")
shift = torch.tensor([-1.0, 0.0], device="cuda")
for _ in range(40):
    env.step_device(torch.rand((N, 2), generator=g, device="cuda") * scale + shift)
n_waves = (N + 63) // 64
env.counters = torch.zeros(16 + 12 * n_waves, dtype=torch.int64, device="cuda")
env._io_cache.clear()
out = []
for rep in range(4):
    env.counters.zero_()
    env.step_device(torch.rand((N, 2), generator=g, device="cuda") * scale + shift, phases=1)
    torch.cuda.synchronize()
    st = env.counters[16:].view(n_waves, 12).cpu().numpy().astype(np.float64)
    s = st[:, [8, 10, 11, 9]]
    ok = (s > 0).all(axis=1)
    if ok.sum() == 0:
        out.append({"rep": rep, "sorted_waves": 0})
        continue
    d = np.diff(s[ok], axis=1)
    out.append({"rep": rep, "sorted_waves": int(ok.sum()), "ranks_scan_copy_median": np.median(d, axis=0).round(0).tolist(),
                "before_sort_median": float(np.median(st[ok, 8] - st[ok, 0]))})
print(json.dumps({"N": N, "phases": ["ranks (rel-angle loads, sectors, LDS atomics)", "scan + LDS scatter",
                                     "row copy + task-id stores"], "reps": out}, indent=1))
