"""Where configs[3]'s per-update opponent draw + env rebuild time goes (SelfPlayPPO.update_opponent
pieces, device-synced), 8,192 two-car envs, pool filled.  One JSON line."""
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rx.configs import self_play_config  # noqa: E402
from rx.envs import MultiRacingEnv  # noqa: E402
from rx.selfplay import SelfPlayPPO  # noqa: E402
from rx.track import gen_tracks  # noqa: E402

N = 8192
cfg = self_play_config(num_envs=N, num_steps=128, kl_target=1e9, shuffle="device")
random.seed(1)
np.random.seed(1)
torch.manual_seed(1)
pool = gen_tracks(N, seed=1)
widths = [np.random.randint(6, 10) for _ in range(N)]
t = SelfPlayPPO(lambda i: MultiRacingEnv(2, 11, pool, i, widths), cfg)
for _ in range(5):
    t.opponent_pool.append(t.snapshot_agent())


def timeit(fn, reps=20):
    torch.cuda.synchronize()
    out = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        out.append((time.perf_counter() - t0) * 1e3)
    return round(float(np.median(out)), 4)


res = {}
t.update_opponent()
res["update_opponent_ms"] = timeit(t.update_opponent)
res["select_ms"] = timeit(t.select_opponent)
opp = t.curr_opponent


def copy_sd():
    with torch.no_grad():
        for dst, src in zip(t._opp_static.state_dict().values(), opp.state_dict().values()):
            dst.copy_(src)


res["state_dict_copy_ms"] = timeit(copy_sd)
from rx import ppo_fused  # noqa: E402
res["set_opponent_ms"] = timeit(lambda: t.envs.set_opponent(t._opp_static, t._opp_flat, ppo_fused.precision(t.config)))
res["reset_device_ms"] = timeit(t.envs.reset_device)
res["advance_pool_ms"] = timeit(lambda: t.advance_pool(1))
print(json.dumps(res), flush=True)
