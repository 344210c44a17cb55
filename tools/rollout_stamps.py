"""Phase timing of the persistent rollout (k_rollout) from a -DRX_ROLL_STAMPS
build: per step, policy / KIN / REWARD+raycast durations of workgroup 0.

    python tools/rollout_stamps.py [N] [T]   (builds rx/lib/librx_rstamps.so)"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))
sys.path.insert(0, ROOT)
LIB = os.environ.get("RSTAMPS_LIB") or os.path.join(ROOT, "self-play-racing_amd", "rx", "lib", "librx_rstamps.so")
if not os.path.exists(LIB):
    from rx import _build
    _build.build(out=LIB, defines=["RX_ROLL_STAMPS"], verbose=False)
os.environ["RX_LIB_PATH"] = LIB
from tests.test_ppo_gpu import _train_single_style  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 16
T = int(sys.argv[2]) if len(sys.argv) > 2 else 512
t, c = _train_single_style(num_envs=N, num_steps=T)
ro = t._fused_rollout(T)
cnt = torch.zeros(16 + 8 * 512, dtype=torch.int64, device="cuda")
t.envs.counters = cnt
t.envs._io_cache.clear()
bufs = t._buffers()
nobs = t.envs.buf["obs"].clone()
nd = torch.zeros(N, device="cuda")
for rep in range(3):
    obs, actions, logprobs, dones, rewards, values = bufs
    obs[0].copy_(nobs)
    dones[0].copy_(nd)
    torch.cuda.synchronize()
    ro(obs, actions, logprobs, dones, rewards, values, nobs, nd)
    torch.cuda.synchronize()
st = cnt[16:].view(512, 8).cpu().numpy().astype(np.float64) * 10e-3  # 100 MHz ticks -> us
n = min(T, 512)
st = st[:n]
pol = st[:, 1] - st[:, 0]
kin = st[:, 2] - st[:, 1]
rest = st[:, 3] - st[:, 2]
step = np.diff(st[:, 0])
rew = st[:, 4] - st[:, 2]
ray = st[:, 5] - st[:, 2]
print(json.dumps({"N": N, "T": T, "us_policy": round(float(np.median(pol)), 2), "us_kin": round(float(np.median(kin)), 2),
                  "us_reward_rays": round(float(np.median(rest)), 2),
                  "us_reward": round(float(np.median(rew)), 2), "us_ray1": round(float(np.median(ray)), 2), "us_step": round(float(np.median(step)), 2)}))
