"""Phase timing of the persistent rollout (k_rollout) from a -DRX_ROLL_STAMPS
build: per step, policy / KIN / REWARD+raycast durations of workgroup 0 (and
the slowest of its ray waves); with "dyn", from a -DRX_DYN_STAMPS build, the
REWARD half's own phases (dyn1_env stamps of workgroup 0's last step).

    python tools/rollout_stamps.py [N] [T] [dyn]   (builds rx/lib/librx_rstamps.so / librx_dstamps.so)"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))
sys.path.insert(0, ROOT)
DYN = len(sys.argv) > 3 and sys.argv[3] == "dyn"
LIB = os.environ.get("RSTAMPS_LIB") or os.path.join(ROOT, "self-play-racing_amd", "rx", "lib",
                                                    "librx_dstamps.so" if DYN else "librx_rstamps.so")
if not os.path.exists(LIB):
    from rx import _build
    _build.build(out=LIB, defines=["RX_DYN_STAMPS" if DYN else "RX_ROLL_STAMPS"], verbose=False)
os.environ["RX_LIB_PATH"] = LIB
from tests.test_ppo_gpu import _train_single_style  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 16
T = int(sys.argv[2]) if len(sys.argv) > 2 else 512
t, c = _train_single_style(num_envs=N, num_steps=T)
ro = t._fused_rollout(T)
cnt = torch.zeros(16 + 16 * 512, dtype=torch.int64, device="cuda")
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
if DYN:  # dyn1_env's stamps (s_memtime cycles) of workgroup 0: the REWARD half of the last step
    s = cnt[16:16 + 9].cpu().numpy().astype(np.float64)
    names = ["loads", "corners", "-", "-", "argmin", "collision_progress", "reward_state", "outputs"]
    ph = {nm: float(s[j + 1] - s[j]) for j, nm in enumerate(names) if nm != "-"}
    ph["argmin"] = float(s[5] - s[2])
    print(json.dumps({"N": N, "T": T, "reward_phase_cycles": ph, "total_cycles": float(s[8] - s[0])}))
    sys.exit(0)
st = cnt[16:].view(512, 16).cpu().numpy().astype(np.float64) * 10e-3  # 100 MHz ticks -> us
n = min(T, 512)
st = st[:n]
pol = st[:, 1] - st[:, 0]
kin = st[:, 2] - st[:, 1]
rest = st[:, 3] - st[:, 2]
step = np.diff(st[:, 0])
rew = st[:, 4] - st[:, 2]
ray = st[:, 5] - st[:, 2]
rays = st[:, 5:16] - st[:, 2:3]
med = lambda v: round(float(np.median(v)), 2)  # noqa: E731
print(json.dumps({"N": N, "T": T, "us_policy": med(pol), "us_kin": med(kin), "us_reward_rays": med(rest),
                  "us_reward": med(rew), "us_ray1": med(ray), "us_ray_slowest": med(rays.max(axis=1)),
                  "us_ray_per_wave": [med(rays[:, j]) for j in range(11)], "us_step": med(step)}))
