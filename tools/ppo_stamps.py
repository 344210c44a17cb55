"""Phase breakdown of k_ppo_grad from in-kernel s_memtime stamps.

    python tools/ppo_stamps.py build             # here: rx/lib/librx_ppostamps.so (-DRX_PPO_STAMPS)
    python tools/ppo_stamps.py [mb] [fp32|bf16]  # on the GPU box: per-phase cycles per wave (JSON)

Stamps (per wave, s_memtime = shader clock): 0 entry, 1 weights staged (barrier),
then per 64-row pass p: 2+4p after phase A (forward, loss, dZ2, transposes
written), 3+4p after B (dW2, db2, dH1, dZ1), 4+4p after C (second transposes),
5+4p after D (dW1, dW3, db3); 14 before the partial-row stores, 15 after the
small-sum barrier.  Profiling variant only; the product library has no stamps.
Reference: agent/ppo.py:170-203 (the minibatch loss and backward the kernel fuses).
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))
sys.path.insert(0, ROOT)
LIB = os.path.join(ROOT, "self-play-racing_amd", "rx", "lib", "librx_ppostamps.so")

if len(sys.argv) > 1 and sys.argv[1] == "build":
    from rx import _build
    print(_build.build(out=LIB, defines=("RX_PPO_STAMPS",)))
    sys.exit(0)

os.environ["RX_LIB_PATH"] = LIB
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rx import _lib  # noqa: E402
from rx.agent import Agent  # noqa: E402
from rx.configs import base_config  # noqa: E402
from rx.optim import FlatAdam  # noqa: E402
from rx.ppo_fused import FusedMinibatchGrad  # noqa: E402
from rx.spaces import Box  # noqa: E402

mb = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
prec = sys.argv[2] if len(sys.argv) > 2 else "fp32"
D, B = 15, 16 * mb
torch.manual_seed(3)
ag = Agent(Box(-1, 1, (D,)), Box(-1, 1, (2,))).cuda()
ag.log_std.fill_(-0.8)
fl = FlatAdam(ag, torch.optim.Adam(ag.parameters(), lr=1e-3, eps=1e-5), 0.5)
g = torch.Generator(device="cuda").manual_seed(0)
obs = torch.rand(B, D, generator=g, device="cuda") * 2 - 1
act = torch.rand(B, 2, generator=g, device="cuda") * 2 - 1
logp = torch.randn(B, generator=g, device="cuda") * 0.3 - 1.0
adv = torch.randn(B, generator=g, device="cuda") * 5
ret = torch.randn(B, generator=g, device="cuda") * 10
val = ret + torch.randn(B, generator=g, device="cuda") * 0.3
perm = torch.randperm(B, device="cuda")
cfg = base_config(kl_target=1e9, policy_dtype=prec)
fg = FusedMinibatchGrad(ag, fl, (obs, act, logp, adv, ret, val), mb, perm, cfg)
fg.adv_stats()
stop = torch.zeros(1, dtype=torch.bool, device="cuda")
kl = torch.zeros(1, device="cuda")
L = _lib.load()
L.rx_ppo_stamps_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
n_wg = L.rx_ppo_workspace_doubles(mb)
NW = int(os.environ.get("RX_PPO_NW", "4"))  # waves per k_ppo_grad workgroup of the build (rx_ppo.hip RX_PPO_NW)
n_waves = 2 * n_wg * NW
buf = np.zeros((8192, 24), np.uint64)
for m in range(4):  # warm
    fg.grad(m, stop, kl)
assert L.rx_ppo_stamps_read(buf.ctypes.data, 8192) == 0
res = []
for m in range(4, 12):
    fg.grad(m, stop, kl)
    assert L.rx_ppo_stamps_read(buf.ctypes.data, 8192) == 0
    st = buf[:n_waves].astype(np.float64)
    passes = (mb // n_wg) // (16 * NW)
    cols = [0, 1] + [c for p in range(passes) for c in (2 + 4 * p, 3 + 4 * p, 4 + 4 * p, 5 + 4 * p)] + [14, 15]
    s = st[:, cols]
    ok = (s > 0).all(axis=1)
    d = np.diff(s[ok], axis=1)
    res.append({"waves": int(ok.sum()), "passes": passes, "phase_cycles_median": np.median(d, axis=0).round(0).tolist(),
                "wave_total_median": float(np.median(s[ok, -1] - s[ok, 0])),
                "launch_span_cycles": float(s[ok, -1].max() - s[ok, 0].min()),
                "start_spread_cycles": float(np.percentile(s[ok, 0], 99) - s[ok, 0].min()),
                "end_spread_cycles": float(s[ok, -1].max() - np.percentile(s[ok, -1], 1))})
    a = st[:, [1, 16, 17, 18, 19, 2]]  # pass 0, phase A: layer 1, layer 2, head, loss, dZ2 + transposes
    ok = (a > 0).all(axis=1)
    if ok.any():  # (the fp32 trunk's forward sub-stamps; the bf16 trunk has none)
        res[-1]["p0A_sub_cycles_median"] = dict(zip(["layer1", "layer2", "head", "loss", "dz2_lds"],
                                                    np.median(np.diff(a[ok], axis=1), axis=0).round(0).tolist()))
labels = ["stage"] + [f"p{p}{ph}" for p in range(res[-1]["passes"]) for ph in "ABCD"] + ["accum", "small"]
out = {"mb": mb, "precision": prec, "n_wg_per_trunk": n_wg, "labels": labels, "runs": res[-3:]}
print(json.dumps(out))
