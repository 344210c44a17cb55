"""Latency breakdown of k_dyn1 from in-kernel s_memtime stamps.

    python tools/dyn_stamps.py build      # here: compiles rx/lib/librx_stamps.so (-DRX_DYN_STAMPS)
    python tools/dyn_stamps.py [N]        # on the GPU box: per-phase cycles per wave
    python tools/dyn_stamps.py kin build / kin [N]   # the split step's k_kin1 (8 -> 9: the ray-task sort)

Phases (k_dyn1, stamps after a full s_waitcnt): 0->1 wave record, perm and
state loads; 1->2 dynamics (sincos); 2->3 argmin window scan; 3->4 waypoint
super-chunk tests; 4->5 leaf visits; 5->6 wall collision; 6->7 reward / done /
state stores; 7->8 outputs; 8->9 episode stats + ray task sort.  Profiling variant only; the product library has no stamps.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))
sys.path.insert(0, ROOT)
LIB = os.path.join(ROOT, "self-play-racing_amd", "rx", "lib", "librx_stamps.so")

KIN = "kin" in sys.argv  # the split step's k_kin1 (a build whose REWARD half writes no stamps)
if KIN:
    sys.argv.remove("kin")
    LIB = LIB.replace("librx_stamps.so", "librx_kstamps.so")
if len(sys.argv) > 1 and sys.argv[1] == "build":
    from rx import _build
    print(_build.build(out=LIB, defines=("RX_DYN_STAMPS",) + (("RX_DYN_STAMPS_NO_REWARD",) if KIN else ())))
    sys.exit(0)

os.environ["RX_LIB_PATH"] = LIB
import numpy as np  # noqa: E402
import torch  # noqa: E402

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
res = []
env.counters = torch.zeros(16 + 12 * n_waves, dtype=torch.int64, device="cuda")
env._io_cache.clear()  # the cached io structs hold the counters pointer
for rep in range(5):
    env.counters.zero_()
    env.step_device(torch.rand((N, 2), generator=g, device="cuda") * scale + shift, phases=1)
    torch.cuda.synchronize()
    st = env.counters[16:].view(n_waves, 12)[:, :10].cpu().numpy().astype(np.float64)
    if KIN:  # KIN runs no argmin: stamps 3-5 stay 0; phases loads, kinematics, state / outputs, obs cols, task sort
        st = st[:, [0, 1, 2, 6, 7, 8, 9]]
    ok = (st > 0).all(axis=1)
    d = np.diff(st[ok], axis=1)
    span = st[ok, -1].max() - st[ok, 0].min()
    res.append({"waves": int(ok.sum()), "phase_cycles_median": np.median(d, axis=0).round(0).tolist(),
                "phase_cycles_mean": d.mean(axis=0).round(0).tolist(),
                "wave_total_median": float(np.median(st[ok, -1] - st[ok, 0])),
                "launch_span_cycles": float(span),
                "start_spread_cycles": float(np.percentile(st[ok, 0], 99) - st[ok, 0].min())})
print(json.dumps(res[-1], indent=1))
