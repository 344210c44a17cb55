"""A/B: GAE's bootstrap value from the fused policy kernel (config fused_next_value, the
default) vs torch's critic forward, on bench.py's ppo_leg (configs[1], 4,096 envs x 128
steps, 3 timed updates), fp32 and bf16, rounds interleaved.  One JSON line per run."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda", 0)
for r in range(2):
    for prec in ("fp32", "bf16"):
        for fused in (True, False):
            out = bench.ppo_leg(1, 0, dev, None, "nccl", 4096, 128, 3, policy_dtype=prec,
                                extra={"fused_next_value": fused})
            print(json.dumps({"round": r, "precision": prec, "fused_next_value": fused, "value": out["value"],
                              "ms_per_update": out["ms_per_update"]}), flush=True)
