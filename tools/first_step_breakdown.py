"""Host-time breakdown of the first env step after a queue-draining sync, in the
bench's own sequence (burn-in, garbage collection, refill steps, sync, stats
read, sync), VERDICT r02 #3.  Wraps RacingVectorEnv.step_device's parts with
perf_counter (this probe only; the product path is not touched) and prints
the per-part host microseconds of the first four steps of a region.

    python tools/first_step_breakdown.py
"""
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import seed1_pool  # noqa: E402
from rx import _lib  # noqa: E402
from rx.vector_env import RacingVectorEnv  # noqa: E402

T = {}


def timed_part(name, fn):
    def w(*a, **k):
        t = time.perf_counter()
        r = fn(*a, **k)
        T.setdefault(name, []).append((time.perf_counter() - t) * 1e6)
        return r
    return w


def main():
    N = 65536
    pool, widths = seed1_pool(N)
    env = RacingVectorEnv(pool, widths, device="cuda", autoreset="next_step")
    env.reset_device()
    dev = env.device
    bank = torch.rand((248, N, 2), device=dev) * torch.tensor([2.0, 1.0], device=dev) - torch.tensor([1.0, 0.0],
                                                                                                      device=dev)
    env._as_actions = timed_part("as_actions", env._as_actions)
    env._io = timed_part("io", env._io)
    L = env.L

    class LW:  # rx_step timed (ctypes call: the C launch path)
        def __getattr__(self, k):
            f = getattr(L, k)
            return timed_part(k, f) if k == "rx_step" else f
    env.L = LW()
    env._launched = timed_part("launched", env._launched)
    it = [0]

    def one_step():
        k = it[0] % 248
        it[0] += 1
        with torch.cuda.stream(torch.cuda.current_stream(dev)):
            env.step_device(bank[k])

    out = []
    for region in range(4):
        for _ in range(50 if region == 0 else 20):
            one_step()
        if region == 1:
            gc.collect()
        torch.cuda.synchronize()
        _ = env.episode_stats()
        torch.cuda.synchronize()
        for v in T.values():
            v.clear()
        t0 = time.perf_counter()
        tk = []
        for _ in range(4):
            one_step()
            tk.append(time.perf_counter())
        torch.cuda.synchronize()
        out.append({"region": region, "step_host_us": [round((b - a) * 1e6, 1) for a, b in zip([t0] + tk, tk)],
                    "parts_us": {k: [round(x, 1) for x in v] for k, v in T.items()}})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
