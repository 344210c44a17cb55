"""Where the first step of a timed region loses ~150-350 us.

    python tools/first_launch_probe.py [envs]

The rocprofv3 trace of the 20-step bench (profiles/r03/trace20_window_*.json)
shows the timed kernels back to back with no gaps, but the FIRST kernel starting
167-356 us after the host's t0.  This probe separates host from device: after a
burn-in and a queue-draining sync, an idle of a given length, then one rx_step
bracketed by host clocks (the call's own duration = host launch cost) and HIP
events on the launch stream (device start-to-end), then the sync.  Repeated
for several idle lengths and for the first vs. the second step after the sync.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import seed1_pool  # noqa: E402
from rx.vector_env import RacingVectorEnv  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    pool, widths = seed1_pool(N)
    env = RacingVectorEnv(pool, widths, device="cuda", autoreset="next_step")
    env.reset_device()
    g = torch.Generator(device="cuda").manual_seed(0)
    bank = torch.rand((64, N, 2), generator=g, device="cuda") * torch.tensor([2.0, 1.0], device="cuda") \
        - torch.tensor([1.0, 0.0], device="cuda")
    for i in range(150):
        env.step_device(bank[i % 64])
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    rows = []
    k = 0
    for idle_ms in (0.0, 0.0, 1.0, 10.0, 100.0, 0.0, 100.0):
        torch.cuda.synchronize()
        if idle_ms:
            time.sleep(idle_ms / 1e3)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        t0 = time.perf_counter()
        ev[0].record(s)
        t1 = time.perf_counter()
        env.step_device(bank[k % 64])
        t2 = time.perf_counter()
        ev[1].record(s)
        ev[2].record(s)
        env.step_device(bank[(k + 1) % 64])
        t3 = time.perf_counter()
        ev[3].record(s)
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        k += 2
        rows.append({"idle_ms": idle_ms, "host_event_record_us": round((t1 - t0) * 1e6, 1),
                     "host_first_step_call_us": round((t2 - t1) * 1e6, 1),
                     "host_second_step_call_us": round((t3 - t2) * 1e6, 1),
                     "dev_first_step_us": round(ev[0].elapsed_time(ev[1]) * 1e3, 1),
                     "dev_second_step_us": round(ev[2].elapsed_time(ev[3]) * 1e3, 1),
                     "host_total_us": round((t4 - t0) * 1e6, 1)})
    print(json.dumps({"envs": N, "rows": rows}), flush=True)


if __name__ == "__main__":
    main()
