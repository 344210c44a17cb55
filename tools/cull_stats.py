"""Culling effectiveness on the bench workload: chunks tested vs scanned per wave."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))
sys.path.insert(0, ROOT)


def main():
    from bench import seed1_pool
    from rx.vector_env import RacingVectorEnv
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    pool, widths = seed1_pool(N)
    out = {}
    combos = [tuple(int(x) for x in c.split(",")) for c in sys.argv[2:]] or [(0, 0), (0, 1), (1, 0), (1, 16)]
    for order, sort in combos:
        env = RacingVectorEnv(pool, widths, device="cuda", sort_interval=sort, ray_order=order)
        env.reset_device()
        g = torch.Generator(device="cuda").manual_seed(0)
        for _ in range(30):
            a = torch.rand((N, 2), generator=g, device="cuda") * 2 - 1
            a[:, 1].abs_()
            env.step_device(a)
        env.enable_counters()
        steps = 20
        for _ in range(steps):
            a = torch.rand((N, 2), generator=g, device="cuda") * 2 - 1
            a[:, 1].abs_()
            env.step_device(a)
        c = env.read_counters()
        ray_waves = env.n_ray_waves * steps if hasattr(env, "n_ray_waves") else N * 11 / 64 * steps
        dyn_waves = N / 64 * steps  # k_dyn1: 64 / RX_DYN1_LPE envs per wave (LPE = 1)
        out[f"order{order}_sort{sort}"] = {"ray_chunks_tested_per_wave": c["ray_chunk_tests"] / ray_waves,
                              "ray_chunks_scanned_per_wave": c["ray_chunks_scanned"] / ray_waves,
                              "wp_chunks_tested_per_wave": c["wp_chunk_tests"] / dyn_waves,
                              "wp_chunks_scanned_per_wave": c["wp_chunks_scanned"] / dyn_waves}
        env.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
