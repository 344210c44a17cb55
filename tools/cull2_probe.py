import os, sys, json, torch
ROOT = "/root/repo" if os.path.exists("/root/repo/bench.py") else os.getcwd()
sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd")); sys.path.insert(0, ROOT)
from bench import seed1_pool
from rx.vector_env import RacingVectorEnv
for A in (1, 2):
    N = 1024
    pool, widths = seed1_pool(N)
    env = RacingVectorEnv(pool, widths, n_agents=A, device="cuda")
    env.reset_device()
    g = torch.Generator(device="cuda").manual_seed(0)
    shp = (N, A, 2) if A == 2 else (N, 2)
    for _ in range(50):
        env.step_device(torch.rand(shp, generator=g, device="cuda") * 2 - 1)
    env.enable_counters(); env._io_cache.clear()
    for _ in range(10):
        env.step_device(torch.rand(shp, generator=g, device="cuda") * 2 - 1)
    c = env.read_counters()
    print(A, {k: v / (10 * (N * (4 if A == 1 else 1) // 64)) for k, v in c.items()})
