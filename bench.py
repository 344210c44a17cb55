"""Headline benchmark: vectorised racing-env steps on MI355X (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs-per-gpu E] [--no-cpu-baseline]

Workload = BASELINE.json configs[2] ("65536 parallel single-agent envs,
1xMI355X"): the reference's seed-1 track pool (train.py:67-80:
random.seed(1); np.random.seed(1); gen_tracks(N, seed=1); widths
randint(6, 10); track_id = env index), 11 sensors, uniform random actions
pre-generated on the device (a bank resident in HBM before the timed region,
one slice per step), gymnasium next-step autoreset.  One bench "step" =
one env step of every env (random actions + rx_step) through ONE env handle
on one stream -- the configuration the PPO rollout uses, and the one whose
per-launch kernel timing the roofline is computed from.  --stream-groups G
steps the envs as G independent groups on G HIP streams instead (as an
asynchronous rollout would); the JSON also reports that throughput for G = 4
as "async_stream_groups", timed after the main region, and PPO training
throughput ("ppo_train": rollout + GAE + the 10 x 16 minibatch update, 4,096
envs per GPU; at N GPUs the update all-reduces one gradient+KL bucket per
optimizer step over RCCL).  With N GPUs
(torch.distributed.run, one rank per GPU) every rank owns 65,536 envs of a
N*65,536-env pool (weak scaling, configs[4]); the env step has no collective.

Prints ONE JSON line (rank 0).  ``roofline`` is for the dominant kernel
(k_rays, the raycast), timed live from per-wave device wall-clock stamps
(rx_profile: first wave start to last wave end, the span rocprofv3 reports); ``cpu_baseline`` times oracle/np_env.py -- the reference's NumPy step
restated (bit-exact vs the reference's golden vectors) -- on this host.
"""
import argparse
import gc
import json
import os
import random
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0     # MI355X HBM3E peak (MI355X_MICROARCH.md chip table)
FP64_VALU_PEAK_TF = 78.6  # MI355X FP64 vector peak (AMD spec)
# VALU issue peak: 256 CUs x 4 SIMDs, one wave64 VALU instruction per 4 cycles each (16 lanes; FP64 FMA is
# full rate: 1024 x 16 x 2 flop x 2.4 GHz = 78.6 TF), at 2.4 GHz
VALU_WAVE_INST_PEAK_G = 1024 * 2.4e9 / 4 / 1e9  # 614.4 G wave-instructions/s
RAY_FLOPS_PER_SEG = 13    # 2 sub, 3 dotp, 3 cross, 3 v1.v3, 2 div per ray x segment
RAYS_BYTES_PER_ENV = 24 + 11 * 4   # k_rays algorithmic HBM bytes/env: read x,y,angle (f64), write 11 f32 obs
STEP_BYTES_PER_ENV = 218           # whole step, SURVEY.md §8(d)


def seed1_pool(n_total):
    """train.py:67-80 track pool for n_total envs (rx.track.gen_tracks == reference, memoised)."""
    from rx.track import gen_tracks
    random.seed(1)
    np.random.seed(1)
    pool = gen_tracks(num_tracks=n_total, seed=1)
    widths = [np.random.randint(6, 10) for _ in range(n_total)]
    return pool, widths


def gae_roofline(n_envs, dev, T=128, reps=20):
    """k_gae (agent/ppo.py:134-154) on a [T, N] rollout: HBM-bound, 20 B per
    (t, env) element (read r, v, d; write A, R; f32) -- SURVEY.md §8(d)."""
    from rx.gae import compute_gae
    g = torch.Generator(device=dev).manual_seed(0)
    r = torch.randn((T, n_envs), generator=g, device=dev)
    v = torch.randn((T, n_envs), generator=g, device=dev)
    d = (torch.rand((T, n_envs), generator=g, device=dev) < 0.02).float()
    nv = torch.randn(n_envs, generator=g, device=dev)
    nd = torch.zeros(n_envs, device=dev)
    out = (torch.empty_like(r), torch.empty_like(r))
    for _ in range(3):
        compute_gae(r, d, v, nv, nd, 0.99, 0.95, out=out)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        compute_gae(r, d, v, nv, nd, 0.99, 0.95, out=out)
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / reps
    gbs = 20.0 * T * n_envs / (ms * 1e-3) / 1e9
    return {"kernel": "k_gae", "T": T, "N": n_envs, "avg_launch_ms": round(ms, 5), "bound": "hbm",
            "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS}


def cpu_baseline(pool, widths, budget_s=15.0, n_envs=16):
    """The reference's CPU execution model (NumPy step per env, sequential loop,
    16 envs = configs/base_config.py num_envs) on one host core, bounded in time."""
    from oracle.np_env import NpRacingEnv, NpSyncVectorEnv, NpTrack
    from rx.track import TrackGeometry
    envs = []
    geo = {}
    for i in range(n_envs):
        key = (id(pool[i]), widths[i])
        if key not in geo:
            g = TrackGeometry(pool[i], widths[i])
            geo[key] = NpTrack(g.waypoints, g.normals, g.segment_cache["starts"], g.segment_cache["v2"],
                               g.track_width, g.get_start_pos())
        envs.append(NpRacingEnv(geo[key], 11))
    venv = NpSyncVectorEnv(envs)
    venv.reset()
    rng = np.random.default_rng(0)
    steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        a = np.stack([rng.uniform(-1, 1, n_envs), rng.uniform(0, 1, n_envs)], 1).astype(np.float32)
        venv.step(a)
        steps += 1
    dt = time.perf_counter() - t0
    return {"value": round(steps * n_envs / dt, 1), "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": f"oracle/np_env.py NumPy restatement, {n_envs} envs x {steps} sequential steps "
                      f"({steps * n_envs} env-steps, {dt:.1f} s), seed-1 pool, random actions, 1 host core"}


def ppo_leg(world, rank, dev, dist, backend, envs_per_gpu, T, updates):
    """PPO training throughput (BASELINE.json configs[1] per GPU; configs[4]'s
    data-parallel update at N GPUs): rx.ppo.PPO on envs_per_gpu envs per rank,
    each update = T-step rollout with the fused policy in the loop + GAE + the
    reference's 10 epochs x 16 minibatches (KL early stop disabled so every
    update does the same work; device shuffles).  With N ranks every optimizer
    step all-reduces ONE bucket [flat gradient, KL] (42,256 B) over RCCL, plus
    one advantage-moment all-reduce per epoch (rx.dist)."""
    from rx.configs import base_config
    from rx.envs import RacingEnv
    from rx.ppo import PPO
    from rx.track import gen_tracks
    n = envs_per_gpu * world
    cfg = base_config(num_envs=n, num_steps=T, kl_target=1e9, shuffle="device")
    cfg["total_timesteps"] = (updates + 1) * cfg["batch_size"]
    random.seed(1)
    np.random.seed(1)
    pool = gen_tracks(n, seed=1)
    widths = [np.random.randint(6, 10) for _ in range(n)]
    t = PPO(lambda i: RacingEnv(11, pool, i, widths[i]), cfg, device=dev)
    it = t.train_iter()
    next(it)  # warm-up update (workspaces, first launches)

    def sync():
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
    sync()
    gc.collect()
    gc.disable()
    t0 = time.perf_counter()
    for _ in range(updates):
        next(it)
    sync()
    gc.enable()
    el = time.perf_counter() - t0
    if dist:
        x = torch.tensor([el], device=dev if backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        el = float(x.item())
    B = T * n
    c = t.config
    n_mb = c["num_minibatches"]
    t.envs.close()
    return {"value": round(B * updates / el, 1), "unit": "train env-steps/s", "updates": updates,
            "ms_per_update": round(el / updates * 1e3, 3), "envs_per_gpu": envs_per_gpu, "global_envs": n,
            "num_steps": T, "batch": B, "epochs_x_minibatches": f"{c['update_epochs']}x{n_mb}",
            "update_path": "fused HIP (rx_ppo_minibatch_grad" + ("_shard + bucket all-reduce)" if world > 1 else ")"),
            "allreduce_per_update": (c["update_epochs"] * (n_mb + 1) + 1) if world > 1 else 0,
            "allreduce_bucket_bytes": 4 * (t._flat.numel + 1) if world > 1 else 0,
            "note": "KL early stop off, device shuffles; timed after one warm-up update"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--envs-per-gpu", type=int, default=65536)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--cull-chunk", type=int, default=8, help="raycast chunk culling (0 = brute force)")
    ap.add_argument("--sort-interval", type=int, default=16, help="spatial env re-sort period (0 = never)")
    ap.add_argument("--ray-order", type=int, default=2,
                    help="raycast lane order (0 env-major, 1 ray-major, 2 direction-sorted tasks)")
    ap.add_argument("--cull-super", type=int, default=8, help="chunks per super-chunk box (0 = one-level culling)")
    ap.add_argument("--stream-groups", type=int, default=1,
                    help="independent env groups, one HIP stream each (1 = one handle on one stream)")
    ap.add_argument("--async-probe-groups", type=int, default=4,
                    help="after the timed region, also time the same workload as this many stream groups "
                         "(reported as 'async_stream_groups'; 0 = skip)")
    ap.add_argument("--no-kernel-profile", action="store_true",
                    help="time without per-launch timestamp events (no per-kernel durations)")
    ap.add_argument("--sample-every", type=int, default=16,
                    help="instrument every k-th timed step with per-kernel HIP events (1 = every step)")
    ap.add_argument("--ppo-updates", type=int, default=2,
                    help="also time this many PPO updates (configs[1] per GPU; 0 = skip), reported as 'ppo_train'")
    ap.add_argument("--ppo-envs-per-gpu", type=int, default=4096)
    ap.add_argument("--ppo-steps", type=int, default=128)
    ap.add_argument("--dist-backend", default="nccl",
                    help="process-group backend (nccl = RCCL; gloo only to rehearse N ranks on one GPU)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    ndev = torch.cuda.device_count()
    if args.dist_backend == "nccl" and local >= ndev:
        raise SystemExit(f"LOCAL_RANK {local} but only {ndev} GPUs visible")
    local_dev = local % max(ndev, 1)  # gloo rehearsal: several ranks may share one GPU
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    from rx.vector_env import RacingVectorEnv
    E = args.envs_per_gpu
    G = args.stream_groups
    if G < 1 or E % G:
        raise SystemExit(f"--stream-groups {G} must divide --envs-per-gpu {E}")
    n_total = E * world
    pool, widths = seed1_pool(n_total)
    lo = rank * E
    torch.manual_seed(1234 + rank)
    scale = torch.tensor([2.0, 1.0], device=dev)
    shift = torch.tensor([-1.0, 0.0], device=dev)

    def make_groups(G):
        """G independent env groups, each stepping on its own HIP stream (a group's
        step depends only on its own envs, so different groups' kernels overlap)."""
        n = E // G
        envs = [RacingVectorEnv(pool[lo + g * n:lo + (g + 1) * n], widths[lo + g * n:lo + (g + 1) * n], n_agents=1,
                                n_sensors=11, device=dev, autoreset="next_step", cull_chunk=args.cull_chunk,
                                sort_interval=args.sort_interval, ray_order=args.ray_order,
                                cull_super=args.cull_super)
                for g in range(G)]
        streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(device=dev) for _ in range(G - 1)]
        # synthetic inputs resident in HBM before the timed region: a bank of uniform random
        # actions (steer ~ U(-1, 1), throttle ~ U(0, 1)), one [n, 2] slice per step, cycled
        # when the run is longer than the bank (<= 512 MB per GPU)
        bank = max(1, min(args.steps + args.warmup, (512 << 20) // (8 * E)))
        acts = [torch.addcmul(shift, torch.rand((bank, n, 2), device=dev), scale) for _ in range(G)]
        for e in envs:
            e.reset_device()
        torch.cuda.synchronize(dev)
        it = [0]

        def one_step(ev=None):
            k = it[0] % bank
            it[0] += 1
            for g in range(G):
                with torch.cuda.stream(streams[g]):
                    if ev is None or g:  # the production call: one rx_step
                        envs[g].step_device(acts[g][k])
                    elif ev == "step":  # recorded production step (group 0)
                        envs[g].profile(2)
                        envs[g].step_device(acts[g][k])
                        envs[g].profile(0)
                    else:  # recorded split step (group 0): dynamics phase, then the raycast on its own
                        envs[g].profile(2)
                        envs[g].step_device(acts[g][k], phases=1)
                        envs[g].step_device(acts[g][k], phases=2)
                        envs[g].profile(0)
        return envs, one_step, n

    def timed(one_step, steps, events=None):
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        gc.collect()
        gc.disable()  # a full collection over the 65,536-track pool stalls the host for tens of ms
        t0 = time.perf_counter()
        for k in range(steps):
            one_step(events.get(k) if events else None)
        torch.cuda.synchronize()  # all streams
        gc.enable()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if dist:
            t = torch.tensor([el], device=dev if args.dist_backend == "nccl" else "cpu", dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    envs, one_step, n = make_groups(G)
    env0 = envs[0]
    n_slots = len(env0.tracks)
    S_of_env = 2 * np.diff(env0.tracks.arrays()["wp_off"])[env0.track_of_env]
    ray_flops_per_launch = float(np.sum(11 * S_of_env * RAY_FLOPS_PER_SEG))  # one launch = group 0's envs
    for _ in range(args.warmup):
        one_step()
    # kernel durations from the dispatch packets' own timestamps (rx_profile, what rocprofv3
    # reports) over the whole timed region; every --sample-every'th step launches the raycast
    # on its own (dynamics phase first), so the dominant kernel has its own duration
    half = max(1, args.sample_every // 2)
    events = {} if args.no_kernel_profile else \
        {k: ("split" if k % args.sample_every == 0 else "step") for k in range(args.steps) if k % half == 0}
    env0.profile(1)
    env0.profile(0)
    elapsed = timed(one_step, args.steps, events)
    prof = env0.profile_read()
    ray_ms = prof["k_rays"][0] if "k_rays" in prof else float("nan")
    ep = [sum(x) for x in zip(*(e.episode_stats() for e in envs))]
    for e in envs:
        e.close()
    async_probe = None
    Ga = args.async_probe_groups
    if Ga > 1 and E % Ga == 0 and Ga != G:
        a_envs, a_step, _ = make_groups(Ga)
        for _ in range(args.warmup):
            a_step()
        a_el = timed(a_step, args.steps)
        async_probe = {"groups": Ga, "envs_per_group": E // Ga, "value": round(n_total * args.steps / a_el, 1),
                       "ms_per_step": round(a_el / args.steps * 1e3, 4),
                       "note": "same workload as independent env groups on separate HIP streams (async rollout); "
                               "timed after the main region, not the headline value"}
        for e in a_envs:
            e.close()
    gae = gae_roofline(E, dev) if rank == 0 else None
    ppo = ppo_leg(world, rank, dev, dist, args.dist_backend, args.ppo_envs_per_gpu, args.ppo_steps,
                  args.ppo_updates) if args.ppo_updates > 0 else None

    if rank == 0:
        value = n_total * args.steps / elapsed
        achieved_gbs = RAYS_BYTES_PER_ENV * n / (ray_ms * 1e-3) / 1e9
        achieved_tf = ray_flops_per_launch / (ray_ms * 1e-3) / 1e12
        traffic = valu_insts = None
        pmc = os.path.join(ROOT, "profiles", "pmc_k_rays.json")
        if os.path.exists(pmc):
            try:
                pj = json.load(open(pmc))
                # PMC counts are per launch: only valid for launches of the same size
                if pj.get("envs_per_launch") == n:
                    traffic = pj.get("hbm_bytes_per_launch")
                    valu_insts = pj.get("valu_insts_per_launch")
            except (OSError, ValueError):
                traffic = None
        out = {
            "metric": "env-steps/sec (whole node) @65536 envs",
            "value": round(value, 1),
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": "configs[2]: 65536 single-agent racing envs per GPU (seed-1 gen_tracks pool, "
                                   "11 sensors, uniform random actions resident in HBM, next-step autoreset)",
                       "envs_per_gpu": E, "global_envs": n_total, "track_slots": n_slots,
                       "stream_groups": G, "envs_per_launch": n,
                       "raycast_cull_chunk": args.cull_chunk, "sort_interval": args.sort_interval,
                       "ray_order": args.ray_order, "cull_super": args.cull_super,
                       "kernel_timing": "per-wave device wall-clock stamps (rx_profile: first wave start .. last "
                                        "wave end) of group 0's kernels on every "
                                        f"{max(1, args.sample_every // 2)}th timed step; every "
                                        f"{args.sample_every}th step launches the raycast on its own",
                       "parallelism": f"env shards x{world}, no collective in the step"},
            "roofline": {"bound": "hbm", "kernel": "k_rays", "achieved": round(achieved_gbs, 3),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved_gbs / HBM_PEAK_GBS,
                         "traffic": traffic, "bytes_per_env": RAYS_BYTES_PER_ENV, "envs_per_launch": n,
                         "avg_launch_ms": round(ray_ms, 5)},
            # the raycast is VALU-issue bound: wave-level VALU instructions per launch (PMC SQ_INSTS_VALU,
            # profiles/pmc_k_rays.json) / launch time vs the chip's issue rate.  The SURVEY §8(d) algorithmic
            # flop count assumes every segment is tested (brute force); culling skips most of them, so that
            # rate is reported as an equivalent, not against the peak.
            "compute_roofline": {"bound": "valu_issue", "kernel": "k_rays",
                                 "achieved": round(valu_insts / (ray_ms * 1e-3) / 1e9, 1) if valu_insts else None,
                                 "peak": VALU_WAVE_INST_PEAK_G, "unit": "G wave-VALU-instructions/s",
                                 "frac": (valu_insts / (ray_ms * 1e-3) / 1e9 / VALU_WAVE_INST_PEAK_G)
                                 if valu_insts else None,
                                 "valu_insts_per_launch": valu_insts,
                                 "brute_force_equiv_tflops": round(achieved_tf, 3),
                                 "brute_force_flops_per_launch": ray_flops_per_launch},
            # production step = k_kin1 + k_step2 (REWARD half beside the raycast); sampled steps run
            # k_kin1 + k_step2_reward (REWARD half alone) + k_rays (raycast alone)
            "kernels_ms": {k: round(v[0], 5) for k, v in prof.items()},
            "kernel_launches": {k: v[1] for k, v in prof.items()},
            "gae": gae,
            "episodes_ended": ep[2],
            "async_stream_groups": async_probe,
            "ppo_train": ppo,
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(pool, widths, budget_s=args.cpu_budget)
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
