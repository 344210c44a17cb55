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
asynchronous rollout would); the JSON also reports that throughput for G = 2
as "async_stream_groups", timed after the main region, and PPO training
throughput ("ppo_train": rollout + GAE + the 10 x 16 minibatch update, 4,096
envs per GPU; at N GPUs the update all-reduces one gradient+KL bucket per
optimizer step over RCCL; "ppo_train_bf16" is the same leg with the bf16
policy kernels, BASELINE configs[1] as named, at N = 1).  With N GPUs
(torch.distributed.run, one rank per GPU) every rank owns 65,536 envs of a
N*65,536-env pool (weak scaling, configs[4]); the env step has no collective.

Order of a run: CPU baseline (host only, before the GPU is touched), at
least --burn-in untimed steps (the steady state: cars spread over their tracks,
episodes ending and resetting), the timed region of --steps production steps
(one rx_step each, nothing instrumented), then --profile-steps instrumented
steps whose per-wave device wall-clock stamps (rx_profile: first wave start
to last wave end, the span rocprofv3 reports) give the kernel durations.

Prints ONE JSON line (rank 0).  ``roofline`` is for the dominant production
kernel, k_step2 (REWARD half beside the raycast), with its algorithmic bytes;
``compute_roofline`` is its VALU busy fraction from the committed steady-state
PMC counts (profiles/r06/pmc_steady.json, same launch size); ``cpu_baseline``
times oracle/np_env.py -- the reference's NumPy step restated (bit-exact vs
the reference's golden vectors) -- on this host's cores; ``time_to_90`` is the
second half of the metric (PPO wall-clock to 90 % success, evaluate.py
protocol) at the reference config and at configs[1].
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
RAYS_BYTES_PER_ENV = 24 + 11 * 4   # k_rays algorithmic HBM bytes/env: read x,y,angle (f64), write 11 f32 obs
# k_step2 algorithmic HBM bytes/env: REWARD half reads x, y, vx, vy, progress, last_progress,
# ep_return (f64), steps, ep_length (i32), flags, env_flags (u8) = 74 B with the raycast's angle; writes progress,
# last_progress, ep_return (f64), ep_length (i32), flags, env_flags, reward, done (f32) = 38 B; raycast writes
# 11 f32 obs = 44 B
STEP2_BYTES_PER_ENV = 74 + 38 + 44
STEP_BYTES_PER_ENV = 218           # whole step, SURVEY.md §8(d)
PMC_FILE = os.path.join(ROOT, "profiles", "r06", "pmc_steady.json")


def load_pmc(n):
    """Per-launch PMC counts of the production kernels (rocprofv3, tools/pmc.sh) committed
    under profiles/: valid only for launches of the same size and the steady state
    (the bench's own state distribution after its burn-in)."""
    try:
        pj = json.load(open(PMC_FILE))
    except (OSError, ValueError):
        return {}
    if pj.get("envs_per_launch") != n:
        return {}
    out = {k: v for k, v in pj.items() if isinstance(v, dict)}
    out["source"] = "profiles (steady state): " + os.path.relpath(PMC_FILE, ROOT)
    return out


FP64_VECTOR_PEAK_TFLOPS = 78.6   # MI355X FP64 vector
FP32_VECTOR_PEAK_TFLOPS = 157.3  # MI355X FP32 vector (MI355X_MICROARCH.md chip table)
# brute-force (unculled) f64 flops of one single-agent env-step at P = 11
# sensors -- every ray tested against all S boundary segments, 5 full argmin scans
ALGO_UNCULLED_FLOP_PER_ENV_STEP = 102830
F64_KEYS = ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64")
F32_KEYS = ("SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_TRANS_F32")


def _flop(c, keys):
    """FLOP of a launch from its wave-level VALU instruction counts: 64 lanes x
    (add + mul + transcendental + 2 x fma).  An upper bound (full exec mask)."""
    if not all(k in c for k in keys):
        return None
    add, mul, fma, trans = (c[k] for k in keys)
    return 64.0 * (add + mul + trans + 2.0 * fma)


def compute_roofline(pmc, launch_ms, n, waves=None):
    """The §8(d) compute roofline of the VALU-bound env step (SURVEY.md:456-457):
    EXECUTED FP64 flops per launch from the committed steady-state PMC counts
    (SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64, same launch size) over the LIVE
    launch duration, against the 78.6 TF FP64 vector peak; the brute-force
    count of §8(d) alongside as the algorithmic (unculled) work -- the culled
    kernel executes far less of it, bit-exactly.  Also the VALU busy fraction
    (SQ_ACTIVE_INST_VALU quad-cycles x 4 over 1,024 SIMDs x the launch's cycles,
    GRBM_GUI_ACTIVE / 8 XCDs) and the live wave-slot utilisation of the
    recorded production launches."""
    res = {"bound": "valu-fp64", "kernel": "k_step2", "source": pmc.get("source"), "envs_per_launch": n,
           "peak": FP64_VECTOR_PEAK_TFLOPS, "unit": "TFLOP/s",
           "fp64_flop_per_env_step_algorithmic_unculled": ALGO_UNCULLED_FLOP_PER_ENV_STEP,
           "flop_note": "executed flops = 64 lanes x (add + mul + trans + 2 fma) wave instructions (PMC, an upper "
                        "bound: full exec mask); algorithmic_unculled = SURVEY.md §8(d) brute force (every segment "
                        "of every ray, full argmin scans)"}
    per_env = 0.0
    for k, t in launch_ms.items():
        c = pmc.get(k, {})
        d = {"launch_ms_live": round(t, 5) if np.isfinite(t) else None}
        act, gui = c.get("SQ_ACTIVE_INST_VALU"), c.get("GRBM_GUI_ACTIVE")
        if act is not None and gui is not None:
            cycles = gui / 8.0  # GRBM_GUI_ACTIVE: summed over the 8 XCDs
            d.update(valu_busy_frac=round(4.0 * act / (1024.0 * cycles), 4), launch_cycles=round(cycles),
                     valu_insts_per_launch=c.get("SQ_INSTS_VALU"))
        f64, f32 = _flop(c, F64_KEYS), _flop(c, F32_KEYS)
        if f64 is not None:
            d["fp64_flop_per_launch"] = round(f64)
            d["fp64_flop_per_env"] = round(f64 / n, 1)
            if k != "k_rays":
                per_env += f64 / n
            if np.isfinite(t) and t > 0:
                tf = f64 / (t * 1e-3) / 1e12
                d["fp64_achieved_tflops"] = round(tf, 3)
                d["fp64_frac"] = round(tf / FP64_VECTOR_PEAK_TFLOPS, 4)
        if f32 is not None:
            d["fp32_flop_per_launch"] = round(f32)
            if np.isfinite(t) and t > 0:
                tf = f32 / (t * 1e-3) / 1e12
                d["fp32_achieved_tflops"] = round(tf, 3)
                d["fp32_frac"] = round(tf / FP32_VECTOR_PEAK_TFLOPS, 4)
        res[k] = d
    s2 = res.get("k_step2", {})
    if "fp64_frac" in s2:
        res["achieved"] = s2["fp64_achieved_tflops"]
        res["frac"] = s2["fp64_frac"]
        res["fp64_flop_per_env_step_executed"] = round(per_env, 1)
        res["executed_over_unculled"] = round(per_env / ALGO_UNCULLED_FLOP_PER_ENV_STEP, 4)
    res["valu_busy_frac"] = s2.get("valu_busy_frac")
    if waves:
        res["wave_slots"] = waves
        res["wave_slot_utilisation"] = waves.get("wave_slot_utilisation")
    return res


def wave_slots(env, n_launches, max_step2=16):
    """Live wave-slot view of the recorded production k_step2 launches (rx_profile
    per-wave stamps): utilisation = summed wave time / (8,192 slots x span), the
    drain after the active waves fall below half the slots, the last wave start,
    and the ray-wave duration / end by class (tools/wave_profile.py summarize)."""
    from tools.wave_profile import summarize
    sched = env.schedule()
    n_rw = sched["reward_lpe"] * ((sched["dyn_waves"] + 7) // 8 * 8)
    tab = env.ray_wave_table()
    got = []
    for k in range(n_launches):
        try:
            st, en, kind, _ = env.profile_waves(k)
        except Exception:  # noqa: BLE001 -- past the record
            break
        if kind == "k_step2":
            got.append(summarize(st, en, n_rw, tab["cls"], tab["sub"]))
            if len(got) >= max_step2:
                break
    if not got:
        return None
    m = lambda key: round(float(np.mean([g[key] for g in got])), 3)  # noqa: E731
    classes = sorted(got[0].get("ray_dur_us_by_class", {}))
    return {"launches": len(got), "span_us": m("span_us"), "wave_slot_utilisation": m("wave_slot_utilisation"),
            "tail_after_half_slots_us": m("tail_after_half_slots_us"), "last_wave_start_us": m("last_wave_start_us"),
            "ray_dur_us_by_class": {j: round(float(np.mean([g["ray_dur_us_by_class"][j] for g in got])), 2)
                                    for j in classes},
            "ray_end_us_by_class_max": {j: round(float(np.mean([g["ray_end_us_by_class_max"][j] for g in got])), 2)
                                        for j in classes},
            "slots": 8192, "source": "live: rx_profile per-wave stamps of the instrumented production launches"}


_MARKS = os.environ.get("RX_BENCH_MARKS") == "1"


def mark(tag):
    """Diagnostics (RX_BENCH_MARKS=1): host clocks at the edges of a timed region on
    stderr, to line the region up with a rocprofv3 kernel trace (CLOCK_BOOTTIME
    and CLOCK_MONOTONIC ns).  Outside the timed interval; changes nothing timed."""
    if _MARKS:
        print(f"RX_MARK {tag} boottime_ns={time.clock_gettime_ns(time.CLOCK_BOOTTIME)} "
              f"monotonic_ns={time.monotonic_ns()}", file=sys.stderr, flush=True)


def seed1_pool(n_total):
    """train.py:67-80 track pool for n_total envs (rx.track.gen_tracks == reference, memoised)."""
    from rx.track import gen_tracks
    random.seed(1)
    np.random.seed(1)
    pool = gen_tracks(num_tracks=n_total, seed=1)
    widths = [np.random.randint(6, 10) for _ in range(n_total)]
    return pool, widths


def stress_pool(n, seed=2):
    """SURVEY.md §8(d) stress variant: all-distinct tracks.  environment/track.py:47-56
    with seed=None draws every track's parameters (P in [10, 14]) and points from the
    global RNG without the per-track reseed (track.py:5-6) that collapses a seeded pool
    to 7 slots; widths randint(6, 10) as train.py:79."""
    from rx.track import gen_tracks
    np.random.seed(seed)
    pool = gen_tracks(num_tracks=n, seed=None)
    widths = [np.random.randint(6, 10) for _ in range(n)]
    return pool, widths


def _stress_run(env, dev, n, steps, untimed, profile_steps):
    """One env handle through the headline protocol: untimed steps, a HIP graph of
    `steps` production steps captured and replayed once untimed, one timed replay,
    then instrumented steps (kernel durations, wave slots) and counter steps."""
    g = torch.Generator(device=dev).manual_seed(4321)
    bank = max(1, min(steps + untimed + profile_steps, (256 << 20) // (8 * n)))
    acts = torch.rand((bank, n, 2), device=dev, generator=g) * torch.tensor([2.0, 1.0], device=dev) + \
        torch.tensor([-1.0, 0.0], device=dev)
    it = [0]

    def run(K):
        while K > 0:
            k = it[0] % bank
            m = min(K, bank - k)
            env.steps_device(acts[k:k + m])
            it[0] += m
            K -= m
    env.reset_device()
    run(untimed)
    torch.cuda.synchronize(dev)
    cap = torch.cuda.Stream(device=dev)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=cap, capture_error_mode="thread_local"):
        run(steps)
    graph.replay()  # untimed: upload + K more burn-in steps
    torch.cuda.synchronize(dev)
    env.episode_stats()
    gc.collect()
    gc.disable()
    t1 = time.perf_counter()
    graph.replay()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t1
    gc.enable()
    ep = env.episode_stats()
    env.profile(1)
    run(profile_steps)
    env.profile(0)
    torch.cuda.synchronize(dev)
    prof = env.profile_read()
    waves = wave_slots(env, profile_steps * 2)
    env.enable_counters(True)
    run(8)
    torch.cuda.synchronize(dev)
    cnt = env.read_counters()
    env.enable_counters(False)
    sch = env.schedule()
    del graph
    step2 = prof.get("k_step2", (float("nan"), 0))[0]
    kin = prof.get("k_kin1", (float("nan"), 0))[0]
    gbs = STEP2_BYTES_PER_ENV * n / (step2 * 1e-3) / 1e9
    return {"value": round(n * steps / el, 1), "ms_per_step": round(el / steps * 1e3, 4),
            "episodes_ended_in_timed_region": ep[2], "lane_tracks": sch["lane_tracks"],
            "kernels_ms": {k: round(v[0], 5) for k, v in prof.items()},
            "roofline": {"bound": "hbm", "kernel": "k_step2", "achieved": round(gbs, 3), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS, "bytes_per_env": STEP2_BYTES_PER_ENV,
                         "avg_launch_ms": round(step2, 5), "step_kernels_ms": round(step2 + kin, 5)},
            "wave_slot_utilisation": waves.get("wave_slot_utilisation") if waves else None,
            "wave_slots": waves,
            "executed_work": {"ray_box_tests_per_ray_wave": round(cnt["ray_chunk_tests"] / (8 * sch["ray_waves"]), 2),
                              "ray_leaf_scans_per_env_step": round(cnt["ray_chunks_scanned"] / (8 * n), 3),
                              "wp_leaf_scans_per_env_step": round(cnt["wp_chunks_scanned"] / (8 * n), 3),
                              "counted": "per lane" if sch["lane_tracks"] else "per wave"},
            "schedule": sch}


def stress_leg(dev, n, steps, untimed, sched, profile_steps=32, seed=2, compare=True):
    """The headline workload (configs[2]: n single-agent envs, uniform random actions
    resident in HBM, next-step autoreset, one HIP graph of `steps` production steps)
    on the all-distinct-track pool of stress_pool: every env its own track slot.  The
    line's numbers come from the schedule rx_assign picks (lane-varying slots);
    ``compare`` also times the slot-grouped schedule (lane_tracks = -1: one env per
    wave) on the same pool, the form the kernels had before ABI v23."""
    from rx.track import TrackSet
    from rx.vector_env import RacingVectorEnv
    t0 = time.perf_counter()
    pool, widths = stress_pool(n, seed)
    ts = TrackSet.build(pool, widths)
    build_s = time.perf_counter() - t0
    P = np.bincount([len(c) for c in pool], minlength=15)[10:15]
    env = RacingVectorEnv(pool, widths, n_agents=1, n_sensors=11, device=dev, autoreset="next_step", track_set=ts,
                          sched=sched)
    n_slots = len(env.tracks)
    res = _stress_run(env, dev, n, steps, untimed, profile_steps)
    env.close()
    if compare:
        env = RacingVectorEnv(pool, widths, n_agents=1, n_sensors=11, device=dev, autoreset="next_step",
                              track_set=ts, sched=dict(sched, lane_tracks=-1))
        r2 = _stress_run(env, dev, n, steps, untimed, profile_steps)
        env.close()
        res["slot_grouped"] = {k: r2[k] for k in ("value", "ms_per_step", "kernels_ms", "wave_slot_utilisation",
                                                  "roofline", "executed_work")}
    res.update(unit="env-steps/s", envs=n, track_slots=n_slots, control_points_hist_P10_to_P14=P.tolist(),
               steps=steps, table_build_s=round(build_s, 2),
               workload=f"configs[2] on the stress pool: np.random.seed({seed}); gen_tracks({n}, seed=None) "
                        "(track.py:47-56, no per-track reseed), widths randint(6, 10): every env its own track; "
                        "uniform random actions resident in HBM, next-step autoreset, one HIP graph replay of "
                        f"{steps} steps after {untimed} + {steps} untimed")
    return res


def gae_roofline(n_envs, dev, T=512, reps=20):
    """k_gae (agent/ppo.py:134-154) on a [T, N] rollout: HBM-bound, 20 B per
    (t, env) element (read r, v, d; write A, R; f32) -- SURVEY.md §8(d).  At the
    default T = 512 the five [T, N] arrays (65,536 envs: 671 MB) exceed the
    256 MiB Infinity Cache, so replaying the same buffers measures HBM; at
    T = 128 (168 MB) they stay cache-resident (reported as such)."""
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
    ws = 20 * T * n_envs
    return {"kernel": "k_gae", "T": T, "N": n_envs, "avg_launch_ms": round(ms, 5), "bound": "hbm",
            "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
            "working_set_bytes": ws,
            "residency": "exceeds the 256 MiB Infinity Cache: HBM" if ws > (256 << 20) else
                         "fits the 256 MiB Infinity Cache: L3-assisted, not an HBM figure"}


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(pool, widths, budget_s=12.0, n_envs=16):
    """BASELINE.md §3 CPU baseline on this host: oracle/np_env.py (the reference's
    NumPy step restated, bit-exact vs the reference's golden vectors).

    Mode B (the reported value): one process per host core, one env each
    (OPENBLAS_NUM_THREADS=1), aggregate env-steps/s.  Cores = the CPUs this
    process may run on (sched_getaffinity), capped by OMP_NUM_THREADS where the
    host sets it (the GPU box exposes the whole machine's CPUs but gives one
    GPU's job a 16-core share).  Mode A: the reference's plumbing, one process
    stepping 16 envs sequentially (SyncVectorEnv, configs/base_config.py)."""
    from oracle.cpu_baseline import np_envs, run_workers
    from oracle.np_env import NpSyncVectorEnv
    aff = len(os.sched_getaffinity(0))
    cap = os.environ.get("OMP_NUM_THREADS")
    cores = min(aff, int(cap)) if cap and cap.isdigit() and int(cap) > 0 else aff
    # Mode A
    venv = NpSyncVectorEnv(np_envs(pool, widths, n_envs))
    venv.reset()
    rng = np.random.default_rng(0)
    steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s / 2:
        a = np.stack([rng.uniform(-1, 1, n_envs), rng.uniform(0, 1, n_envs)], 1).astype(np.float32)
        venv.step(a)
        steps += 1
    dt = time.perf_counter() - t0
    mode_a = {"value": round(steps * n_envs / dt, 1), "unit": "env-steps/s", "cores": 1,
              "sample": f"{n_envs} envs x {steps} sequential steps ({steps * n_envs} env-steps, {dt:.1f} s)"}
    # Mode B: torch-free child processes (oracle/cpu_baseline.py), each exits 0 on its own
    res = run_workers([(pool[i % len(pool)], widths[i % len(pool)], budget_s, i) for i in range(cores)],
                      timeout_s=budget_s + 600)
    tot = sum(r[0] for r in res)
    el = max(r[1] for r in res)
    return {"value": round(tot / el, 1), "unit": "env-steps/s", "cores": cores, "kind": "port",
            "cpu_model": _cpu_model(), "sched_getaffinity": aff,
            "sample": f"oracle/np_env.py NumPy restatement of RacingEnv.step (bit-exact vs the reference's golden "
                      f"vectors), Mode B: {cores} processes x 1 env, {tot} env-steps in {el:.1f} s, seed-1 pool, "
                      f"uniform random actions, OPENBLAS_NUM_THREADS=1",
            "workers": "python -m oracle.cpu_baseline child processes (numpy/scipy only, never torch or HIP), "
                       "each exits 0 on its own",
            "mode_a_one_core_16_envs": mode_a}


def time_to_90(configs, seeds=(1, 2, 3)):
    """Second half of BASELINE.json's metric: PPO wall-clock to 90 % success
    (evaluate.py protocol; tools/time_to_success.py), training time only, as a
    distribution over ``seeds`` (config["seed"]: the track pool, the initial
    policy and the sampling streams all change with it, as in train.py).
    build_s = PPO construction (env table upload, agent, flat buffers), which
    the training time excludes."""
    from tools.time_to_success import run as tts
    out = []
    for cfg in configs:
        ne, ns, shuffle = cfg[:3]
        pdt = cfg[3] if len(cfg) > 3 else "fp32"
        runs = []
        for sd in seeds:
            r = tts(num_envs=ne, num_steps=ns, eval_every=1, device_shuffle=shuffle == "device", max_minutes=1.0,
                    quiet=True, seed=sd, policy_dtype=pdt)
            runs.append({"seed": sd, "value_s": r["value_s"], "build_s": r["build_s"],
                         "reached_at_step": r["reached_at_step"], "updates": len(r["curve"]),
                         "success_rate": r["curve"][-1].get("success_rate") if r["curve"] else None})
        vals = sorted(x["value_s"] for x in runs if x["value_s"] is not None)
        dist = {"min": vals[0], "median": vals[len(vals) // 2] if len(vals) % 2 else
                round(0.5 * (vals[len(vals) // 2 - 1] + vals[len(vals) // 2]), 4), "max": vals[-1]} if vals else None
        out.append({"num_envs": ne, "num_steps": ns, "shuffle": shuffle, "policy_dtype": pdt, "value_s": dist,
                    "reached": f"{len(vals)}/{len(runs)} seeds", "runs": runs})
    return {"metric": "PPO wall-clock to 90% success rate", "unit": "s", "higher_is_better": False,
            "protocol": "evaluate.py: 40 tracks (seed 42) x 5 runs, widths by run, <= 2000 steps, stochastic "
                        "policy, evaluated after every update; training time only (evaluations and PPO "
                        "construction, build_s, excluded); min / median / max over config seeds",
            "configs": out}


# Algorithmic flops of one minibatch row through k_ppo_grad (both trunks,
# agent/ppo.py:11-62 + the backward of :183-203): forward 2(15*64 + 64*64 +
# 64*n_out), backward dZ2 / dW3 2*64*n_out each, dW2 / dH1 2*64*64 each, dW1
# 2*64*15; actor (n_out 2) 29,184 + critic (n_out 1) 28,800.
PPO_GRAD_FLOP_PER_ROW = 57984
FP32_MATRIX_PEAK_TFLOPS = 157.3  # MI355X dense FP32 MFMA
BF16_MATRIX_PEAK_TFLOPS = 2500.0  # MI355X dense BF16 MFMA (no sparsity)


def ppo_grad_roofline(t, dev, reps=160):
    """Live MFMA roofline of the PPO minibatch gradient: ``reps`` back-to-back
    rx_ppo_minibatch_grad calls (k_ppo_grad + its split-K k_ppo_reduce) over
    the last update's batch, bracketed by HIP events on the launch stream.
    k_ppo_reduce is inside the timed launches, so ``frac`` is a lower bound
    for k_ppo_grad alone (its rocprofv3 share: profiles/r02/ppo_prof_fp32_kernel_stats.csv)."""
    ents = [e for e in t.__dict__.get("_upd_graphs", {}).values() if e.fused is not None]
    if not ents:
        return None
    f = ents[-1].fused
    stop = torch.zeros(1, dtype=torch.bool, device=dev)  # KL target 1e9: never raised
    kl = torch.zeros(1, dtype=torch.float32, device=dev)
    for m in range(f.n_mb):
        f.grad(m, stop, kl)
    s = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    e0.record(s)
    for i in range(reps):
        f.grad(i % f.n_mb, stop, kl)
    e1.record(s)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    tf = PPO_GRAD_FLOP_PER_ROW * f.mb / (ms * 1e-3) / 1e12
    prec = t.config.get("policy_dtype", "fp32")
    peak = BF16_MATRIX_PEAK_TFLOPS if prec == "bf16" else FP32_MATRIX_PEAK_TFLOPS
    return {"bound": "mfma", "kernel": "k_ppo_grad + k_ppo_reduce", "precision": prec,
            "flop_per_row": PPO_GRAD_FLOP_PER_ROW, "rows_per_launch": f.mb, "avg_launch_ms": round(ms, 5),
            "achieved": round(tf, 2), "peak": peak, "unit": "TFLOP/s", "frac": round(tf / peak, 4),
            "note": f"live HIP events over {reps} back-to-back minibatch gradient calls; includes k_ppo_reduce, "
                    "so frac is a lower bound for k_ppo_grad alone"}


def ppo_leg(world, rank, dev, dist, backend, envs_per_gpu, T, updates, policy_dtype="fp32", extra=None):
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
    cfg = base_config(num_envs=n, num_steps=T, kl_target=1e9, shuffle="device", policy_dtype=policy_dtype,
                      **(extra or {}))
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
    from rx import dist as rdist
    ar0 = dict(rdist.COUNTS)
    t0 = time.perf_counter()
    for _ in range(updates):
        next(it)
    sync()
    gc.enable()
    el = time.perf_counter() - t0
    ar = {k: (rdist.COUNTS[k] - ar0[k]) / updates for k in ar0}
    if dist:
        x = torch.tensor([el], device=dev if backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        el = float(x.item())
    B = T * n
    c = t.config
    n_mb = c["num_minibatches"]
    dp_ranks = None
    if dist:  # what every rank ran: the epoch's launch form (rdist.capture_all_or_none) and its all-reduces
        me = {"rank": rank, "graph_dp": dict(rdist.GRAPH_DP), "allreduce_per_update": ar["all_reduce"],
              "allreduce_bytes_per_update": ar["bytes"]}
        dp_ranks = [None] * world
        dist.all_gather_object(dp_ranks, me)
    grad_rf = ppo_grad_roofline(t, dev) if world == 1 else None
    t.envs.close()
    return {"value": round(B * updates / el, 1), "unit": "train env-steps/s", "updates": updates,
            "grad_roofline": grad_rf,
            "ms_per_update": round(el / updates * 1e3, 3), "envs_per_gpu": envs_per_gpu, "global_envs": n,
            "num_steps": T, "batch": B, "epochs_x_minibatches": f"{c['update_epochs']}x{n_mb}",
            "update_path": "fused HIP (rx_ppo_minibatch_grad" + ("_shard + bucket all-reduce)"
                                                                if world > 1 or c.get("shard_update") else ")"),
            "allreduce_per_update": ar["all_reduce"], "allreduce_bytes_per_update": ar["bytes"],
            "allreduce_per_update_expected": (c["update_epochs"] * (n_mb + 1) + 1) if world > 1 else 0,
            "allreduce_bucket_bytes": 4 * (t._flat.numel + 1) if world > 1 else 0,
            "dp_ranks": dp_ranks,
            "note": "KL early stop off, device shuffles; timed after one warm-up update"}


def rccl_world1_leg(dev, envs, T, updates):
    """the data-parallel update priced on ONE GPU before the driver's
    8-GPU run -- a 1-rank RCCL process group, the shard path forced (config
    shard_update: per epoch rx_ppo_adv_moments -> RCCL all-reduce -> finalize, per
    optimizer step rx_ppo_minibatch_grad_shard -> RCCL all-reduce of the 42 KB
    [gradient, KL] bucket -> rx_ppo_kl_check -> rx_adam_clip_step) with the
    collectives really issued (rx.dist.FORCE_COLLECTIVES), as ONE captured HIP
    graph per epoch (graph_dp) and as eager launches.  Beside ppo_train (the
    single-rank fused update) it is the floor of the data-parallel overhead."""
    import torch.distributed as td
    from rx import dist as rdist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    td.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    rdist.FORCE_COLLECTIVES["on"] = True
    out = {}
    try:
        for graph in (True, False):
            rdist.GRAPH_DP.clear()
            rdist.GRAPH_DP.update(captured=None, error=None)
            r = ppo_leg(1, 0, dev, None, "nccl", envs, T, updates, extra=dict(shard_update=True, graph_dp=graph))
            out["graph" if graph else "eager"] = {k: r[k] for k in ("value", "ms_per_update", "allreduce_per_update",
                                                                    "allreduce_bytes_per_update", "update_path")}
            if graph:
                out["graph_capture"] = dict(rdist.GRAPH_DP)
        out.update(unit="train env-steps/s", backend="nccl (RCCL), world size 1",
                   rccl=".".join(str(v) for v in torch.cuda.nccl.version()),
                   note="collectives issued at world size 1 (no peer traffic): the launch / collective sequence "
                        "of the data-parallel update on one GPU; allreduce_per_update counts Python-issued "
                        "all-reduces (a graph replay issues its captured ones without Python)")
    finally:
        rdist.FORCE_COLLECTIVES["on"] = False
        td.destroy_process_group()
    return out


def selfplay_leg(dev, envs, T, updates, pool_size=5):
    """BASELINE.json configs[3]: two-car self-play PPO (agent/self_play_ppo.py:70-187)
    at ``envs`` envs with an opponent pool of ``pool_size``: rx.selfplay.SelfPlayPPO's
    own train_iter (pool advance, opponent draw + env rebuild, rollout with the
    frozen opponent's rx_policy_act in the loop, GAE, the 10 x 16 fused update).
    The snapshot cadence is shortened to every update while the pool fills
    (pool_size snapshots, FIFO), then set back to the reference's 15 for the timed
    updates (a snapshot -- one device deepcopy of the policy, ~1 ms -- every 15th
    update, as configs[3] runs); KL early stop off and device shuffles so every
    update does the same work; no checkpoint files.
    Then one more update with a sync between phases gives the split."""
    from rx.configs import self_play_config
    from rx.envs import MultiRacingEnv
    from rx.selfplay import SelfPlayPPO
    from rx.track import gen_tracks
    warm = pool_size + 1
    cfg = self_play_config(num_envs=envs, num_steps=T, kl_target=1e9, shuffle="device", snapshot_freq=1,
                           pool_size=pool_size, checkpoint=False)
    cfg["total_timesteps"] = (warm + updates + 2) * cfg["batch_size"]
    random.seed(1)
    np.random.seed(1)
    torch.manual_seed(1)
    pool = gen_tracks(envs, seed=1)
    widths = [np.random.randint(6, 10) for _ in range(envs)]
    t = SelfPlayPPO(lambda i: MultiRacingEnv(2, 11, pool, i, widths), cfg, device=dev)
    it = t.train_iter()
    for _ in range(warm):  # pool filled, graphs captured, workspaces sized
        next(it)
    torch.cuda.synchronize()
    pool_before = len(t.opponent_pool)
    t.snapshot_freq = 15  # self_play_config's cadence (agent/self_play_ppo.py:115-122) from here on
    taken = [0]  # snapshots the timed updates really take (an update index that is a multiple of 15)
    snap0 = t.snapshot_agent

    def counted():
        taken[0] += 1
        return snap0()
    t.snapshot_agent = counted
    gc.collect()
    gc.disable()
    t0 = time.perf_counter()
    for _ in range(updates):
        next(it)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    gc.enable()
    t.snapshot_agent = snap0
    # the reference cadence's snapshot, amortised: updates / 15 snapshots belong to the timed
    # updates; the ones they took are inside `el` already, the rest (one snapshot_agent(),
    # timed here, synced) are added -- never counted twice
    ts = time.perf_counter()
    t.snapshot_agent()
    torch.cuda.synchronize()
    snap_s = time.perf_counter() - ts
    el += max(0.0, updates / t.snapshot_freq - taken[0]) * snap_s
    # phase split of one more update of the same loop (same buffers and graphs), a device
    # sync at every phase boundary (SelfPlayPPO.phase_ms)
    t.phase_ms = {}
    next(it)
    ph = dict(t.phase_ms)
    t.phase_ms = None
    ph["rollout_env_steps_per_s"] = round(T * envs / (ph["rollout_ms"] * 1e-3), 1)
    B = T * envs
    res = {"value": round(B * updates / el, 1), "unit": "train env-steps/s (agent-steps = 2x)", "updates": updates,
           "ms_per_update": round(el / updates * 1e3, 3), "envs": envs, "cars_per_env": 2, "num_steps": T,
           "batch": B, "pool_size": pool_size, "pool_filled_before_timing": pool_before,
           "opponent": "frozen pool snapshot, one rx_policy_act launch per step over all envs",
           "phase_split_one_update": ph,
           "snapshot_freq_timed": t.snapshot_freq, "snapshot_ms_amortised": round(snap_s * 1e3, 3),
           "snapshots_taken_in_timed_updates": taken[0],
           "note": "BASELINE configs[3]; snapshot every update until the pool is full, then the reference's every 15 "
                   "updates; KL early stop off, device shuffles, no checkpoint files; timed after the pool-filling "
                   "updates"}
    t.envs.close()
    return res


def _lib_path():
    from rx import _lib
    return _lib.load()._name


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(n, argv, poll_s=0.2):
    """`python bench.py --gpus N` without an external launcher: start N fresh
    rank processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, rendezvous on
    127.0.0.1), one per GPU, exactly as `torch.distributed.run --nproc-per-node N`
    would.  This parent never initialises HIP (it has only parsed arguments), and
    it starts the ranks as children -- no exec.  Rank 0's JSON line is relayed
    to this process's stdout; everything else the ranks print (library chatter
    such as gloo's connection messages included) goes to stderr, so stdout
    carries the one line.  If any rank fails, the others are terminated (their
    own PIDs) and its exit code is returned."""
    import subprocess
    import threading
    port = _free_port()
    me = os.path.abspath(__file__)
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, me] + list(argv), env=env, text=True,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno()))

    def relay(f):
        for line in f:
            (sys.stdout if line.startswith("{") else sys.stderr).write(line)
            sys.stdout.flush()
    th = threading.Thread(target=relay, args=(procs[0].stdout,), daemon=True)
    th.start()
    rc = 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad:
            rc = bad[0]
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            print(f"bench.py: a rank exited with {rc}; the others were stopped", file=sys.stderr, flush=True)
            return rc if rc > 0 else 1
        if all(c == 0 for c in codes):
            th.join(timeout=30)
            return 0
        time.sleep(poll_s)


def gather_dist_info(dist, backend, world, rank, local, dev):
    """What the process group saw: backend, world size and per rank its host,
    LOCAL_RANK, device ordinal and PCI location (all_gather_object), plus the
    RCCL version for the nccl backend."""
    me = {"rank": rank, "local_rank": local, "host": os.uname().nodename}
    if dev is not None and torch.cuda.is_available():
        p = torch.cuda.get_device_properties(dev)
        me.update(device=dev.index, name=p.name, gcn_arch=getattr(p, "gcnArchName", None),
                  pci=f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}")
    else:
        me.update(device="cpu")
    allinfo = [None] * world
    dist.all_gather_object(allinfo, me)
    out = {"backend": backend, "world_size": world, "ranks": allinfo,
           "distinct_devices": len({(i.get("host"), i.get("pci", i.get("device"))) for i in allinfo})}
    if backend == "nccl":
        try:
            out["rccl_version"] = ".".join(str(v) for v in torch.cuda.nccl.version())
        except Exception:  # noqa: BLE001 -- informational only
            out["rccl_version"] = None
    return out


def launch_selftest(args, world, rank, local):
    """--launch-selftest: the N-rank plumbing without a GPU -- join the process
    group (gloo), gather the per-rank info, one all-reduce of a host tensor
    (the MAX-over-ranks the timed region uses), rank 0 prints one JSON line."""
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group(args.dist_backend)
        info = gather_dist_info(dist, args.dist_backend, world, rank, local, None)
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        mx = float(t.item())
    else:
        info, mx = None, 1.0
    if rank == 0:
        print(json.dumps({"metric": "launch selftest (no measurement)", "value": None, "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "dist": info, "max_over_ranks": mx}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--burn-in", type=int, default=100,
                    help="untimed steps before the timed region counted together with --warmup: at least this many "
                         "(a run that starts with every car on its start line is not the steady state)")
    ap.add_argument("--refill", type=int, default=50,
                    help="the pre-timing garbage collection runs this many untimed steps before the timed region "
                         "(part of the untimed count) so the GPU is back at its loaded clock when timing starts; "
                         "0 = collect right before timing (round-2 order)")
    ap.add_argument("--envs-per-gpu", type=int, default=65536)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--cull-chunk", type=int, default=8, help="raycast chunk culling (0 = brute force)")
    ap.add_argument("--sort-interval", type=int, default=None,
                    help="spatial env re-sort period (0 = never; default rx.vector_env.default_sort_interval)")
    ap.add_argument("--ray-order", type=int, default=2,
                    help="raycast lane order (0 env-major, 1 ray-major, 2 direction-sorted tasks)")
    ap.add_argument("--cull-super", type=int, default=8, help="chunks per super-chunk box (0 = one-level culling)")
    ap.add_argument("--stream-groups", type=int, default=1,
                    help="independent env groups, one HIP stream each (1 = one handle on one stream)")
    ap.add_argument("--async-probe-groups", type=int, default=2,
                    help="after the timed region, also time the same workload as this many stream groups "
                         "(reported as 'async_stream_groups'; 0 = skip)")
    ap.add_argument("--profile-steps", type=int, default=128,
                    help="instrumented steps AFTER the timed region: per-kernel durations from per-wave device "
                         "wall-clock stamps (0 = none)")
    ap.add_argument("--counter-steps", type=int, default=16,
                    help="after timing, this many steps with the per-wave culling counters on (executed work)")
    ap.add_argument("--ppo-updates", type=int, default=2,
                    help="also time this many PPO updates (configs[1] per GPU; 0 = skip), reported as 'ppo_train'")
    ap.add_argument("--ppo-envs-per-gpu", type=int, default=4096)
    ap.add_argument("--selfplay-updates", type=int, default=2,
                    help="also time this many two-car self-play PPO updates (configs[3], pool 5; 0 = skip), "
                         "reported as 'selfplay_train'")
    ap.add_argument("--selfplay-envs", type=int, default=8192)
    ap.add_argument("--ppo-steps", type=int, default=128)
    ap.add_argument("--no-time-to-90", action="store_true", help="skip the PPO wall-clock-to-90%% runs")
    ap.add_argument("--dist-backend", default="nccl",
                    help="process-group backend (nccl = RCCL; gloo only to rehearse N ranks on one GPU)")
    ap.add_argument("--sched", default="",
                    help="launch-schedule overrides for A/B runs, 'key=value,...' over rx_config's ABI v17 fields "
                         "(split, wide_n, dyn_lpe, ray_lpr, reward_lpe, argmin_window, seg_filter, box_quadrants; "
                         "0 = auto, -1 = off); scheduling only, results are identical")
    ap.add_argument("--sync", choices=("spin", "block"), default="spin",
                    help="how the host waits at the timed region's edges: spin on the streams' queues, then "
                         "torch.cuda.synchronize() (default), or the blocking synchronize alone")
    ap.add_argument("--graph", choices=("on", "off"), default="on",
                    help="on (default, one stream group): the timed region replays ONE HIP graph holding exactly "
                         "--steps production steps (each one rx_step: k_kin1 + k_step2, the re-sorts where they "
                         "fall), captured untimed before the refill steps -- the launch path of the captured PPO "
                         "rollout; off: one rx_step call per step from Python")
    ap.add_argument("--graph-head", type=int, default=0,
                    help="with --graph on: the first H steps form a graph of their own, replayed just before the "
                         "graph of the other K - H (the GPU starts on the head while the host submits the rest); "
                         "0 = one graph (default: H = 1 / 2 measured no better, profiles/r05/ab_graph_head.jsonl)")
    ap.add_argument("--multi-step", choices=("on", "off"), default="on",
                    help="on (default): the production steps are rx_steps calls over the HBM-resident action bank "
                         "(k_kin1 + k_step2 per step, the re-sort every sort_interval steps); off: one rx_step call "
                         "per step")
    ap.add_argument("--rccl-world1", choices=("on", "off"), default="on",
                    help="at N = 1: also time the data-parallel PPO update over a 1-rank RCCL group "
                         "('ppo_train_rccl_world1': captured epoch graphs and eager)")
    ap.add_argument("--stress", choices=("on", "off"), default="on",
                    help="also time the headline workload on SURVEY.md §8(d)'s stress pool (all-distinct tracks, "
                         "gen_tracks(N, seed=None)), reported as 'stress'")
    ap.add_argument("--stress-envs", type=int, default=None, help="envs of the stress leg (default --envs-per-gpu)")
    ap.add_argument("--launch-selftest", action="store_true",
                    help="launcher / process-group check only: every rank joins the group, reports its device and "
                         "runs one all-reduce; no GPU work, no measurement (tests/test_bench_launch_cpu.py)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # plain `python bench.py --gpus N`: this process (which has not touched HIP)
        # starts the N ranks itself and relays rank 0's JSON line
        raise SystemExit(self_launch(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.launch_selftest:
        return launch_selftest(args, world, rank, local)
    E = args.envs_per_gpu
    G = args.stream_groups
    if G < 1 or E % G:
        raise SystemExit(f"--stream-groups {G} must divide --envs-per-gpu {E}")
    n_total = E * world
    pool, widths = seed1_pool(n_total)
    cpu = None
    if world == 1 and not args.no_cpu_baseline:  # host-only work first: no process here has touched the GPU yet
        cpu = cpu_baseline(pool, widths, budget_s=args.cpu_budget)

    ndev = torch.cuda.device_count()
    if args.dist_backend == "nccl" and local >= ndev:
        raise SystemExit(f"LOCAL_RANK {local} but only {ndev} GPUs visible")
    local_dev = local % max(ndev, 1)  # gloo rehearsal: several ranks may share one GPU
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    dist = None
    dist_info = None
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)
        dist_info = gather_dist_info(dist, args.dist_backend, world, rank, local, dev)

    from rx.vector_env import RacingVectorEnv
    lo = rank * E
    torch.manual_seed(1234 + rank)
    scale = torch.tensor([2.0, 1.0], device=dev)
    shift = torch.tensor([-1.0, 0.0], device=dev)
    untimed = max(args.warmup, args.burn_in)

    sched = {k: int(v) for k, v in (kv.split("=") for kv in args.sched.split(",") if kv)}

    def make_groups(G):
        """G independent env groups, each stepping on its own HIP stream (a group's
        step depends only on its own envs, so different groups' kernels overlap)."""
        n = E // G
        envs = [RacingVectorEnv(pool[lo + g * n:lo + (g + 1) * n], widths[lo + g * n:lo + (g + 1) * n], n_agents=1,
                                n_sensors=11, device=dev, autoreset="next_step", cull_chunk=args.cull_chunk,
                                sort_interval=args.sort_interval, ray_order=args.ray_order,
                                cull_super=args.cull_super, sched=sched)
                for g in range(G)]
        # several groups: every group on a stream of its own (torch's current stream is the
        # null stream, which would serialise against the others)
        streams = [torch.cuda.current_stream(dev)] if G == 1 else [torch.cuda.Stream(device=dev) for _ in range(G)]
        # synthetic inputs resident in HBM before the timed region: a bank of uniform random
        # actions (steer ~ U(-1, 1), throttle ~ U(0, 1)), one [n, 2] slice per step, cycled
        # when the run is longer than the bank (<= 512 MB per GPU)
        bank = max(1, min(args.steps + untimed + args.profile_steps, (512 << 20) // (8 * E)))
        acts = [torch.addcmul(shift, torch.rand((bank, n, 2), device=dev), scale) for _ in range(G)]
        for e in envs:
            e.reset_device()
        torch.cuda.synchronize(dev)
        it = [0]

        def one_step(ev=None):
            k = it[0] % bank
            it[0] += 1
            if G == 1 and ev is None:  # one handle on the current stream: no stream context to enter
                envs[0].step_device(acts[0][k])
                return
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
        def run_steps(K):
            """K production steps of group 0 as rx_steps calls (one per contiguous bank stretch)."""
            while K > 0:
                k = it[0] % bank
                m = min(K, bank - k)
                envs[0].steps_device(acts[0][k:k + m])
                it[0] += m
                K -= m

        active["streams"] = streams
        active["run_steps"] = run_steps
        return envs, one_step, n

    active = {"streams": [torch.cuda.current_stream(dev)]}

    def drain():
        """torch.cuda.synchronize(), after spinning on the active streams until
        their queues are empty (--sync spin, default): a blocking synchronize
        parks the host thread, and the first launch after the wake-up took
        120-270 us of host time in the 20-step region against ~30 us for the
        next ones (tools/first_launch_probe.py, profiles/r03/); spinning first
        keeps the thread awake, the synchronize itself then returns at once."""
        if args.sync == "spin":
            while not all(st.query() for st in active["streams"]):
                pass
        torch.cuda.synchronize()

    def sync_all():
        drain()
        if dist:
            dist.barrier()
        drain()

    def timed(one_step, steps, events=None, collect=True):
        sync_all()
        if collect:
            gc.collect()
        gc.disable()  # a full collection over the 65,536-track pool stalls the host for tens of ms
        mark("t0")
        t0 = time.perf_counter()
        tk = []
        for k in range(steps):
            one_step(events.get(k) if events else None)
            if k < 4 and _MARKS:
                tk.append(time.perf_counter())  # diagnostics only: host time of the first launches
        drain()  # all streams
        gc.enable()
        if dist:
            dist.barrier()
        drain()
        el = time.perf_counter() - t0
        mark("t1")
        if _MARKS and tk:
            print("RX_FIRST_STEPS_US " + " ".join(f"{(b - a) * 1e6:.1f}" for a, b in zip([t0] + tk, tk)),
                  file=sys.stderr, flush=True)
        if dist:
            t = torch.tensor([el], device=dev if args.dist_backend == "nccl" else "cpu", dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    envs, one_step, n = make_groups(G)
    env0 = envs[0]
    n_slots = len(env0.tracks)
    schedule = env0.schedule()
    # untimed steps; the garbage collection that keeps it out of the timed region runs
    # BEFORE the last --refill of them: it stalls the host for tens of ms, the GPU idles
    # and drops its clock meanwhile, and the refill steps bring it back under load
    # (timing starts with a queue-drain sync, as always)
    # The pre-timing sequence (sync, episode-statistics read, sync) runs twice: the
    # first time that sequence runs in a process, the host's first launch after it
    # takes 150-220 us instead of ~40 (tools/first_step_breakdown.py: every part of
    # the call is 5-10x slower, a cold-start effect, gone from the second region on),
    # and the GPU idles meanwhile.  All of it is untimed.
    refill = max(0, min(args.refill, untimed))
    multi = args.multi_step == "on" and G == 1
    run_steps = active["run_steps"]

    def steps(k):  # k production steps in the configured form
        if multi:
            run_steps(k)
        else:
            for _ in range(k):
                one_step()

    steps(untimed - refill)
    # the timed steps as one HIP graph (--graph on): captured here, before the refill
    # steps bring the GPU back to its loaded clock; capturing executes nothing (the
    # library's host-side schedule -- re-sort and task-order launches -- is recorded
    # as it falls for these steps), the timed region replays it exactly once
    step_graph = None
    graph_parts = []
    if args.graph == "on" and G == 1:
        torch.cuda.synchronize(dev)
        # --graph-head H: the first H steps as a graph of their own, the rest as a second
        # graph.  A graph launch submits all of its nodes before the first one runs
        # (t0 -> first kernel ~70 us for the 20-step graph, profiles/r05/window20_*),
        # so the small head graph starts the GPU while the host still submits the rest.
        head = max(0, min(args.graph_head, args.steps - 1))
        graph_parts = [head, args.steps - head] if head > 0 else [args.steps]
        cap = torch.cuda.Stream(device=dev)
        step_graph = []
        for k in graph_parts:
            g = torch.cuda.CUDAGraph()
            # thread_local: a process group's watchdog thread may query its events meanwhile
            with torch.cuda.graph(g, stream=cap, capture_error_mode="thread_local"):
                steps(k)
            step_graph.append(g)
        torch.cuda.synchronize(dev)
        # one untimed replay (K more burn-in steps of the same work): a graph's first
        # launch also uploads it, which would otherwise sit at the timed region's edge
        for g in step_graph:
            g.replay()
        torch.cuda.synchronize(dev)
    ep_untimed = [0.0, 0.0, 0]
    if refill:
        gc.collect()
        gc.disable()
        for half in (refill // 2, refill - refill // 2):
            steps(half)
            sync_all()
            ep_untimed = [a + b for a, b in zip(ep_untimed, (sum(x) for x in zip(*(e.episode_stats() for e in envs))))]
    else:
        sync_all()
        ep_untimed = [sum(x) for x in zip(*(e.episode_stats() for e in envs))]
    # ---- timed region: production steps only (one rx_step per step, no instrumentation)
    if step_graph is not None:
        elapsed = timed(lambda ev=None: [g.replay() for g in step_graph], 1, collect=refill == 0)
    elif multi:
        elapsed = timed(lambda ev=None: run_steps(args.steps), 1, collect=refill == 0)
    else:
        elapsed = timed(one_step, args.steps, collect=refill == 0)
    ep = [sum(x) for x in zip(*(e.episode_stats() for e in envs))]
    # ---- instrumented region (after, same state distribution): per-kernel durations of the
    # production launches (k_kin1, k_step2) on every other step; on the others the dynamics
    # phase and the raycast run as separate launches so the raycast has a duration of its own
    prof = {}
    waves = None
    if args.profile_steps > 0:
        events = {k: ("step" if k % 2 == 0 else "split") for k in range(args.profile_steps)}
        mark("instrumented_begin")
        env0.profile(1)
        env0.profile(0)
        prof_el = timed(one_step, args.profile_steps, events)
        prof = env0.profile_read()
        mark("instrumented_end")
        waves = wave_slots(env0, args.profile_steps * 3) if G == 1 else None
    # ---- executed-work counters (after timing): per ray wave its box tests and leaf scans,
    # per REWARD wave its waypoint-box tests and leaf scans (rx_io.counters, one atomic per wave)
    work = None
    if args.counter_steps > 0 and G == 1:
        mark("counters_begin")
        env0.enable_counters(True)
        for _ in range(args.counter_steps):
            one_step()
        torch.cuda.synchronize()
        cnt = env0.read_counters()
        env0.enable_counters(False)
        mark("counters_end")
        sch = env0.schedule()
        steps_n = args.counter_steps * n
        work = {k: v for k, v in cnt.items()}
        work.update(steps=args.counter_steps, envs=n,
                    ray_box_tests_per_ray_wave=round(cnt["ray_chunk_tests"] / (args.counter_steps * sch["ray_waves"]), 2),
                    ray_leaf_scans_per_ray_wave=round(cnt["ray_chunks_scanned"] / (args.counter_steps * sch["ray_waves"]),
                                                      2),
                    ray_leaf_scans_per_env_step=round(cnt["ray_chunks_scanned"] / steps_n, 3),
                    wp_leaf_scans_per_env_step=round(cnt["wp_chunks_scanned"] / steps_n, 3),
                    note="counted per wave (a wave's box test / leaf scan covers its 64 lanes); scheduling-only "
                         "counters, after the timed region")
    for e in envs:
        e.close()
    stress = None
    if args.stress == "on" and rank == 0:
        stress = stress_leg(dev, args.stress_envs or E, args.steps, untimed, sched)
    async_probe = None
    Ga = args.async_probe_groups
    if Ga > 1 and E % Ga == 0 and Ga != G:
        a_envs, a_step, _ = make_groups(Ga)
        for _ in range(untimed):
            a_step()
        a_el = timed(a_step, args.steps)
        async_probe = {"groups": Ga, "envs_per_group": E // Ga, "value": round(n_total * args.steps / a_el, 1),
                       "ms_per_step": round(a_el / args.steps * 1e3, 4),
                       "note": "same workload as independent env groups on separate HIP streams (async rollout); "
                               "timed after the main region, not the headline value"}
        for e in a_envs:
            e.close()
    gae = gae_roofline(E, dev) if rank == 0 else None
    if gae is not None:
        gae["cache_resident_T128"] = gae_roofline(E, dev, T=128)
    ppo = ppo_leg(world, rank, dev, dist, args.dist_backend, args.ppo_envs_per_gpu, args.ppo_steps,
                  args.ppo_updates) if args.ppo_updates > 0 else None
    # BASELINE configs[1] is named "PPO bf16": the same leg with the bf16 policy kernels
    # (bf16 MFMA operands, f32 accumulation, f32 master weights / Adam), at N = 1 only
    ppo_bf16 = ppo_leg(world, rank, dev, dist, args.dist_backend, args.ppo_envs_per_gpu, args.ppo_steps,
                       args.ppo_updates, "bf16") if args.ppo_updates > 0 and world == 1 else None
    rccl1 = None
    if args.ppo_updates > 0 and world == 1 and args.rccl_world1 == "on":
        try:
            rccl1 = rccl_world1_leg(dev, args.ppo_envs_per_gpu, args.ppo_steps, args.ppo_updates)
        except Exception as e:  # noqa: BLE001 -- reported in the line, the headline is unaffected
            rccl1 = {"error": f"{type(e).__name__}: {e}"[:400]}
    sp = None
    if args.selfplay_updates > 0 and world == 1:
        sp = selfplay_leg(dev, args.selfplay_envs, args.ppo_steps, args.selfplay_updates)
    tt90 = None
    if world == 1 and not args.no_time_to_90:
        # configs[1] is named "PPO bf16": its 4,096-env entry runs in both precisions
        tt90 = time_to_90([(16, 2048, "numpy"), (4096, 128, "device"), (4096, 128, "device", "bf16")])

    if rank == 0:
        value = n_total * args.steps / elapsed
        ms = lambda k: prof[k][0] if k in prof else float("nan")  # noqa: E731
        step2_ms, kin_ms, ray_ms = ms("k_step2"), ms("k_kin1"), ms("k_rays")
        pmc = load_pmc(n)
        step2_gbs = STEP2_BYTES_PER_ENV * n / (step2_ms * 1e-3) / 1e9
        ray_gbs = RAYS_BYTES_PER_ENV * n / (ray_ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "kernel": "k_step2", "achieved": round(step2_gbs, 3),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": step2_gbs / HBM_PEAK_GBS,
                "traffic": pmc.get("k_step2", {}).get("hbm_bytes_per_launch"),
                "traffic_source": pmc.get("source"),
                "bytes_per_env": STEP2_BYTES_PER_ENV, "envs_per_launch": n,
                "avg_launch_ms": round(step2_ms, 5),
                "note": "the step is VALU-bound (branchy f64 ray/segment math): the HBM fraction is "
                        "expected to be tiny; see compute_roofline"}
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
                       "raycast_cull_chunk": args.cull_chunk, "sort_interval": env0.sort_interval,
                       "ray_order": args.ray_order, "cull_super": args.cull_super,
                       "schedule": schedule, "sched_overrides": sched or None,
                       "library": os.path.relpath(_lib_path(), ROOT),
                       "parallelism": f"env shards x{world}, no collective in the step"},
            "steady_state": {"untimed_steps_before_timing": untimed + (args.steps if step_graph is not None else 0),
                             "episodes_ended_before_timing": ep_untimed[2],
                             "episodes_ended_in_timed_region": ep[2],
                             "timed_region": ("production steps only: rx_steps over the HBM-resident action bank "
                                              "(the per-step launches k_kin1 + k_step2, the re-sort every "
                                              "sort_interval steps), no instrumentation"
                                              if multi else
                                              "production steps only: one rx_step (k_kin1 + k_step2) per step, "
                                              "no instrumentation"),
                             "launch": ((f"HIP graph replays of {' + '.join(map(str, graph_parts))} steps (captured "
                                         "and replayed once untimed; the second graph's host submission overlaps "
                                         "the first's execution)" if len(graph_parts) > 1 else
                                         f"one HIP graph replay of the {args.steps} steps (captured and replayed "
                                         "once untimed)")
                                        if step_graph is not None else
                                        ("one rx_steps call" if multi else "one rx_step call per step from Python"))},
            # dominant kernel of the production step: k_step2 (REWARD half beside the raycast)
            "roofline": roof,
            "compute_roofline": compute_roofline(pmc, {"k_step2": step2_ms, "k_kin1": kin_ms, "k_rays": ray_ms}, n,
                                                 waves),
            "executed_work": work,
            "kernels_ms": {k: round(v[0], 5) for k, v in prof.items()},
            "kernel_launches": {k: v[1] for k, v in prof.items()},
            "kernel_timing": f"{args.profile_steps} instrumented steps after the timed region (per-wave device "
                             "wall-clock stamps, rx_profile: first wave start .. last wave end); even steps record "
                             "the production launches, odd steps run k_kin1 + k_step2_reward + k_rays so the "
                             "raycast has its own duration",
            "k_rays_alone": {"avg_launch_ms": round(ray_ms, 5), "bytes_per_env": RAYS_BYTES_PER_ENV,
                             "achieved_GBs": round(ray_gbs, 3),
                             "traffic": pmc.get("k_rays", {}).get("hbm_bytes_per_launch")},
            "step_roofline": {"kernels": "k_kin1 + k_step2", "avg_step_kernels_ms": round(kin_ms + step2_ms, 5),
                              "bytes_per_env_step": STEP_BYTES_PER_ENV,
                              "achieved_GBs": round(STEP_BYTES_PER_ENV * n / ((kin_ms + step2_ms) * 1e-3) / 1e9, 3)},
            "dist": dist_info,
            "gae": gae,
            "stress": stress,
            "async_stream_groups": async_probe,
            "ppo_train": ppo,
            "ppo_train_bf16": ppo_bf16,
            "ppo_train_rccl_world1": rccl1,
            "selfplay_train": sp,
            "time_to_90": tt90,
        }
        if cpu is not None:
            out["cpu_baseline"] = cpu
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
