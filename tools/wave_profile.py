"""How k_step2's waves fill the chip over one production launch (diagnostic).

    python tools/wave_profile.py [n_envs] [steps] [sched k=v,...]      (GPU box)

The bench workload (seed-1 pool, uniform random actions, next-step autoreset)
after a 150-step burn-in; `steps` production steps are recorded with
rx_profile and their per-wave wall-clock stamps read back (rx_profile_waves,
100 MHz).  Per recorded k_step2 launch: span, REWARD vs ray wave durations,
the active-wave count over time (1 us bins against the 8,192 wave slots of
1,024 SIMDs at 8 waves each), the time of the last wave start, the tail after
the active count falls below half the slots, and the mean ray-wave duration
by dispatch-order decile.  One JSON object on stdout.
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))
sys.path.insert(0, ROOT)


def summarize(st, en, n_rw, cls=None, sub=None, slots=8192):
    """One recorded k_step2 launch.  st / en: per-wave start / end (us from the
    first start, NaN = no wave) in workgroup order, REWARD waves [0, n_rw) first;
    cls / sub: per RAY wave (dispatch order) its class and tail sub-wave from the
    library's own table (RacingVectorEnv.ray_wave_table: exact for every
    dispatch mode and tail split).  wave_slot_utilisation = the launch's summed
    wave time over slots x span (8 waves on each of 1,024 SIMDs)."""
    live = ~np.isnan(st)
    span = float(np.nanmax(en[live]))
    dur = en - st
    rw = np.arange(len(st)) < n_rw
    ray = live & ~rw
    bins = np.arange(0.0, span + 1.0, 1.0)
    act = np.array([int(np.sum(live & (st <= t) & (en > t))) for t in bins])
    below = np.nonzero(act >= slots // 2)[0]
    half_t = float(bins[below[-1]]) if len(below) else 0.0
    ray_idx = np.nonzero(ray)[0]
    dec = np.array_split(ray_idx, 10)
    res = {
        "span_us": round(span, 2),
        "reward_waves": int(np.sum(live & rw)), "ray_waves": int(np.sum(ray)),
        "reward_dur_us_p50_p90_max": [round(float(np.percentile(dur[live & rw], q)), 2) for q in (50, 90, 100)]
        if np.any(live & rw) else None,
        "ray_dur_us_p10_p50_p90_max": [round(float(np.percentile(dur[ray], q)), 2) for q in (10, 50, 90, 100)],
        "last_wave_start_us": round(float(np.nanmax(st[live])), 2),
        "first_wave_end_us": round(float(np.nanmin(en[live])), 2),
        "active_waves_by_us": act.tolist(),
        "tail_after_half_slots_us": round(span - half_t, 2),
        "wave_slot_utilisation": round(float(np.nansum(dur[live])) / (slots * span), 3),
        "ray_dur_us_by_dispatch_decile": [round(float(np.mean(dur[d])), 2) for d in dec if len(d)],
        "ray_start_us_by_dispatch_decile": [round(float(np.mean(st[d])), 2) for d in dec if len(d)],
    }
    if cls is not None:
        c = np.full(len(st), -1, np.int64)
        m = min(len(cls), len(st) - n_rw)
        c[n_rw:n_rw + m] = cls[:m]
        classes = sorted(int(j) for j in np.unique(c[ray]) if j >= 0)
        res["ray_dur_us_by_class"] = {j: round(float(np.nanmean(dur[ray & (c == j)])), 2) for j in classes}
        res["ray_start_us_by_class"] = {j: round(float(np.nanmean(st[ray & (c == j)])), 2) for j in classes}
        res["ray_end_us_by_class_max"] = {j: round(float(np.nanmax(en[ray & (c == j)])), 2) for j in classes}
    return res


def record(env, act, steps):
    """Record `steps` production steps of `env` and summarise every k_step2 launch."""
    sched = env.schedule()
    n_rw = sched["reward_lpe"] * ((sched["dyn_waves"] + 7) // 8 * 8)  # k_step2: REWARD workgroups first
    tab = env.ray_wave_table()
    torch.cuda.synchronize()
    env.profile(1)
    for _ in range(steps):
        env.step_device(act())
    env.profile(0)
    torch.cuda.synchronize()
    out = []
    k = 0
    while True:
        try:
            st, en, kind, n = env.profile_waves(k)
        except Exception:  # noqa: BLE001 -- past the record
            break
        if kind == "k_step2":
            s = summarize(st, en, n_rw, tab["cls"], tab["sub"])
            s["launch"] = k
            out.append((s, st, en))
        k += 1
    return sched, out


def main():
    from bench import seed1_pool
    from rx.vector_env import RacingVectorEnv
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    sched = {k: int(v) for k, v in (kv.split("=") for kv in (sys.argv[3] if len(sys.argv) > 3 else "").split(",") if kv)}
    pool, widths = seed1_pool(N)
    env = RacingVectorEnv(pool, widths, device="cuda", autoreset="next_step", sched=sched)
    env.reset_device()
    g = torch.Generator(device="cuda").manual_seed(0)
    scale = torch.tensor([2.0, 1.0], device="cuda")
    shift = torch.tensor([-1.0, 0.0], device="cuda")

    def act():
        return torch.addcmul(shift, torch.rand((N, 2), generator=g, device="cuda"), scale)
    for _ in range(150):
        env.step_device(act())
    sched, launches = record(env, act, steps)
    out = {"n_envs": N, "schedule": sched, "launches": []}
    for i, (s, st, en) in enumerate(launches):
        if i == 0:
            s["raw_start_us"] = np.round(st, 2).tolist()
            s["raw_end_us"] = np.round(en, 2).tolist()
        out["launches"].append(s)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
