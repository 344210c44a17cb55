"""Steady-state PMC counters of the production env kernels (bench.py's state).

Runs bench.py under rocprofv3 --pmc, one pass per counter group (TCC slot
limits: FETCH_SIZE and WRITE_SIZE never share a pass; counters only, no
trace domains), and keeps, per kernel and launch size, only the LAST
dispatches -- those of the timed and instrumented regions after the bench's
burn-in, i.e. the steady state the bench line reports.  Writes one JSON of
per-launch averages:

    python tools/pmc_steady.py OUT.json [--envs 65536] [--last 16]

FETCH_SIZE / WRITE_SIZE are KiB in rocprofv3 (x1024 here).  gfx950's
FETCH_SIZE counts 64 B per 128-B request of a wide coalesced stream
(MI355X_MICROARCH.md §HBM); these kernels read 1-8 B per lane (an
uncalibrated width), so raw counts are reported and fetch_x2 is given as the
upper bound.  SQ_* quad-cycle counters are summed over waves; GRBM_GUI_ACTIVE
is summed over the 8 XCDs.
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PASSES = [
    ["FETCH_SIZE"],
    ["WRITE_SIZE"],
    ["SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
     "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "GRBM_GUI_ACTIVE"],
    ["TCC_HIT_sum", "TCC_MISS_sum", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS", "SQ_WAVES",
     "SQ_BUSY_CYCLES", "SQ_INST_LEVEL_VMEM", "GRBM_GUI_ACTIVE"],
    # executed floating-point work (bench.py compute_roofline): wave-level VALU instructions by kind, 8 SQ
    ["SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64",
     "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_TRANS_F32"],
]
KERNELS = ("k_step2", "k_kin1", "k_kin2", "k_rays", "k_dyn1", "k_dyn2", "k_gae",
           "k_sort_hist", "k_sort_scan",
           "k_sort_scatter", "k_state_copy", "k_state_sync", "k_ppo_grad", "k_policy_act")


def short(name):
    if "k_dyn1<1, 1>" in name or "k_dyn1<1, 1, " in name:  # the split step's k_kin1 (PART = KIN)
        return "k_kin1"
    if "k_dyn2<1>" in name:
        return "k_kin2"
    for k in KERNELS:
        if k in name:
            return k
    return None


def run_pass(out, i, counters, cmd, timeout, required=True):
    d = os.path.join(out, f"pass{i}")
    os.makedirs(d, exist_ok=True)
    full = ["rocprofv3", "--pmc"] + counters + ["-d", d, "-o", "run", "--output-format", "csv", "--"] + cmd
    with open(os.path.join(d, "log.txt"), "w") as log:
        rc = subprocess.run(["timeout", "-s", "KILL", str(timeout)] + full, stdout=log, stderr=subprocess.STDOUT,
                            cwd=ROOT).returncode
    if rc != 0:
        sys.stderr.write(open(os.path.join(d, "log.txt")).read()[-3000:])
        if required:
            raise SystemExit(f"pass {i} ({' '.join(counters)}) failed rc={rc}")
        sys.stderr.write(f"\noptional pass {i} ({' '.join(counters)}) failed rc={rc}: skipped\n")
        return None
    return d


def collect(d):
    """{(kernel, grid): {counter: [per-dispatch values in dispatch order]}}"""
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r.get("Kernel_Name", ""))
            if k is None:
                continue
            rows.append((int(r.get("Dispatch_Id", 0)), k, int(r.get("Grid_Size", 0) or 0), r["Counter_Name"],
                         float(r["Counter_Value"])))
    rows.sort()
    out = defaultdict(lambda: defaultdict(list))
    per_dispatch = defaultdict(lambda: defaultdict(float))
    for did, k, g, c, v in rows:  # a counter may be reported per XCD / instance: sum within a dispatch
        per_dispatch[(did, k, g)][c] += v
    for (did, k, g), cs in sorted(per_dispatch.items()):
        for c, v in cs.items():
            out[(k, g)][c].append(v)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--last", type=int, default=16, help="dispatches per (kernel, grid) kept: the steady state")
    ap.add_argument("--scratch", default=os.path.join(os.environ.get("GRAFT_REPO_ROOT", ROOT), "gpurun_out",
                                                      "pmc_steady"))
    ap.add_argument("--timeout", type=int, default=240)
    ap.add_argument("--cmd", default=None, help="profile this command instead of bench.py (e.g. tools/bench_ppo.py ...)")
    ap.add_argument("--passes", default=None, help="counter passes 'C1,C2;C3,...' instead of the default four")
    ap.add_argument("--bench-args", default="--steps 24 --burn-in 100 --warmup 0 --profile-steps 128 "
                                            "--no-cpu-baseline --async-probe-groups 0 --ppo-updates 0 "
                                            "--no-time-to-90 --selfplay-updates 0 --counter-steps 0 --stress off "
                                            "--rccl-world1 off")
    args = ap.parse_args()
    cmd = [sys.executable, "bench.py", "--envs-per-gpu", str(args.envs)] + args.bench_args.split()
    if args.cmd:
        cmd = [sys.executable] + args.cmd.split()
    passes = [p.split(",") for p in args.passes.split(";")] if args.passes else PASSES
    acc = defaultdict(dict)
    for i, counters in enumerate(passes):
        d = run_pass(args.scratch, i, counters, cmd, args.timeout, required=args.passes is not None or i in (0, 1, 2, 4))
        if d is None:
            continue
        for (k, g), cs in collect(d).items():
            for c, vals in cs.items():
                keep = vals[-args.last:]
                acc[(k, g)][c] = sum(keep) / len(keep)
                acc[(k, g)]["dispatches_seen"] = max(acc[(k, g)].get("dispatches_seen", 0), len(vals))
    res = {"envs_per_launch": args.envs, "command": " ".join(["rocprofv3", "--pmc", "<pass>", "--"] + cmd[1:]),
           "passes": passes, "last_dispatches_kept": args.last,
           "units": "per launch: FETCH_SIZE / WRITE_SIZE in bytes (rocprofv3 KiB x 1024, raw, no x2 read "
                    "correction); SQ_* summed over waves (quad-cycles for *_CYCLES / WAIT / ACTIVE); "
                    "GRBM_GUI_ACTIVE summed over 8 XCDs"}
    # the largest grid of each kernel is its production launch (k_step2: REWARD + raycast workgroups)
    by_kernel = defaultdict(list)
    for (k, g), cs in acc.items():
        by_kernel[k].append((g, cs))
    for k, lst in by_kernel.items():
        lst.sort(key=lambda t: -t[0])
        for j, (g, cs) in enumerate(lst):
            name = k if j == 0 else f"{k}@grid{g}"
            cs = dict(cs, grid=g)
            if "FETCH_SIZE" in cs:
                cs["FETCH_SIZE"] *= 1024
            if "WRITE_SIZE" in cs:
                cs["WRITE_SIZE"] *= 1024
            if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
                cs["hbm_bytes_per_launch"] = cs["FETCH_SIZE"] + cs["WRITE_SIZE"]
                cs["hbm_bytes_per_launch_fetch_x2"] = 2 * cs["FETCH_SIZE"] + cs["WRITE_SIZE"]
            if "TCC_HIT_sum" in cs and "TCC_MISS_sum" in cs and cs["TCC_HIT_sum"] + cs["TCC_MISS_sum"] > 0:
                cs["l2_hit_rate"] = cs["TCC_HIT_sum"] / (cs["TCC_HIT_sum"] + cs["TCC_MISS_sum"])
            res[name] = cs
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: {c: (round(v, 4) if isinstance(v, float) else v) for c, v in d.items()}
                      for k, d in res.items() if isinstance(d, dict)}, indent=1))


if __name__ == "__main__":
    main()
