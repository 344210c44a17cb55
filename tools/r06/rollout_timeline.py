"""Per-step kernel timeline of the configs[1] rollout (rx_rollout_steps at 4,096 envs,
bf16 policy) from a rocprofv3 --kernel-trace CSV: for the last rollout in the trace,
per step the launches (k_policy_act, k_kin1 = k_dyn1<1, KIN>, k_step2), their mean
durations and the mean idle gaps between consecutive kernels.

    python tools/r06/rollout_timeline.py 'gpurun_out/<dir>/**/*kernel_trace.csv' [out.json]
"""
import collections
import csv
import glob
import json
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    base = n.split("(")[0]
    name = base.split("<")[0].split("::")[-1]
    return name + ("<" + base.split("<", 1)[1] if "<" in base else "")


def main():
    files = glob.glob(sys.argv[1], recursive=True)
    rows = []
    for f in files:
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    # the last run of consecutive step triples: k_policy_act*, k_dyn1*KIN*, k_step2*
    is_pol = lambda n: n.startswith("k_policy_act")  # noqa: E731
    starts = [i for i, r in enumerate(rows) if is_pol(r[2]) and i + 2 < len(rows)
              and rows[i + 1][2].startswith("k_dyn1") and rows[i + 2][2].startswith("k_step2")]
    # group consecutive steps (policy launches 3 apart) and keep the last group = the last rollout
    groups, cur = [], [starts[0]]
    for a, b in zip(starts, starts[1:]):
        if b - a == 3:
            cur.append(b)
        else:
            groups.append(cur)
            cur = [b]
    groups.append(cur)
    steps = groups[-1]
    kd = collections.defaultdict(list)
    gaps = collections.defaultdict(list)
    per_step = []
    for s in steps[2:]:  # skip the first steps (cold)
        tri = rows[s:s + 3]
        nxt = rows[s + 3] if s + 3 < len(rows) else None
        for r in tri:
            kd[r[2]].append((r[1] - r[0]) / 1e3)
        gaps["policy->kin"].append((tri[1][0] - tri[0][1]) / 1e3)
        gaps["kin->step2"].append((tri[2][0] - tri[1][1]) / 1e3)
        if nxt is not None and is_pol(nxt[2]):
            gaps["step2->policy"].append((nxt[0] - tri[2][1]) / 1e3)
            per_step.append((nxt[0] - tri[0][0]) / 1e3)
    mean = lambda v: round(sum(v) / len(v), 3) if v else None  # noqa: E731
    out = {"steps_in_rollout": len(steps), "steps_averaged": len(steps) - 2,
           "kernel_us": {k: mean(v) for k, v in kd.items()}, "gap_us": {k: mean(v) for k, v in gaps.items()},
           "step_us": mean(per_step)}
    print(json.dumps(out))
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
