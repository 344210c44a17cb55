"""Kernel statistics of a rocprofv3 *_kernel_trace.csv split by launch size.

    python tools/kstats_by_grid.py TRACE.csv [OUT.csv] [--top 30]

rocprofv3's --stats summary averages every launch of a kernel name, whatever
its grid: a bench run launches k_step2 at 65,536 envs (the timed and
instrumented regions) and at 32,768 envs (the two-group async probe), and the
PPO legs at 4,096 / 8,192 envs, so one average mixes them.
This groups the trace by (kernel name, grid size, workgroup size) and writes
calls / total / average / min / max per group, largest total first.
"""
import csv
import sys
from collections import defaultdict


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    top = 30
    if "--top" in sys.argv:
        top = int(sys.argv[sys.argv.index("--top") + 1])
        args = [a for a in args if a != str(top)]
    rows = list(csv.DictReader(open(args[0])))
    g = defaultdict(list)
    for r in rows:
        name = r.get("Kernel_Name", "")
        grid = r.get("Grid_Size", r.get("Grid_Size_X", ""))
        wg = r.get("Workgroup_Size", r.get("Workgroup_Size_X", ""))
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        g[(name, grid, wg)].append(dur)
    out = []
    for (name, grid, wg), d in g.items():
        out.append({"Name": name, "Grid_Size": grid, "Workgroup_Size": wg, "Calls": len(d), "TotalDurationNs": sum(d),
                    "AverageNs": round(sum(d) / len(d), 1), "MinNs": min(d), "MaxNs": max(d)})
    out.sort(key=lambda r: -r["TotalDurationNs"])
    if len(args) > 1:
        with open(args[1], "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(out[0].keys()))
            w.writeheader()
            w.writerows(out)
    for r in out[:top]:
        print(f"{r['TotalDurationNs'] / 1e6:9.3f} ms {r['Calls']:6d} {r['AverageNs'] / 1e3:9.2f} us grid {r['Grid_Size']:>9} "
              f"wg {r['Workgroup_Size']:>4}  {r['Name'][:90]}")


if __name__ == "__main__":
    main()
