"""Line a bench timed region up with a rocprofv3 kernel trace.

    python tools/trace_window.py <kernel_trace.csv> <bench stderr with RX_MARK lines> [--out summary.json]

bench.py (RX_BENCH_MARKS=1) prints the host CLOCK_BOOTTIME / CLOCK_MONOTONIC at
the edges of each timed region; rocprofv3 stamps kernels on the same host clock.
For the FIRST timed region (the headline) this reports: host t0 -> first kernel
start, the span of the region's kernels, idle gaps between them, the last
kernel end -> host t1 (end sync + return), per-launch durations of the region's
k_kin1 / k_step2 against the same kernels of the steady-state window right after
it, and whether the spatial re-sort (k_sort_*) lands in the region.
"""
import collections
import csv
import json
import re
import statistics
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0].split("<")[0].split("::")[-1][:40]


def main():
    trace, errf = sys.argv[1], sys.argv[2]
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None
    marks = []
    for line in open(errf):
        m = re.match(r"RX_MARK (\w+) boottime_ns=(\d+) monotonic_ns=(\d+)", line)
        if m:
            marks.append((m.group(1), int(m.group(2)), int(m.group(3))))
    rows = []
    for r in csv.DictReader(open(trace)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    fsm = [m for m in marks if m[0] == "first_step_issued"]
    t0m = [m for m in marks if m[0] == "t0"][0]
    t1m = [m for m in marks if m[0] == "t1"][0]
    # pick the clock the trace uses: the one whose t0 lies within the trace span
    res = {}
    for ci, cname in ((1, "boottime"), (2, "monotonic")):
        t0, t1 = t0m[ci], t1m[ci]
        win = [r for r in rows if t0 <= r[0] <= t1]
        if win:
            res = {"clock": cname, "t0": t0, "t1": t1, "win": win}
            break
    if not res:
        print(json.dumps({"error": "no kernel inside the marked region on either clock",
                          "trace_span": [rows[0][0], rows[-1][1]], "marks": marks}))
        return
    win, t0, t1 = res["win"], res["t0"], res["t1"]
    after = [r for r in rows if r[0] > t1][:len(win) * 5]
    def per(rs):
        d = collections.defaultdict(list)
        for s, e, n in rs:
            d[n].append((e - s) / 1e3)
        return {k: {"n": len(v), "mean_us": round(statistics.mean(v), 3), "first_us": [round(x, 2) for x in v[:4]],
                    "max_us": round(max(v), 2)} for k, v in d.items()}
    busy = sum(e - s for s, e, _ in win)
    gaps = [win[i][0] - win[i - 1][1] for i in range(1, len(win))]
    summary = {
        "clock": res["clock"],
        "host_region_us": round((t1 - t0) / 1e3, 2),
        "t0_to_first_kernel_us": round((win[0][0] - t0) / 1e3, 2),
        "kernel_span_us": round((win[-1][1] - win[0][0]) / 1e3, 2),
        "kernel_busy_us": round(busy / 1e3, 2),
        "idle_gaps_us": round(sum(max(g, 0) for g in gaps) / 1e3, 2),
        "largest_gaps_us": sorted((round(g / 1e3, 2) for g in gaps), reverse=True)[:5],
        "last_kernel_to_t1_us": round((t1 - win[-1][1]) / 1e3, 2),
        "t0_to_first_step_issued_us": (round((fsm[0][1 if res["clock"] == "boottime" else 2] - t0) / 1e3, 2)
                                       if fsm else None),
        "kernels_in_region": per(win),
        "same_kernels_after_region": per(after),
        "sort_in_region": any(n.startswith("k_sort") for _, _, n in win),
    }
    # the whole trace split by the bench's region marks: the timed region
    # (the first t0 .. t1), the instrumented per-wave-stamped steps, the instrumented windows,
    # the executed-work counter steps; "other" = burn-in, graph capture, legs after the env part
    ci = 1 if res["clock"] == "boottime" else 2
    spans = [("timed", t0, t1)]
    for name in ("instrumented", "windows", "counters"):
        b = [m[ci] for m in marks if m[0] == name + "_begin"]
        e = [m[ci] for m in marks if m[0] == name + "_end"]
        if b and e:
            spans.append((name, b[0], e[0]))
    regions = collections.defaultdict(list)
    for r in rows:
        tag = next((n for n, lo, hi in spans if lo <= r[0] <= hi), "other")
        regions[tag].append(r)
    summary["regions"] = {k: per(v) for k, v in regions.items()}
    summary["region_spans_us"] = {n: round((hi - lo) / 1e3, 2) for n, lo, hi in spans}
    s = json.dumps(summary, indent=1)
    print(s)
    if out:
        open(out, "w").write(s)


if __name__ == "__main__":
    main()
