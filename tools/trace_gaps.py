"""Per-step GPU timeline from a rocprofv3 --kernel-trace CSV: kernel durations,
and the idle gaps between consecutive kernels on the device (launch overhead
the step pays on top of its kernels).

    python tools/trace_gaps.py gpurun_out/prof/**/*kernel_trace.csv [--last N]  (window: the last N kernels up to the last k_rays)
"""
import collections
import csv
import glob
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0].split("<")[0].split("::")[-1][:40]


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    last = 400
    if "--last" in sys.argv:
        last = int(sys.argv[sys.argv.index("--last") + 1])
    files = [f for a in args for f in glob.glob(a, recursive=True)]
    rows = []
    for f in files:
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    ks = [i for i, r in enumerate(rows) if r[2] == "k_rays"]  # the step loop: first..last raycast
    if ks:
        rows = rows[max(ks[0], ks[-1] + 1 - last):ks[-1] + 1]
    busy = collections.defaultdict(float)
    cnt = collections.Counter()
    gaps = collections.defaultdict(float)
    for i, (s, e, n) in enumerate(rows):
        busy[n] += (e - s) / 1e3
        cnt[n] += 1
        if i:
            g = s - rows[i - 1][1]
            gaps[(rows[i - 1][2], n)] += max(g, 0) / 1e3
    span = (rows[-1][1] - rows[0][0]) / 1e3
    tot_busy = sum(busy.values())
    print(f"window {len(rows)} kernels, {span:.1f} us; busy {tot_busy:.1f} us ({100 * tot_busy / span:.1f} %)")
    for n in sorted(busy, key=lambda k: -busy[k]):
        print(f"  {n:40s} n={cnt[n]:5d} avg {busy[n] / cnt[n]:8.2f} us  total {busy[n]:9.1f} us")
    print("gaps (prev -> next): total / count")
    pairs = collections.Counter((rows[i - 1][2], rows[i][2]) for i in range(1, len(rows)))
    for k in sorted(gaps, key=lambda k: -gaps[k])[:12]:
        print(f"  {k[0]:28s} -> {k[1]:28s} {gaps[k]:9.1f} us / {pairs[k]} = {gaps[k] / pairs[k]:.2f} us")


if __name__ == "__main__":
    main()
