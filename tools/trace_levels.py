"""Per-launch timeline of the LAST solve in a rocprofv3 kernel trace: every
launch's kernel, duration, grid and the idle gap before it, plus totals of
busy time and gaps per kernel -- where a latency-bound solve loses its time.

  python tools/trace_levels.py TRACE.csv NSOLVES FIRST_KERNEL_SUBSTRING [--all] [--back K]
(--back K: the K-th solve from the end, default 1 = the last)"""
import csv
import sys


def main():
    path, nsolves, first = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    show_all = "--all" in sys.argv
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
    per = len(starts) // nsolves
    k = int(sys.argv[sys.argv.index("--back") + 1]) if "--back" in sys.argv else 1
    i0 = starts[-k * per]  # first launch of the chosen solve
    rs = rows[i0:starts[-(k - 1) * per]] if k > 1 else rows[i0:]
    t0 = int(rs[0]["Start_Timestamp"])
    prev_end = t0
    tot = {}
    for j, r in enumerate(rs):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0]
        gap = max(0, s - prev_end) / 1e3
        dur = (e - s) / 1e3
        t = tot.setdefault(name, [0, 0.0, 0.0])
        t[0] += 1
        t[1] += dur
        t[2] += gap
        if show_all:
            grid = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
            print("%4d %-40s dur %8.1f us gap %6.1f us grid %6d" % (j, name[:40], dur, gap, grid))
        prev_end = max(prev_end, e)
    span = (prev_end - t0) / 1e3
    print("span of the last solve: %.1f us" % span)
    for name, (n, d, g) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print("  %-44s %5d launches  busy %9.1f us  gaps before %8.1f us" % (name[:44], n, d, g))


if __name__ == "__main__":
    main()
