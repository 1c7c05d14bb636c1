"""Per-launch duration digest of a rocprofv3 kernel trace: for each kernel
name substring, the launches of the LAST solve (the trace holds N solves of
equal launch counts), their sum, span, gaps and the widest launches.

  python tools/trace_stats.py TRACE.csv NSOLVES name-substring ..."""
import csv
import sys


def main():
    path, nsolves = sys.argv[1], int(sys.argv[2])
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    for sub in sys.argv[3:]:
        rs = [r for r in rows if sub in r["Kernel_Name"]]
        per = len(rs) // nsolves
        rs = rs[-per:]
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rs]
        g = [int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]) for r in rs]
        span = (int(rs[-1]["End_Timestamp"]) - int(rs[0]["Start_Timestamp"])) / 1e3
        print("%s: %d launches, sum %.1f us, span %.1f us" % (sub, len(d), sum(d), span))
        b = {}
        for x in d:
            k = "<8" if x < 8 else "<16" if x < 16 else "<32" if x < 32 else "<64" if x < 64 else ">=64"
            b.setdefault(k, [0, 0.0])
            b[k][0] += 1
            b[k][1] += x
        print("   by duration (us): %s" % {k: (v[0], round(v[1], 1)) for k, v in sorted(b.items())})
        top = sorted(zip(d, g, range(len(d))), reverse=True)[:5]
        print("   widest: %s" % [(round(a, 1), gg, i) for a, gg, i in top])


if __name__ == "__main__":
    main()
