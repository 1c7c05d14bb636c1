"""Per-launch PMC of one dense solve (tools/pmc_dense.sh): the widest
launches of a kernel with fetched / written MB (FETCH_SIZE x 2) and L2 hit.

  python tools/pmc_dense_launches.py OUTDIR kernel-substring [N]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    root, sub = sys.argv[1], sys.argv[2]
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    per = defaultdict(lambda: defaultdict(dict))
    for path in glob.glob(os.path.join(root, "*", "*counter_collection.csv")):
        p = os.path.basename(os.path.dirname(path))
        for r in csv.DictReader(open(path)):
            if sub in r["Kernel_Name"]:
                per[p][int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    f, w, h = (per[k] for k in ("fetch", "write", "hit"))
    fi, wi, hi = sorted(f), sorted(w), sorted(h)
    rows = []
    for k in range(min(len(fi), len(wi), len(hi))):
        F = f[fi[k]]["FETCH_SIZE"] * 2048 / 1e6
        W = w[wi[k]]["WRITE_SIZE"] * 1024 / 1e6
        hh = h[hi[k]]
        rows.append((k, F, W, hh["TCC_HIT_sum"] / max(1.0, hh["TCC_HIT_sum"] + hh["TCC_MISS_sum"])))
    print("%s: %d launches, fetch %.0f MB, write %.0f MB" % (sub, len(rows), sum(r[1] for r in rows),
                                                            sum(r[2] for r in rows)))
    for r in sorted(rows, key=lambda r: -r[1])[:n]:
        print("  launch %3d fetch %6.1f MB write %5.1f MB l2 hit %.2f" % r)


if __name__ == "__main__":
    main()
