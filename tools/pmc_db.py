#!/usr/bin/env python3
"""Per-kernel sums of rocprofv3 PMC counters from its sqlite output
(rocpd *.db, the default format of ROCm 7.2's rocprofv3): launches and the
per-launch mean of every counter, by kernel name.

  python tools/pmc_db.py DIR [DIR ...] [--match SUBSTR]
"""
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def load(d):
    per = defaultdict(lambda: defaultdict(float))
    launches = defaultdict(set)
    for db in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        c = sqlite3.connect(db)
        cols = [r[1] for r in c.execute("pragma table_info(counters_collection)")]
        kcol = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else None)
        q = "select %s, dispatch_id, counter_name, value from counters_collection" % kcol
        for name, disp, cn, v in c.execute(q):
            per[name][cn] += float(v)
            launches[name].add((db, disp))
    return per, launches


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    match = None
    if "--match" in sys.argv:
        match = sys.argv[sys.argv.index("--match") + 1]
        args.remove(match)
    for d in args:
        per, launches = load(d)
        for name in sorted(per):
            if match and match not in name:
                continue
            n = len(launches[name])
            vals = ", ".join("%s %.4g" % (k, v / n) for k, v in sorted(per[name].items()))
            print("%s | %s | launches %d | per launch: %s" % (d, name[:60], n, vals))


if __name__ == "__main__":
    main()
