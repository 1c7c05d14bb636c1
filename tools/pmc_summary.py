#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (tools/pmc_passes.sh) per kernel: launch
count and per-launch means of every counter, plus derived HBM-side bytes
(FETCH_SIZE is in KB and, on gfx950, half the bytes of wide coalesced
reads -- MI355X_MICROARCH.md §HBM) and the L2 hit rate.

  python tools/pmc_summary.py gpurun_out/pmc2 [kernel-substring ...]
  python tools/pmc_summary.py --traffic WORKLOAD OUT.json gpurun_out/pmc2
      writes {kernel: {workload, bytes_per_launch, fetch_bytes_per_launch,
      write_bytes_per_launch, l2_hit_rate, source}} for bench.py's
      roofline.traffic (FETCH_SIZE x 2: calibrated on gfx950 with
      tools/calib_fetch.hip for 4-, 8- and 16-B-per-lane reads; WRITE_SIZE
      exact for 4-B stores).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(root):
    per = defaultdict(lambda: defaultdict(float))
    launches = defaultdict(set)
    for path in glob.glob(os.path.join(root, "*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"]
            key = (os.path.basename(os.path.dirname(path)), r["Dispatch_Id"])
            launches[name].add(key)
            per[name][r["Counter_Name"]] += float(r["Counter_Value"])
    return per, launches


KERNEL_SOURCES = ("gamesmanmpi_amd/csrc/gm_plane.h", "gamesmanmpi_amd/csrc/gm_plane_run.h",
                  "gamesmanmpi_amd/csrc/gm_dense.h")


def kernel_sources_sha16(root_dir):
    """Fingerprint of the kernel sources the PMC passes measured: bench.py
    reports the counter traffic only while its own sources still match."""
    import hashlib
    h = hashlib.sha256()
    for rel in KERNEL_SOURCES:
        with open(os.path.join(root_dir, rel), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


KEYED_WORKLOAD = "toot_and_otto_bitstring length=6,height=4"  # the bench keyed record and tools/pmc_ranked.sh


def traffic(workload, out_path, root):
    per, launches = load(root)
    res = {}
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src_sha = kernel_sources_sha16(repo)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from codeobj import kernel_code_sha16
    so = os.path.join(repo, "gamesmanmpi_amd", "libgamesman_hip.so")
    for name, ctr in per.items():
        if "FETCH_SIZE" not in ctr or "WRITE_SIZE" not in ctr:
            continue
        short = name.split("(")[0].replace("void ", "").split("<")[0].split("::")[-1]
        n = len(launches[name]) / max(1, len({p for p, _ in launches[name]}))
        f = ctr["FETCH_SIZE"] * 1024 * 2 / n
        w = ctr["WRITE_SIZE"] * 1024 / n
        # one bench.py run holds several records: the synthetic's kernels, the
        # keyed toot 6x4 record's (RANKED k_rk_*, BUCKETED k_bk_*), the runtime's
        # copies and fills -- label each kernel by the record it served
        wl = (KEYED_WORKLOAD if short.startswith(("k_rk_", "k_bk_", "k_rko_"))
              else workload if short.startswith(("k_plane", "k_dense", "k_fill", "k_checksum"))
              else "bench.py run (every record: runtime copies / fills)")
        row = {"workload": wl, "bytes_per_launch": f + w,
               "fetch_bytes_per_launch": f, "write_bytes_per_launch": w,
               "launches": n, "source": root, "kernel_sources_sha16": src_sha,
               # the key bench.py checks: the measured kernel's own gfx950 code
               "kernel_code_sha16": kernel_code_sha16(so, short)}
        if "TCC_HIT_sum" in ctr:
            row["l2_hit_rate"] = ctr["TCC_HIT_sum"] / max(1.0, ctr["TCC_HIT_sum"] + ctr["TCC_MISS_sum"])
        res[short] = row
    with open(out_path, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


def main():
    if sys.argv[1] == "--traffic":
        return traffic(sys.argv[2], sys.argv[3], sys.argv[4])
    root = sys.argv[1]
    subs = sys.argv[2:] or ["k_dense_resolve", "k_dense_pull", "k_expand", "k_resolve"]
    per, launches = load(root)
    out = {}
    for name, ctr in per.items():
        if not any(s in name for s in subs):
            continue
        short = name.split("(")[0]
        passes = {p for p, _ in launches[name]}
        n = len(launches[name]) / max(1, len(passes))  # launches per pass
        row = {"launches_per_pass": n}
        for c, v in sorted(ctr.items()):
            row[c + "_per_launch"] = v / n
        if "FETCH_SIZE" in ctr:
            row["fetch_bytes_per_launch_x2"] = ctr["FETCH_SIZE"] * 1024 * 2 / n
        if "WRITE_SIZE" in ctr:
            row["write_bytes_per_launch"] = ctr["WRITE_SIZE"] * 1024 / n
        if "TCC_HIT_sum" in ctr:
            row["l2_hit_rate"] = ctr["TCC_HIT_sum"] / max(1.0, ctr["TCC_HIT_sum"] + ctr["TCC_MISS_sum"])
        out[short] = row
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
