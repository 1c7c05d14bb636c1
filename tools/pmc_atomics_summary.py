"""Per-kernel atomic counts and rates of tools/pmc_atomics.sh output (one
toot 6x4 BUCKETED solve): L2 atomic requests (TCC_ATOMIC_sum) and LDS atomic
wave-instructions (SQ_INSTS_LDS_ATOMIC) per solve, and their rates over the
kernel's own time in the trace pass.  Reference rates (MI355X_MICROARCH.md):
memory-side atomics ~1.3 TB/s of 256-B wave-instructions (~5e9 wave-instr/s
chip-wide) -- one L2 atomic request is one 64-B piece; LDS: one LDS
instruction issue per CU per cycle-ish (256 CUs x 2.4 GHz = 6.1e11/s upper
bound).

  python3 tools/pmc_atomics_summary.py OUTDIR > profiles/keyed_atomics.json
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(__file__))
from pmc_summary import load  # noqa: E402

BK_SOURCES = ("gamesmanmpi_amd/csrc/gm_bucketed.h", "gamesmanmpi_amd/csrc/gm_games.h")


def sources_sha16(root_dir):
    import hashlib
    h = hashlib.sha256()
    for rel in BK_SOURCES:
        with open(os.path.join(root_dir, rel), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def short(name):
    return name.split("(")[0].replace("void ", "").split("<")[0].split("::")[-1]


def main():
    root = sys.argv[1]
    per = {}
    p, _ = load(root)  # root/l2/, root/lds/: one counter pass each
    for name, ctr in p.items():
        d = per.setdefault(short(name), {})
        for c, v in ctr.items():
            d[c] = d.get(c, 0.0) + v
    ns = {}
    for path in glob.glob(os.path.join(root, "trace", "**", "run_kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            k = short(r["Kernel_Name"])
            ns[k] = ns.get(k, 0) + int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    out = {"workload": "toot_and_otto_bitstring length=6,height=4", "layout": "bucketed",
           "source": root, "sources_sha16": sources_sha16(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
           "units": "per solve; rates over the kernel's own time (trace pass)", "kernels": {}}
    tot = {"l2_atomic_requests": 0.0, "lds_atomic_insts": 0.0, "kernel_ms": 0.0}
    for k in sorted(per):
        if not k.startswith("k_bk"):
            continue
        c = per[k]
        ms = ns.get(k, 0) / 1e6
        l2 = c.get("TCC_ATOMIC_sum", 0.0)
        lds = c.get("SQ_INSTS_LDS_ATOMIC", 0.0)
        row = {"kernel_ms": ms, "l2_atomic_requests": l2, "l2_atomic_to_memory": c.get("TCC_EA0_ATOMIC_sum", 0.0),
               "lds_atomic_insts": lds, "lds_atomic_64B_units": c.get("SQ_INSTS_LDS_ATOMIC_BANDWIDTH", 0.0),
               "lds_insts": c.get("SQ_INSTS_LDS", 0.0)}
        if ms > 0:
            row["l2_atomic_per_s"] = l2 / (ms / 1e3)
            row["lds_atomic_insts_per_s"] = lds / (ms / 1e3)
        out["kernels"][k] = row
        tot["l2_atomic_requests"] += l2
        tot["lds_atomic_insts"] += lds
        tot["kernel_ms"] += ms
    if tot["kernel_ms"] > 0:
        tot["l2_atomic_per_s"] = tot["l2_atomic_requests"] / (tot["kernel_ms"] / 1e3)
        tot["lds_atomic_insts_per_s"] = tot["lds_atomic_insts"] / (tot["kernel_ms"] / 1e3)
    out["total"] = tot
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
