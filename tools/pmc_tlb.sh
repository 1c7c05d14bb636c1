#!/bin/bash
# TLB counter pass over one toot 6x4 bucketed solve: bash tools/pmc_tlb.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/pmc_tlb}
export TMPDIR=/tmp
mkdir -p "$out"
timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum --output-format csv \
  -d "$out/tlb" -o run -- python3 tools/solve_once.py toot_and_otto_bitstring "length=6,height=4" bucketed 0 \
  > "$out/tlb.log" 2>&1 || { echo "tlb pass failed"; tail -5 "$out/tlb.log"; exit 1; }
python3 - "$out" <<'PY'
import csv, collections, sys, glob
f = glob.glob(sys.argv[1] + "/tlb/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in sorted(agg.items(), key=lambda kv: -sum(kv[1].values())):
    m, h = c.get("TCP_UTCL1_TRANSLATION_MISS_sum", 0), c.get("TCP_UTCL1_TRANSLATION_HIT_sum", 0)
    print("%-40s miss %.3g hit %.3g miss-rate %.3f" % (k[:40], m, h, m / max(1, m + h)))
PY
