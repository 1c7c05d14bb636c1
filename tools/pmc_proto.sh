#!/bin/bash
# PMC passes over plane_proto runs: bash tools/pmc_proto.sh TAG "ARGS" [counters...]
set -o pipefail
export TMPDIR=/tmp
tag=$1; args=$2; shift 2
out=gpurun_out/pmcp_$tag
mkdir -p $out
i=0
for ctr in "$@"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $ctr --output-format csv -d $out/p$i -o run -- ./tools/plane_proto $args > $out/p$i.log 2>&1 || { echo "pass $ctr failed"; tail -5 $out/p$i.log; exit 1; }
done
python3 - $out <<'PY'
import csv, collections, sys, glob
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.defaultdict(set)
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[k].add((f, r["Dispatch_Id"]))
for k, c in agg.items():
    print(k[:60], {a: "%.4g" % b for a, b in c.items()}, "dispatches(all passes)", len(n[k]))
PY
