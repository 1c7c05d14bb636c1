#!/bin/bash
# A/B of the narrow-level run threshold (passes of a 512-thread workgroup):
# in-tree builds gamesmanmpi_amd/libgamesman_hip_runs{1,3,4}.so against the
# default (2), loaded through GM_LIBPATH
set -o pipefail
tag=${1:-r03ab}
mkdir -p gpurun_out
for i in 1 2; do
  for t in 1 0.5 0.75; do
    lib=""
    lib="GM_LIBPATH=$PWD/gamesmanmpi_amd/libgamesman_hip_runs$t.so"
    env $lib timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-keyed > gpurun_out/${tag}_t${t}_$i.json 2>/dev/null || { echo bench $t failed; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['roofline']['ms_kernel_total'], d['roofline']['launches'], round(d['roofline']['frac'],4))" gpurun_out/${tag}_t${t}_$i.json passes=$t
  done
done
