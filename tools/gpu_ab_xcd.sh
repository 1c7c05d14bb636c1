#!/bin/bash
# A/B: XCD-affine plane order (GM_PLANE_XCD_ORDER=0 turns it off)
set -o pipefail
tag=${1:-r03o}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_planes.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
for i in 1 2 3; do
  for x in 1 0; do
    GM_PLANE_XCD_ORDER=$x timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-keyed > gpurun_out/${tag}_x${x}_$i.json 2>/dev/null || { echo bench failed; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['roofline']['ms_kernel_total'], round(d['roofline']['frac'],4))" gpurun_out/${tag}_x${x}_$i.json xcd=$x
  done
done
