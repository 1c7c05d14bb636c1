#!/bin/bash
set -o pipefail
tag=${1:-bk}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_edge_shapes.py tests/test_gpu_parity.py tests/test_gpu_full_size.py -k "keyed or bucketed or toot" -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/${tag}_tests.log; exit 1; }
echo tests ok; tail -2 gpurun_out/${tag}_tests.log
bash tools/prof_bk.sh ${tag}_prof > /dev/null || exit 1
grep wall gpurun_out/${tag}_prof.log | tail -1
