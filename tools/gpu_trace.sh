#!/bin/bash
# Kernel traces of one dense bench solve and one keyed toot 6x4 solve, and
# their per-launch timelines (tools/trace_levels.py).  Usage: bash tools/gpu_trace.sh TAG
set -o pipefail
tag=${1:-trace}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${tag}_dense -o run \
  -- python3 tools/solve_once.py sum_four_to_one "heaps=31:31:31:31:31:31" dense 2 > gpurun_out/${tag}_dense.log 2>&1 \
  || { echo dense trace failed; tail -20 gpurun_out/${tag}_dense.log; exit 1; }
f=$(find gpurun_out/${tag}_dense -name '*kernel_trace.csv' | head -1)
python3 tools/trace_levels.py $f 3 k_dense_pull_words --all --back 2 > gpurun_out/${tag}_dense_levels.txt
tail -12 gpurun_out/${tag}_dense_levels.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${tag}_toot -o run \
  -- python3 tools/solve_once.py toot_and_otto_bitstring "length=6,height=4" bucketed 2 > gpurun_out/${tag}_toot.log 2>&1 \
  || { echo toot trace failed; tail -20 gpurun_out/${tag}_toot.log; exit 1; }
f=$(find gpurun_out/${tag}_toot -name '*kernel_trace.csv' | head -1)
python3 tools/trace_levels.py $f 3 k_bk_expand --all --back 2 > gpurun_out/${tag}_toot_levels.txt
tail -14 gpurun_out/${tag}_toot_levels.txt
