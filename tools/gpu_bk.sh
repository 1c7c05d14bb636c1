#!/bin/bash
# Bucketed-levels bring-up: keyed edge shapes + golden tables + full-size
# toot checksums, then toot 6x4 timings (bucketed vs hash table).
set -o pipefail
tag=${1:-bk}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_edge_shapes.py tests/test_gpu_parity.py -k "keyed or bucketed" -x -v \
  --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/${tag}_tests.log; exit 1; }
echo tests ok; tail -2 gpurun_out/${tag}_tests.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_size.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_full.log 2>&1 || { echo full-size failed; tail -40 gpurun_out/${tag}_full.log; exit 1; }
echo full ok; tail -2 gpurun_out/${tag}_full.log
timeout -k 10 300 python -u tools/solve_once.py toot_and_otto_bitstring "length=6,height=4" bucketed 2 > gpurun_out/${tag}_toot64_bk.jsonl 2>&1 || { echo bk timing failed; tail gpurun_out/${tag}_toot64_bk.jsonl; exit 1; }
cat gpurun_out/${tag}_toot64_bk.jsonl
