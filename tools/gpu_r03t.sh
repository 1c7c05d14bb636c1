#!/bin/bash
# md5 owners: power-of-two fast path + inlined owner in the sharded expand
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r03t}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_keyed.py tests/test_gpu_full_size.py -m gpu -x -q --timeout 300 --timeout-method thread -k "owner or keyed or md5 or shards or bucketed" > gpurun_out/${tag}_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
for w in 2; do
  timeout -k 10 300 python -u tools/group_keyed_time.py toot_and_otto_bitstring "length=6,height=4" $w 2 > gpurun_out/${tag}_toot64_w$w.jsonl 2>&1 || { echo group $w failed; tail gpurun_out/${tag}_toot64_w$w.jsonl; exit 1; }
  tail -1 gpurun_out/${tag}_toot64_w$w.jsonl
done
timeout -k 10 300 python -u tools/group_keyed_time.py othello_bit_new "length=4,height=4" 8 2 > gpurun_out/${tag}_oth8.jsonl 2>&1 || { echo oth8 failed; exit 1; }
tail -1 gpurun_out/${tag}_oth8.jsonl
timeout -k 10 300 python -u tools/group_keyed_time.py othello_bit_new "length=4,height=4" 1 2 > gpurun_out/${tag}_oth1.jsonl 2>&1 || { echo oth1 failed; exit 1; }
tail -1 gpurun_out/${tag}_oth1.jsonl
for w in 1 2 4 8; do
  timeout -k 10 300 python -u tools/group_keyed_time.py toot_and_otto_bitstring "length=5,height=4" $w 2 > gpurun_out/${tag}_toot54_w$w.jsonl 2>&1 || { echo toot54 $w failed; tail gpurun_out/${tag}_toot54_w$w.jsonl; exit 1; }
  tail -1 gpurun_out/${tag}_toot54_w$w.jsonl
done
