#!/bin/bash
# md5-sharded bucketed levels: local-dedup form (GM_F_BKS_LOCAL) tests and timings
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r03x}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_keyed.py tests/test_gpu_full_size.py -m gpu -x -v --timeout 200 --timeout-method thread -k "local_dedup or toot_5x4 or group_keyed or toot_6x4_two or two_processes" > gpurun_out/${tag}_tests.log 2>&1 || { echo tests failed; grep -v "^  " gpurun_out/${tag}_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
for fl in 0 16384; do  # 0: hybrid (local for levels of >= 1 M parents), 16384: every level local
  timeout -k 10 300 python -u tools/group_keyed_time.py toot_and_otto_bitstring "length=6,height=4" 2 2 $fl > gpurun_out/${tag}_toot64_w2_f$fl.jsonl 2>&1 || { echo toot64 $fl failed; tail gpurun_out/${tag}_toot64_w2_f$fl.jsonl; exit 1; }
  tail -1 gpurun_out/${tag}_toot64_w2_f$fl.jsonl
  for w in 2 4 8; do
    timeout -k 10 300 python -u tools/group_keyed_time.py toot_and_otto_bitstring "length=5,height=4" $w 2 $fl > gpurun_out/${tag}_toot54_w${w}_f$fl.jsonl 2>&1 || { echo toot54 $w $fl failed; tail gpurun_out/${tag}_toot54_w${w}_f$fl.jsonl; exit 1; }
    tail -1 gpurun_out/${tag}_toot54_w${w}_f$fl.jsonl
  done
done
