#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/r03i_keyed_group.jsonl
: > $o
for w in 1 2 4 8; do
  timeout -k 10 300 python -u tools/group_keyed_time.py toot_and_otto_bitstring "length=5,height=4" $w 3 >> $o 2>&1 || { echo "toot54 w$w failed"; tail -5 $o; exit 1; }
done
timeout -k 10 400 python -u tools/group_keyed_time.py toot_and_otto_bitstring "length=6,height=4" 2 2 >> $o 2>&1 || { echo "toot64 w2 failed"; tail -5 $o; exit 1; }
cat $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03i_prof -o run -- python3 tools/group_keyed_time.py toot_and_otto_bitstring "length=5,height=4" 4 2 > gpurun_out/r03i_prof.log 2>&1 || { echo prof failed; tail -20 gpurun_out/r03i_prof.log; exit 1; }
python3 tools/kstats.py gpurun_out/r03i_prof/run_kernel_stats.csv | head -24
