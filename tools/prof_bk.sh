#!/bin/bash
# rocprofv3 kernel stats of one toot 6x4 bucketed solve (after a warm-up)
set -o pipefail
tag=${1:-bkprof}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag} -o run \
  -- python3 tools/solve_once.py toot_and_otto_bitstring "length=6,height=4" ${2:-bucketed} 1 > gpurun_out/${tag}.log 2>&1 || { echo prof failed; tail -20 gpurun_out/${tag}.log; exit 1; }
echo prof ok
f=$(find gpurun_out/${tag} -name '*kernel_stats.csv' | head -1)
cat "$f" | cut -d, -f1-8 | head -30
