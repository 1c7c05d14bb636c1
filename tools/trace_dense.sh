#!/bin/bash
# rocprofv3 kernel trace of the bench workload (dense 2^30): per-launch durations
set -o pipefail
tag=${1:-dtrace}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${tag} -o run \
  -- python3 tools/solve_once.py sum_four_to_one "heaps=31:31:31:31:31:31" dense 2 > gpurun_out/${tag}.log 2>&1 || { echo trace failed; tail -20 gpurun_out/${tag}.log; exit 1; }
grep wall_ms gpurun_out/${tag}.log
