#!/bin/bash
# round 3: the changed GPU tests, PLANES shard-group device times, a kernel
# trace of the 2-shard group
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist_host.py tests/test_gpu_keyed.py tests/test_gpu_full_size.py tests/test_gpu_planes.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r03d_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r03d_tests.log; exit 1; }
tail -2 gpurun_out/r03d_tests.log
for w in 2 4 8; do
  timeout -k 10 300 python -u tools/group_planes.py $w 5 > gpurun_out/r03d_group$w.jsonl 2>&1 || { echo group $w failed; tail gpurun_out/r03d_group$w.jsonl; exit 1; }
  tail -2 gpurun_out/r03d_group$w.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03d_prof2 -o run -- python3 tools/group_planes.py 2 3 > gpurun_out/r03d_prof2.log 2>&1 || { echo prof failed; tail -20 gpurun_out/r03d_prof2.log; exit 1; }
python3 tools/kstats.py gpurun_out/r03d_prof2/run_kernel_stats.csv | head -12
