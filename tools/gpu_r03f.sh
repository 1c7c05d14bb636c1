#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist_host.py tests/test_gpu_planes.py tests/test_gpu_keyed.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r03f_tests.log 2>&1 || { echo tests failed; grep -v "^  " gpurun_out/r03f_tests.log | tail -40; exit 1; }
tail -2 gpurun_out/r03f_tests.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --transport host > gpurun_out/r03f_bench_n2_host.json 2> gpurun_out/r03f_bench_n2_host.err || { echo bench n2 failed; tail -20 gpurun_out/r03f_bench_n2_host.err; exit 1; }
cat gpurun_out/r03f_bench_n2_host.json
for w in 2 4 8; do
  timeout -k 10 300 python -u tools/group_planes.py $w 5 > gpurun_out/r03f_group$w.jsonl 2>&1 || { echo group $w failed; tail gpurun_out/r03f_group$w.jsonl; exit 1; }
  tail -1 gpurun_out/r03f_group$w.jsonl
done
