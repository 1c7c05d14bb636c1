#!/bin/bash
# staged PLANES shards: group / host-transport / full-size shard tests, then
# per-shard device time of the bench shapes, staged vs level-synchronous
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r03l}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_planes.py tests/test_gpu_dist_host.py tests/test_gpu_full_size.py -m gpu -x -v --timeout 300 --timeout-method thread -k "planes or host or shards" > gpurun_out/${tag}_tests.log 2>&1 || { echo tests failed; grep -v "^  " gpurun_out/${tag}_tests.log | tail -30; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
for w in 2 4 8; do
  timeout -k 10 200 python -u tools/group_planes.py $w 3 > gpurun_out/${tag}_group${w}.jsonl 2>&1 || { echo group $w failed; tail gpurun_out/${tag}_group${w}.jsonl; exit 1; }
  tail -1 gpurun_out/${tag}_group${w}.jsonl
  timeout -k 10 200 python -u tools/group_planes.py $w 3 4096 > gpurun_out/${tag}_group${w}_ls.jsonl 2>&1 || { echo group $w ls failed; tail gpurun_out/${tag}_group${w}_ls.jsonl; exit 1; }
  tail -1 gpurun_out/${tag}_group${w}_ls.jsonl
done
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --transport host > gpurun_out/${tag}_bench_n2_host.json 2> gpurun_out/${tag}_bench_n2_host.err || { echo bench n2 host failed; tail -20 gpurun_out/${tag}_bench_n2_host.err; exit 1; }
cat gpurun_out/${tag}_bench_n2_host.json
