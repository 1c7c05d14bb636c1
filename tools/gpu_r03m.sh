#!/bin/bash
# narrow-level runs + staged shards: planes / host / full-size shard tests,
# bench line, rocprof of the bench, group timings staged vs level-sync
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r03m}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_planes.py tests/test_gpu_dist_host.py tests/test_gpu_full_size.py -m gpu -x -v --timeout 300 --timeout-method thread -k "planes or host or shards or sum_31" > gpurun_out/${tag}_tests.log 2>&1 || { echo tests failed; grep -v "^  " gpurun_out/${tag}_tests.log | tail -30; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { echo bench failed; tail -20 gpurun_out/${tag}_bench.err; exit 1; }
cat gpurun_out/${tag}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-keyed > gpurun_out/${tag}_prof.log 2>&1 || { echo prof failed; tail -20 gpurun_out/${tag}_prof.log; exit 1; }
python3 tools/kstats.py gpurun_out/${tag}_prof/run_kernel_stats.csv | head -8
for w in 2 4 8; do
  timeout -k 10 200 python -u tools/group_planes.py $w 3 > gpurun_out/${tag}_group${w}.jsonl 2>&1 || { echo group $w failed; tail gpurun_out/${tag}_group${w}.jsonl; exit 1; }
  tail -1 gpurun_out/${tag}_group${w}.jsonl
done
