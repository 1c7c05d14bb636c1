#!/bin/bash
# A/B: split fine partition (K workgroups per coarse partition) vs k_bk_fine
set -o pipefail
tag=${1:-r03q}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_keyed.py tests/test_gpu_full_size.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "toot or othello or keyed or bucketed or ttt or mttt" > gpurun_out/${tag}_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
for i in 1 2; do
  for fs in 1 0; do
    GM_BK_FINE_SPLIT=$fs timeout -k 10 200 python tools/solve_once.py toot_and_otto_bitstring "length=6,height=4" bucketed 3 > gpurun_out/${tag}_f${fs}_$i.jsonl 2>&1 || { echo solve failed; tail gpurun_out/${tag}_f${fs}_$i.jsonl; exit 1; }
    python3 -c "import json,sys; L=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')]; print(sys.argv[2], [round(x['ms_total'],1) for x in L], [round(x['ms_forward'],1) for x in L])" gpurun_out/${tag}_f${fs}_$i.jsonl fsplit=$fs
  done
done
GM_BK_FINE_SPLIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run -- python3 tools/solve_once.py toot_and_otto_bitstring "length=6,height=4" bucketed 1 > gpurun_out/${tag}_prof.log 2>&1 || { echo prof failed; exit 1; }
python3 tools/kstats.py gpurun_out/${tag}_prof/run_kernel_stats.csv | head -14
