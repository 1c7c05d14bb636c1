set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s5_tests.log 2>&1 || { echo tests failed; exit 1; }
bash tools/ab_sweep.sh gpurun_out/ab3.jsonl "GM_DENSE_SWEEP=list" "GM_DENSE_SWEEP=cols" || exit 1
timeout -k 10 200 python tools/group_bench.py 2 3 > gpurun_out/s5_group2.json 2>&1 || exit 1
timeout -k 10 200 python tools/group_bench.py 4 2 > gpurun_out/s5_group4.json 2>&1 || exit 1
echo ok
