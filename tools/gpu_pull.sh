set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/q5_tests.log 2>&1 || { echo tests failed; exit 1; }
bash tools/ab_sweep.sh gpurun_out/ab6.jsonl "GM_X=0" "GM_PULL_BAND=1" || exit 1
timeout -k 10 200 python3 tools/group_bench.py 2 3 > gpurun_out/q5_g2.json 2>&1 || exit 1
echo ok
