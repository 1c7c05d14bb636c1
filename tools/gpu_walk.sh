set -o pipefail
export TMPDIR=/tmp
GM_DENSE_SWEEP=walk timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/w1_tests.log 2>&1 || { echo tests failed; exit 1; }
bash tools/ab_sweep.sh gpurun_out/ab4.jsonl "GM_DENSE_SWEEP=list" "GM_DENSE_SWEEP=walk" || exit 1
GM_DENSE_SWEEP=walk bash tools/pmc_quick.sh gpurun_out/pmc_walk || exit 1
echo ok
