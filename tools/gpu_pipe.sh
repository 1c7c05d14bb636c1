set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/p1_tests.log 2>&1 || { echo tests failed; exit 1; }
bash tools/ab_sweep.sh gpurun_out/ab5.jsonl "GM_DENSE_PIPE=1" "GM_DENSE_PIPE=0" || exit 1
bash tools/pmc_quick.sh gpurun_out/pmc_pipe || exit 1
echo ok
