set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${1:-t}_tests.log 2>&1 || { echo tests failed; exit 1; }
echo ok
