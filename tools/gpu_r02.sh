#!/bin/bash
# One GPU session: the -m gpu suite, then the bench line, then a rocprofv3
# kernel-trace summary of a short bench (each step under its own timeout;
# the script stops at the first failure).  Usage: bash tools/gpu_r02.sh TAG
set -o pipefail
tag=${1:-r02}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/${tag}_gpu_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/${tag}_gpu_tests.log; exit 1; }
echo tests ok
tail -3 gpurun_out/${tag}_gpu_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err \
  || { echo bench failed; tail -20 gpurun_out/${tag}_bench.err; exit 1; }
echo bench ok
cat gpurun_out/${tag}_bench.json
