#!/bin/bash
# dense-path GPU checks: variant / checkpoint / full-size parity tests, then a
# kernel trace of the bench workload (tools/trace_dense.sh)
set -o pipefail
tag=${1:-dense}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_variants.py tests/test_gpu_checkpoint.py tests/test_gpu_full_size.py \
  tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 \
  || { echo tests failed; tail -40 gpurun_out/${tag}_tests.log; exit 1; }
echo tests ok; tail -2 gpurun_out/${tag}_tests.log
bash tools/trace_dense.sh ${tag}_trace
