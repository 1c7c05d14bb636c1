#!/bin/bash
# full -m gpu suite on the final tree
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/r06g
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gpu_tests.txt 2>&1 || { tail -40 $out/gpu_tests.txt; exit 1; }
tail -3 $out/gpu_tests.txt
