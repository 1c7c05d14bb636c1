#!/bin/bash
# pairs + queued solves: plane tests, the 2^30 fingerprint, the async probe
# (product build), the pair-range sweep in the lab, then the bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/r06c
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_planes.py "tests/test_gpu_full_size.py::test_gpu_sum_31x6_checksum" -x -q -m gpu --timeout 300 --timeout-method thread > $out/gpu_tests.txt 2>&1 || { tail -30 $out/gpu_tests.txt; exit 1; }
tail -2 $out/gpu_tests.txt
timeout -k 10 200 python3 tools/async_probe.py 30 > $out/async_probe.txt 2>&1 || { cat $out/async_probe.txt; exit 1; }
cat $out/async_probe.txt
for r in "4 17 107 120" "4 21 103 120" "4 25 99 120"; do
  echo "== pair_lab $r" >> $out/pair_lab.txt
  timeout -k 10 120 ./tools/pair_lab $r 10 0 >> $out/pair_lab.txt 2>&1 || { echo "pair_lab rc $?"; cat $out/pair_lab.txt; exit 1; }
done
grep -E "==|best|check" $out/pair_lab.txt
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail $out/bench.err; exit 1; }
cut -c1-400 $out/bench.json
