#!/bin/bash
# forward at the narrow tail: plane tests, the async probe, the bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/r06d
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_planes.py "tests/test_gpu_full_size.py::test_gpu_sum_31x6_checksum" tests/test_gpu_checkpoint.py -x -q -m gpu --timeout 300 --timeout-method thread > $out/gpu_tests.txt 2>&1 || { tail -30 $out/gpu_tests.txt; exit 1; }
tail -2 $out/gpu_tests.txt
timeout -k 10 200 python3 tools/async_probe.py 30 > $out/async_probe.txt 2>&1 || { cat $out/async_probe.txt; exit 1; }
cat $out/async_probe.txt
for m in 1 2; do
  echo "== GM_PLANE_FWD=$m (lab build)" >> $out/fwd_ab.txt
  GM_LIBPATH=$PWD/gamesmanmpi_amd/libgamesman_hip_lab.so GM_PLANE_FWD=$m timeout -k 10 200 python3 tools/async_probe.py 30 >> $out/fwd_ab.txt 2>&1 || { cat $out/fwd_ab.txt; exit 1; }
done
cat $out/fwd_ab.txt
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail $out/bench.err; exit 1; }
cut -c1-300 $out/bench.json
