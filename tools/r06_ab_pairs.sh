#!/bin/bash
# pair items in the one-launch backward: tests + poisoned stress on the new build, then same-box A/B
# (pairs / lab GM_PLANE_FLOW_PAIRS=0 / the previous commit's library)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/r06ac
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_planes.py "tests/test_gpu_shard_faults.py::test_flow_backward_stall_returns" tests/test_gpu_full_size.py -x -q -m gpu --timeout 300 --timeout-method thread > $out/gpu_tests.txt 2>&1 || { tail -40 $out/gpu_tests.txt; exit 1; }
tail -1 $out/gpu_tests.txt
POISON=1 REPS=10 timeout -k 10 250 python3 tools/flow_check.py heaps=31:31:1:127 heaps=31:31:3:63 heaps=31:31:1:1:63 heaps=31:31:7:7:7:7 heaps=31:31:15:15:15 > $out/stress.txt 2>&1 || { cat $out/stress.txt; exit 1; }
echo "stress: $(grep -c 'bad words 0 ' $out/stress.txt) clean of $(grep -c 'bad words' $out/stress.txt)"
PREV=$PWD/gamesmanmpi_amd/libgamesman_hip_prev.so
LAB=$PWD/gamesmanmpi_amd/libgamesman_hip_lab.so
b() {
  timeout -k 10 300 env "$@" python3 bench.py --gpus 1 --steps 40 --warmup 5 --no-keyed --no-cpu-baseline > $out/b.json 2> $out/b.err || { tail $out/b.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$out/b.json').read().strip().splitlines()[-1]);print('$*'.replace('$PREV','prev').replace('$LAB','lab'), d['ms_per_step'], round(d['phase_ms']['resolve_kernels'],4), round(d['roofline']['frac'],3))"
}
for i in 1 2 3; do b X=pairs; b GM_LIBPATH=$LAB GM_PLANE_FLOW_PAIRS=0; b GM_LIBPATH=$PREV; done
