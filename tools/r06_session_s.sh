#!/bin/bash
# k_plane_flow with pipelined polls: tests, poisoned stress, bench A/B (lab GM_PLANE_FLOW_PIPE=0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/r06z
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_planes.py "tests/test_gpu_shard_faults.py::test_flow_backward_stall_returns" tests/test_gpu_full_size.py tests/test_gpu_checkpoint.py tests/test_gpu_parity.py tests/test_gpu_edge_shapes.py -x -q -m gpu --timeout 300 --timeout-method thread > $out/gpu_tests.txt 2>&1 || { tail -40 $out/gpu_tests.txt; exit 1; }
tail -2 $out/gpu_tests.txt
POISON=1 REPS=10 timeout -k 10 250 python3 tools/flow_check.py heaps=31:31:1:127 heaps=31:31:3:63 heaps=31:31:1:1:63 heaps=31:31:7:7:7:7 > $out/stress.txt 2>&1 || { cat $out/stress.txt; exit 1; }
echo "stress: $(grep -c 'bad words 0 ' $out/stress.txt) clean of $(grep -c 'bad words' $out/stress.txt)"
LAB=$PWD/gamesmanmpi_amd/libgamesman_hip_lab.so
b() {
  timeout -k 10 300 env "$@" python3 bench.py --gpus 1 --steps 30 --warmup 5 --no-keyed --no-cpu-baseline > $out/b.json 2> $out/b.err || { tail $out/b.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$out/b.json').read().strip().splitlines()[-1]);print('$*'.replace('$LAB','lab'), d['ms_per_step'], round(d['phase_ms']['resolve_kernels'],4), round(d['roofline']['frac'],3), d['roofline']['kernel'])"
}
true
true
true
true
true
