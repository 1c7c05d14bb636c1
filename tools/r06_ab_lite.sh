#!/bin/bash
# queued one-launch solves recording only start/completion events: tests + same-box A/B (lab GM_PLANE_FLOW_LITE=0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/r06af
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_planes.py -x -q -m gpu --timeout 300 --timeout-method thread > $out/gpu_tests.txt 2>&1 || { tail -30 $out/gpu_tests.txt; exit 1; }
tail -1 $out/gpu_tests.txt
LAB=$PWD/gamesmanmpi_amd/libgamesman_hip_lab.so
b() {
  timeout -k 10 300 env "$@" python3 bench.py --gpus 1 --steps 40 --warmup 5 --no-keyed --no-cpu-baseline > $out/b.json 2> $out/b.err || { tail $out/b.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$out/b.json').read().strip().splitlines()[-1]);print('$*'.replace('$LAB','lab'), d['ms_per_step'], round(d['phase_ms']['resolve_kernels'],4), round(d['roofline']['frac'],3))"
}
for i in 1 2 3; do b X=lite; b GM_LIBPATH=$LAB GM_PLANE_FLOW_LITE=0; done
