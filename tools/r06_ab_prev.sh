#!/bin/bash
# same-box A/B: this tree (self-finishing launch), its lab build with GM_PLANE_FLOW_SELFFIN=0, and the previous commit's library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/r06y
mkdir -p $out
PREV=$PWD/gamesmanmpi_amd/libgamesman_hip_prev.so
LAB=$PWD/gamesmanmpi_amd/libgamesman_hip_lab.so
b() {
  timeout -k 10 300 env "$@" python3 bench.py --gpus 1 --steps 40 --warmup 5 --no-keyed --no-cpu-baseline > $out/b.json 2> $out/b.err || { tail $out/b.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$out/b.json').read().strip().splitlines()[-1]);print('$*'.replace('$PREV','prev').replace('$LAB','lab'), d['ms_per_step'], round(d['phase_ms']['resolve_kernels'],4), round(d['roofline']['frac'],3))"
}
for i in 1 2 3; do b X=new; b GM_LIBPATH=$PREV; done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/prof -o run -- python3 bench.py --gpus 1 --steps 10 --warmup 2 --no-keyed --no-cpu-baseline > /dev/null 2>&1 || exit 1
