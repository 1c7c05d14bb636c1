#!/bin/bash
# one-launch backward: XCD slabs of the top digit (lab GM_PLANE_FLOW_DEAL=1) against even per-level chunks
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/r06aj
mkdir -p $out
export TMPDIR=/tmp
LAB=$PWD/gamesmanmpi_amd/libgamesman_hip_lab.so
GM_LIBPATH=$LAB GM_PLANE_FLOW_DEAL=1 POISON=1 REPS=4 timeout -k 10 250 python3 tools/flow_check.py heaps=31:31:1:127 heaps=31:31:3:63 heaps=31:31:7:7:7:7 > $out/stress.txt 2>&1 || { cat $out/stress.txt; exit 1; }
echo "stress: $(grep -c 'bad words 0 ' $out/stress.txt) clean of $(grep -c 'bad words' $out/stress.txt)"
b() {
  timeout -k 10 300 env "$@" python3 bench.py --gpus 1 --steps 40 --warmup 5 --no-keyed --no-cpu-baseline > $out/b.json 2> $out/b.err || { tail $out/b.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$out/b.json').read().strip().splitlines()[-1]);print('$*'.replace('$LAB','lab'), d['ms_per_step'], round(d['phase_ms']['resolve_kernels'],4), round(d['roofline']['frac'],3))"
}
for i in 1 2; do b X=default; b GM_LIBPATH=$LAB GM_PLANE_FLOW_DEAL=1; done
