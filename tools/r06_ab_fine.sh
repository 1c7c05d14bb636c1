#!/bin/bash
# BUCKETED fine pass split over 4 workgroups per partition: full suite, then same-box A/B of the keyed
# toot 6x4 BUCKETED solve (lab GM_BK_FINE_SPLIT=0 = one workgroup per partition)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/r06ak
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.txt 2>&1 || { tail -40 $out/gpu_tests.txt; exit 1; }
tail -1 $out/gpu_tests.txt
LAB=$PWD/gamesmanmpi_amd/libgamesman_hip_lab.so
b() {
  timeout -k 10 300 env "$@" python3 tools/solve_once.py toot_and_otto_bitstring "length=6,height=4" bucketed 3 > $out/s.txt 2>&1 || { tail $out/s.txt; exit 1; }
  python3 -c "
import json
L=[json.loads(l) for l in open('$out/s.txt') if l.startswith('{')]
print('$*'.replace('$LAB','lab'), [round(x['ms_total'],1) for x in L], L[-1].get('checksum', L[-1].get('root')))"
}
for i in 1 2; do b X=split; b GM_LIBPATH=$LAB GM_BK_FINE_SPLIT=0; done
