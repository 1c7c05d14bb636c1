#!/bin/bash
# BUCKETED count-free expand staged in one run per XCD and partition (wide levels) against one run
# per partition (the previous library, GM_LIBPATH=prev): the BUCKETED GPU tests, then same-box A/B of
# the keyed toot 6x4 BUCKETED solve
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/r06ap
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_keyed.py tests/test_gpu_parity.py tests/test_toot_6x4_fixtures.py \
  tests/test_gpu_full_size.py tests/test_gpu_edge_shapes.py tests/test_gpu_checkpoint.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > $out/gpu_tests_bk.txt 2>&1 || { tail -40 $out/gpu_tests_bk.txt; exit 1; }
tail -1 $out/gpu_tests_bk.txt
PREV=$PWD/gamesmanmpi_amd/libgamesman_hip_prev.so
b() {
  timeout -k 10 300 env "$@" python3 tools/solve_once.py toot_and_otto_bitstring "length=6,height=4" bucketed 3 > $out/s.txt 2>&1 || { tail $out/s.txt; exit 1; }
  python3 -c "
import json
L=[json.loads(l) for l in open('$out/s.txt') if l.startswith('{')]
print('$*'.replace('$PREV','prev'), [round(x['ms_total'],1) for x in L], L[-1].get('checksum', L[-1].get('root')))"
}
for i in 1 2; do b X=xcd || exit 1; b GM_LIBPATH=$PREV || exit 1; done
