#!/bin/bash
# A/B of two builds on the bench workload: bash tools/ab_dense.sh LIB_B TAG
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in gamesmanmpi_amd/libgamesman_hip.so "$1"; do
  GM_LIBPATH=$PWD/$lib timeout -k 10 120 python3 tools/solve_once.py sum_four_to_one "heaps=31:31:31:31:31:31" dense 3 \
    > gpurun_out/${2}_$(basename $lib .so).log 2>&1 || { echo "run $lib failed"; tail gpurun_out/${2}_$(basename $lib .so).log; exit 1; }
  echo "$lib"; grep wall_ms gpurun_out/${2}_$(basename $lib .so).log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('  wall %.2f fwd %.2f bwd %.2f' % (d['wall_ms'], d['ms_forward'], d['ms_backward']), d.get('ms_resolve_kernels',''), d.get('checksum',{}).get('checksum',''))"
done
