#!/bin/bash
# Which child streams miss in L2: diagnostic builds of the quad resolve with
# streams skipped (-DGM_DIAG_SKIP bitmask: 1<<i heap-i children, 64 the
# heap-1 lower quads, 128 the stores; tools/diag_so/), each timed and given
# one TCC hit/miss pass.  Results of these builds are wrong by construction.
export TMPDIR=/tmp
out=gpurun_out/diag
mkdir -p $out
: > $out/times.jsonl
for m in "$@"; do
  GM_LIBPATH=$PWD/tools/diag_so/libgm_diag$m.so timeout -k 10 120 python3 tools/diag_solve.py >> $out/times.jsonl 2> $out/err$m.log || exit 1
  GM_LIBPATH=$PWD/tools/diag_so/libgm_diag$m.so timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $out/m$m -o run -- python3 tools/diag_solve.py > $out/pmc$m.log 2>&1 || exit 1
done
echo ok
