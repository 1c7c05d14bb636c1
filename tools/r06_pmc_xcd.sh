#!/bin/bash
# why the fine pass slows down on per-XCD staging runs: SQ and UTCL1 counters of the toot 6x4
# BUCKETED solve, XCD runs against the previous library (GM_LIBPATH)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/r06ar
mkdir -p $out
export TMPDIR=/tmp
PREV=$PWD/gamesmanmpi_amd/libgamesman_hip_prev.so
pass() {
  local tag=$1 lib=$2 name=$3
  shift 3
  GM_LIBPATH=$lib timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $out/${name}_$tag -o run -- python3 tools/solve_once.py toot_and_otto_bitstring "length=6,height=4" bucketed 0 > $out/${name}_$tag.log 2>&1 || { tail $out/${name}_$tag.log; return 1; }
}
for t in xcd prev; do
  lib=$PWD/gamesmanmpi_amd/libgamesman_hip.so
  [ $t = prev ] && lib=$PREV
  pass $t $lib sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES || exit 1
  pass $t $lib tlb TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum || exit 1
  pass $t $lib hit TCC_HIT_sum TCC_MISS_sum || exit 1
  echo "$t ok"
done
