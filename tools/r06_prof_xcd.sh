#!/bin/bash
# per-kernel times (rocprofv3 stats) and WRITE_SIZE / FETCH_SIZE of the toot 6x4 BUCKETED solve, XCD runs against the previous library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/r06aq
mkdir -p $out
export TMPDIR=/tmp
PREV=$PWD/gamesmanmpi_amd/libgamesman_hip_prev.so
run() {
  local tag=$1 lib=$2
  GM_LIBPATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/st_$tag -o run -- python3 tools/solve_once.py toot_and_otto_bitstring "length=6,height=4" bucketed 1 > $out/st_$tag.log 2>&1 || { tail $out/st_$tag.log; return 1; }
  GM_LIBPATH=$lib timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/wr_$tag -o run -- python3 tools/solve_once.py toot_and_otto_bitstring "length=6,height=4" bucketed 0 > $out/wr_$tag.log 2>&1 || { tail $out/wr_$tag.log; return 1; }
  GM_LIBPATH=$lib timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fe_$tag -o run -- python3 tools/solve_once.py toot_and_otto_bitstring "length=6,height=4" bucketed 0 > $out/fe_$tag.log 2>&1 || { tail $out/fe_$tag.log; return 1; }
  echo "$tag ok"
}
run xcd $PWD/gamesmanmpi_amd/libgamesman_hip.so && run prev $PREV
