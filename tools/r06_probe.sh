#!/bin/bash
# forward placement A/B on the lab build (queued vs blocking steps), then the
# pair-fusion lab.  Output: gpurun_out/r06_probe.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/r06_probe.txt
: > $out
for m in 0 1 2; do
  echo "== GM_PLANE_FWD=$m (lab build)" >> $out
  GM_LIBPATH=$PWD/gamesmanmpi_amd/libgamesman_hip_lab.so GM_PLANE_FWD=$m timeout -k 10 200 python3 tools/async_probe.py 30 >> $out 2>&1 || { echo "probe $m failed"; cat $out; exit 1; }
done
echo "== pair_lab 4 17 107 120" >> $out
timeout -k 10 120 ./tools/pair_lab 4 17 107 120 10 1 >> $out 2>&1 || { echo "pair_lab rc $?" >> $out; }
cat $out
