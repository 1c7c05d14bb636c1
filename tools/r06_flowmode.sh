#!/bin/bash
# k_plane_flow memory-ordering A/B on chain-like shapes, table poisoned before every solve
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/r06m
mkdir -p $out
echo "== product" >> $out/flowmode.txt
POISON=1 REPS=12 timeout -k 10 250 python3 tools/flow_check.py heaps=31:31:1:127 heaps=31:31:3:63 heaps=31:31:7:7:7:7 >> $out/flowmode.txt 2>&1 || { echo "rc $?" >> $out/flowmode.txt; cat $out/flowmode.txt; exit 1; }
for m in 1 4 5; do
  echo "== lab mode $m" >> $out/flowmode.txt
  GM_LIBPATH=$PWD/gamesmanmpi_amd/libgamesman_hip_lab.so GM_PLANE_FLOW_MODE=$m POISON=1 REPS=8 timeout -k 10 200 python3 tools/flow_check.py heaps=31:31:1:127 heaps=31:31:3:63 heaps=31:31:7:7:7:7 >> $out/flowmode.txt 2>&1 || { echo "rc $?" >> $out/flowmode.txt; cat $out/flowmode.txt; exit 1; }
done
grep -v amdgpu.ids $out/flowmode.txt | grep -v "bad words 0 "
echo; grep -c "bad words 0 " $out/flowmode.txt
