#!/bin/bash
# dataflow lab: plain loads without acquire (var 9) against the lab body's per-level launches (var 7) and sc1 loads (var 1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/r06h
mkdir -p $out
for v in 0 7 1 9 9; do
  echo "== var $v" >> $out/flow.txt
  timeout -k 10 60 ./tools/flow_lab 6 $v 5 >> $out/flow.txt 2>&1 || { echo "rc $?" >> $out/flow.txt; cat $out/flow.txt; exit 1; }
done
cat $out/flow.txt
