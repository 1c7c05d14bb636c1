#!/bin/bash
# ticketed dataflow backward (product visit) against the product's per-level launches: grid / sequences / sleep sweep
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/r06j
mkdir -p $out
run() {
  echo "== $*" >> $out/flow2.txt
  timeout -k 10 60 ./tools/flow2_lab "$@" >> $out/flow2.txt 2>&1 || { echo "rc $?" >> $out/flow2.txt; cat $out/flow2.txt; exit 1; }
}
run 0 5
for ns in 2 4 8 16; do run 1 5 2 $ns 8; done
for sl in 1 2 4 16; do run 1 5 2 4 $sl; done
for b in 3 4; do run 1 5 $b 8 4; done
run 0 5
grep -h "^var\|^==" $out/flow2.txt
