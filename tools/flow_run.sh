#!/bin/bash
# Runs tools/flow_lab cases in one GPU call: bash tools/flow_run.sh TAG "K var reps bpc" ...
# A case that mismatches (rc 2) or gives up waiting (rc 3) is reported and the
# next case runs; a time limit, abort or fault ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
tag=$1; shift
mkdir -p gpurun_out
out=gpurun_out/flow_$tag.log
: > $out
for c in "$@"; do
  echo "== $c" >> $out
  timeout -k 10 150 ./tools/flow_lab $c >> $out 2>&1
  rc=$?
  echo "rc $rc" >> $out
  if [ $rc -ne 0 ] && [ $rc -ne 2 ] && [ $rc -ne 3 ]; then echo "stopping after rc $rc"; cat $out; exit $rc; fi
done
cat $out
