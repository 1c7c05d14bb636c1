#!/bin/bash
# Runs tools/stream_lab over a list of "[ENV=..] K variant reps level_times threshold"
# argument sets, each under its own time limit; output to gpurun_out/stream_<tag>.log.
#   bash tools/stream_run.sh TAG "6 0 10 1" "6 4 10 1 4096" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
tag=$1
shift
log=gpurun_out/stream_$tag.log
: > "$log"
for a in "$@"; do
  echo "== stream_lab $a" >> "$log"
  envs=()
  set -- $a
  while [[ "$1" == *=* ]]; do envs+=("$1"); shift; done
  timeout -k 10 120 env "${envs[@]}" ./tools/stream_lab "$@" >> "$log" 2>&1
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 2 ]; then echo "stream_lab $a: exit $rc" >> "$log"; cat "$log"; exit $rc; fi
done
cat "$log"
