#!/bin/bash
# A/B of library variants (GM_LIBPATH) on the toot 6x4 bucketed solve:
# bash tools/ab_bk.sh build/ab_b.so ...  -- one throwaway warm-up process
# (the first process on a fresh box runs ~6 % slow), then the default
# library and each variant twice, interleaved.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  local lib=$1
  if [ "$lib" = default ]; then unset GM_LIBPATH; else export GM_LIBPATH=$PWD/$lib; fi
  timeout -k 10 200 python3 tools/solve_once.py toot_and_otto_bitstring "length=6,height=4" bucketed ${REPS:-2} > gpurun_out/ab_bk.jsonl 2>&1 || { echo failed; tail -5 gpurun_out/ab_bk.jsonl; exit 1; }
  python3 -c "
import json,sys
out=[]
for l in open('gpurun_out/ab_bk.jsonl'):
    if l.startswith('{'):
        r=json.loads(l); out.append('%.1f/%.1f/%.1f %s' % (r['ms_total'], r['ms_forward'], r['ms_backward'], r.get('checksum',{}).get('checksum','')))
print('$lib:', ' | '.join(out))"
}
REPS=1 run default > /dev/null
for pass in 1 2; do
  for lib in default "$@"; do run $lib; done
done
