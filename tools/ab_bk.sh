#!/bin/bash
# A/B of library variants (GM_LIBPATH) on the toot 6x4 bucketed solve:
# bash tools/ab_bk.sh build/ab_b.so build/ab_c.so ...  (default library first)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in default "$@"; do
  if [ "$lib" = default ]; then unset GM_LIBPATH; else export GM_LIBPATH=$PWD/$lib; fi
  echo "== $lib"
  timeout -k 10 200 python3 tools/solve_once.py toot_and_otto_bitstring "length=6,height=4" bucketed 2 > gpurun_out/ab_bk.jsonl 2>&1 || { echo failed; tail -5 gpurun_out/ab_bk.jsonl; exit 1; }
  python3 -c "
import json,sys
for l in open('gpurun_out/ab_bk.jsonl'):
    if l.startswith('{'):
        r=json.loads(l); print(round(r['ms_total'],1), round(r['ms_forward'],1), round(r['ms_backward'],1), r.get('checksum',{}).get('checksum',''))"
done
