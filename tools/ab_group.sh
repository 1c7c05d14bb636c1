#!/bin/bash
# A/B of library variants (GM_LIBPATH) on the in-process group solve of the
# N-GPU bench shape (tools/group_time.py): bash tools/ab_group.sh WORLD lib ...
set -o pipefail
mkdir -p gpurun_out
world=$1; shift
run() {
  local lib=$1
  if [ "$lib" = default ]; then unset GM_LIBPATH; else export GM_LIBPATH=$PWD/$lib; fi
  timeout -k 10 200 python3 tools/group_time.py $world ${REPS:-4} > gpurun_out/ab_group.jsonl 2>&1 \
    || { echo "run $lib failed"; tail -5 gpurun_out/ab_group.jsonl; exit 1; }
  python3 -c "
import json
out=[]
for l in open('gpurun_out/ab_group.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); out.append('%.1f/%.1f/%.1f' % (d['ms_total'], d['ms_forward'], d['ms_backward']))
print('$lib:', ' | '.join(out[1:]))"
}
for pass in 1 2; do
  for lib in default "$@"; do run $lib; done
done
