#!/bin/bash
# A/B of library variants (GM_LIBPATH) on the bench workload (dense 2^30):
# bash tools/ab_dense.sh build/ab_x.so ...  -- a warm-up process first, then the
# default library and each variant twice, interleaved.  A variant is a
# library path or flags=N (the default library, solver flags N); PATH:N or
# default:N runs that library with solver flags N.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  local lib=$1
  unset SOLVE_FLAGS
  local path=${lib%%:*}
  if [ "$path" != "$lib" ]; then export SOLVE_FLAGS=${lib#*:}; fi
  if [ "$path" = default ]; then unset GM_LIBPATH
  elif [ "${path#flags=}" != "$path" ]; then unset GM_LIBPATH; export SOLVE_FLAGS=${path#flags=}
  else export GM_LIBPATH=$PWD/$path; fi
  timeout -k 10 120 python3 tools/solve_once.py sum_four_to_one "heaps=31:31:31:31:31:31" dense ${REPS:-4} \
    > gpurun_out/ab_dense.jsonl 2>&1 || { echo "run $lib failed"; tail -5 gpurun_out/ab_dense.jsonl; exit 1; }
  python3 -c "
import json
out=[]
for l in open('gpurun_out/ab_dense.jsonl'):
    if l.startswith('{'):
        d=json.loads(l)
        if 'checksum' not in d: out.append('%.2f/%.2f/%.2f' % (d['ms_total'], d['ms_forward'], d['ms_backward']))
        else: out.append(d['checksum']['checksum'])
print('$lib:', ' | '.join(out))"
}
REPS=1 run default > /dev/null
for pass in 1 2; do
  for lib in default "$@"; do run $lib; done
done
