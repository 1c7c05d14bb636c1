#!/bin/bash
# A/B sweep of environment knobs over the default bench shape:
#   bash tools/ab_sweep.sh OUT "ENV=VAL ..." "ENV=VAL ..." ...
# one bench run (3 steps, no CPU baseline) per setting, each under its own
# time limit; stops at the first failure.
out=$1
shift
mkdir -p "$(dirname "$out")"
: > "$out"
for setting in "$@"; do
  env $setting timeout -k 10 120 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > /tmp/ab.json || exit 1
  python3 -c "import json,sys; d=json.load(open('/tmp/ab.json')); print(json.dumps({'setting': sys.argv[1], 'ms_per_step': d['ms_per_step'], 'resolve_ms': d['phase_ms']['resolve_kernels'], 'pull_ms': d['phase_ms']['expand_kernels'], 'frac': d['roofline']['frac']}))" "$setting" >> "$out"
done
cat "$out"
