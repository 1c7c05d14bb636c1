#!/bin/bash
# Two PMC passes (HBM-side fetch bytes, L2 hit/miss) over one bench step:
#   bash tools/pmc_quick.sh OUTDIR [bench args...]
set -e
out=${1:-gpurun_out/pmcq}
shift || true
args=("$@")
[ ${#args[@]} -eq 0 ] && args=(--steps 1 --warmup 0 --no-cpu-baseline)
export TMPDIR=/tmp
mkdir -p "$out"
pass() {
  local name=$1
  shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d "$out/$name" -o run \
    -- python3 bench.py "${args[@]}" > "$out/$name.log" 2>&1
  echo "pass $name ok"
}
pass fetch FETCH_SIZE
pass hit TCC_HIT_sum TCC_MISS_sum
