#!/bin/bash
# PMC passes over one bench step (run on the GPU box via gpurun):
#   bash tools/pmc_passes.sh OUTDIR [bench args...]
# One counter group per rocprofv3 run (MI355X_MICROARCH.md "rocprofv3 PMC
# slots": FETCH_SIZE and WRITE_SIZE cannot share a pass), each bounded by
# its own timeout; the script stops at the first failing pass.
set -e
out=${1:-gpurun_out/pmc}
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
pass write WRITE_SIZE
pass hit TCC_HIT_sum TCC_MISS_sum
pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES
