#!/bin/bash
# FETCH / WRITE / L2-hit passes over one bench-workload solve: bash tools/pmc_dense.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/pmc_dense}
export TMPDIR=/tmp
mkdir -p "$out"
cmd=(python3 tools/solve_once.py sum_four_to_one "heaps=31:31:31:31:31:31" dense 0 timing)
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$out/$name" -o run -- "${cmd[@]}" > "$out/$name.log" 2>&1 || { echo "pass $name failed"; exit 1; }
  echo "pass $name ok"
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass hit TCC_HIT_sum TCC_MISS_sum
pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_BUSY_CYCLES
