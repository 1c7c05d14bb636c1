#!/bin/bash
# SQ / TCC counter passes over one toot 6x4 bucketed solve (no warm-up, no
# checksum): bash tools/pmc_bk.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/pmc_bk}
export TMPDIR=/tmp
mkdir -p "$out"
cmd=(python3 tools/solve_once.py toot_and_otto_bitstring "length=6,height=4" bucketed 0)
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$out/$name" -o run -- "${cmd[@]}" > "$out/$name.log" 2>&1 || { echo "pass $name failed"; exit 1; }
  echo "pass $name ok"
}
pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD
pass sq2 SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVES
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass tcc TCC_HIT_sum TCC_MISS_sum
