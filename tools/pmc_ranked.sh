#!/bin/bash
# PMC passes over one RANKED toot 6x4 solve (run on the GPU box via gpurun):
#   bash tools/pmc_ranked.sh OUTDIR
# one counter group per rocprofv3 run, each bounded by its own timeout;
# summary: python3 tools/pmc_summary.py OUTDIR (per kernel)
set -e
out=${1:-gpurun_out/pmc_ranked}
export TMPDIR=/tmp
mkdir -p "$out"
cmd=(python3 tools/solve_once.py toot_and_otto_bitstring "length=6,height=4" ranked 0)
pass() {
  local name=$1
  shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d "$out/$name" -o run -- "${cmd[@]}" > "$out/$name.log" 2>&1
  echo "pass $name ok"
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass hit TCC_HIT_sum TCC_MISS_sum
pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES
