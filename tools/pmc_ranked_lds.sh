#!/bin/bash
# One extra PMC pass over a RANKED toot 6x4 solve: where the backward's waves wait
# (LDS, scalar memory, VALU) -- run on the GPU box: bash tools/pmc_ranked_lds.sh OUTDIR
out=${1:-gpurun_out/pmc_ranked_lds}
export TMPDIR=/tmp
mkdir -p "$out"
cmd=(python3 tools/solve_once.py toot_and_otto_bitstring "length=6,height=4" ranked 0)
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_WAVES --output-format csv -d "$out/lds" -o run -- "${cmd[@]}" > "$out/lds.log" 2>&1 && echo "pass lds ok"
