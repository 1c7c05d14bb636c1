#!/bin/bash
# Atomic-operation counters of one toot 6x4 BUCKETED solve (the bench's keyed
# record), one rocprofv3 run per counter group, plus a kernel trace for the
# durations: bash tools/pmc_atomics.sh OUTDIR
#   l2     TCC_ATOMIC_sum (atomic requests the L2s serve), TCC_EA0_ATOMIC_sum
#          (the part sent on to memory)
#   lds    SQ_INSTS_LDS_ATOMIC (LDS atomic wave-instructions),
#          SQ_INSTS_LDS_ATOMIC_BANDWIDTH (64-B units of active lanes),
#          SQ_LDS_ATOMIC_RETURN (returning-atomic LDS cycles), SQ_INSTS_LDS
#   trace  --kernel-trace --stats
# Summary: python3 tools/pmc_atomics_summary.py OUTDIR > profiles/keyed_atomics.json
set -o pipefail
out=${1:-gpurun_out/pmc_atomics}
export TMPDIR=/tmp
mkdir -p "$out"
cmd=(python3 tools/solve_once.py toot_and_otto_bitstring "length=6,height=4" bucketed 0)
pass() {
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 "$@" --output-format csv -d "$out/$name" -o run -- "${cmd[@]}" > "$out/$name.log" 2>&1 \
    || { echo "pass $name failed"; tail -5 "$out/$name.log"; exit 1; }
  echo "pass $name ok"
}
pass l2 --pmc TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum
pass lds --pmc SQ_INSTS_LDS_ATOMIC SQ_INSTS_LDS_ATOMIC_BANDWIDTH SQ_LDS_ATOMIC_RETURN SQ_INSTS_LDS
pass trace --kernel-trace --stats
