#!/bin/bash
# Round-3 closing measurement session (staged shards, narrow runs): the -m gpu suite, PMC passes over one solve of
# the bench workload (PLANES layout) -> profiles/pmc_traffic.json, the bench
# line, and a rocprofv3 kernel trace + stats of a short bench.  Every step
# under its own timeout; the script stops at the first failure.
# Usage: bash tools/gpu_r03.sh TAG [skip-tests]
set -o pipefail
tag=${1:-r03r}
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${tag}_gpu_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/${tag}_gpu_tests.log; exit 1; }
  echo tests ok
  tail -3 gpurun_out/${tag}_gpu_tests.log
fi
out=gpurun_out/${tag}_pmc
mkdir -p $out
cmd=(python3 tools/solve_once.py sum_four_to_one "heaps=31:31:31:31:31:31" auto 0 timing)
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$out/$name" -o run -- "${cmd[@]}" > "$out/$name.log" 2>&1 || { echo "pass $name failed"; exit 1; }
  echo "pass $name ok"
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass hit TCC_HIT_sum TCC_MISS_sum
pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_BUSY_CYCLES
python3 tools/pmc_summary.py --traffic "sum_four_to_one heaps=31:31:31:31:31:31" gpurun_out/${tag}_pmc_traffic.json $out > /dev/null || exit 1
python3 tools/pmc_summary.py $out k_plane > gpurun_out/${tag}_pmc_summary.txt 2>&1 || true
cp gpurun_out/${tag}_pmc_traffic.json profiles/pmc_traffic.json
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err \
  || { echo bench failed; tail -20 gpurun_out/${tag}_bench.err; exit 1; }
echo bench ok
cat gpurun_out/${tag}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run \
  -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-keyed > gpurun_out/${tag}_prof.log 2>&1 \
  || { echo prof failed; tail -20 gpurun_out/${tag}_prof.log; exit 1; }
python3 tools/kstats.py $(find gpurun_out/${tag}_prof -name '*kernel_stats.csv' | head -1) | head -20
python3 tools/trace_levels.py $(find gpurun_out/${tag}_prof -name '*kernel_trace.csv' | head -1) 8 k_plane_reach > gpurun_out/${tag}_trace_levels.txt 2>&1 || true
tail -8 gpurun_out/${tag}_trace_levels.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/${tag}_smoke.log; exit 1; }
tail -1 gpurun_out/${tag}_smoke.log
