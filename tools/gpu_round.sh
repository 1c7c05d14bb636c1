#!/bin/bash
# One measurement session: the -m gpu suite, the bench line, a rocprofv3
# kernel-stats summary of a short bench, and the dense PMC passes whose
# per-launch traffic bench.py reads (profiles/pmc_traffic.json).  Each step
# under its own timeout; the script stops at the first failure.
# Usage: bash tools/gpu_round.sh TAG
set -o pipefail
tag=${1:-round}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/${tag}_gpu_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/${tag}_gpu_tests.log; exit 1; }
echo tests ok
tail -3 gpurun_out/${tag}_gpu_tests.log
bash tools/pmc_dense.sh gpurun_out/${tag}_pmc || exit 1
python3 tools/pmc_summary.py --traffic "sum_four_to_one heaps=31:31:31:31:31:31" gpurun_out/${tag}_pmc_traffic.json \
  gpurun_out/${tag}_pmc > /dev/null || exit 1
cp gpurun_out/${tag}_pmc_traffic.json profiles/pmc_traffic.json
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err \
  || { echo bench failed; tail -20 gpurun_out/${tag}_bench.err; exit 1; }
echo bench ok
cat gpurun_out/${tag}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run \
  -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${tag}_prof.log 2>&1 \
  || { echo prof failed; tail -20 gpurun_out/${tag}_prof.log; exit 1; }
python3 tools/kstats.py $(find gpurun_out/${tag}_prof -name '*kernel_stats.csv' | head -1) | head -20
