#!/bin/bash
# round 3 closing-style session: full -m gpu suite, smoke, bench line, rocprof
# of the bench, and a HIP API trace of the othello 4x4 8-shard md5 group solve
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r03k}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || { echo tests failed; grep -v "^  " gpurun_out/${tag}_gpu_tests.log | tail -30; exit 1; }
tail -2 gpurun_out/${tag}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/${tag}_smoke.log; exit 1; }
tail -1 gpurun_out/${tag}_smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { echo bench failed; tail -20 gpurun_out/${tag}_bench.err; exit 1; }
cat gpurun_out/${tag}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-keyed > gpurun_out/${tag}_prof.log 2>&1 || { echo prof failed; tail -20 gpurun_out/${tag}_prof.log; exit 1; }
python3 tools/kstats.py gpurun_out/${tag}_prof/run_kernel_stats.csv | head -8
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --output-format csv -d gpurun_out/${tag}_oth8 -o run -- python3 tools/group_keyed_time.py othello_bit_new "length=4,height=4" 8 2 > gpurun_out/${tag}_oth8.log 2>&1 || { echo oth8 trace failed; tail -20 gpurun_out/${tag}_oth8.log; exit 1; }
tail -2 gpurun_out/${tag}_oth8.log
