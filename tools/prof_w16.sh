# Kernel stats of the 2-shard group solve, then PMC passes of the default
# bench (16-bit table): bash tools/prof_w16.sh TAG
set -o pipefail
tag=${1:-w16}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_gprof -o run -- python3 tools/group_bench.py 2 2 > gpurun_out/${tag}_gprof.log 2>&1 || { echo group prof failed; exit 1; }
bash tools/pmc_passes.sh gpurun_out/${tag}_pmc || { echo pmc failed; exit 1; }
echo ok
