set -o pipefail
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s6_prof -o run -- python3 tools/group_bench.py 2 2 > gpurun_out/s6.log 2>&1 || exit 1
echo ok
