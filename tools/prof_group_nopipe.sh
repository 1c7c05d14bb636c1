set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s8_tests.log 2>&1 || { echo tests failed; exit 1; }
timeout -k 10 200 python3 tools/group_bench.py 2 3 > gpurun_out/s8_g2.json 2>&1 || exit 1
GM_SHARD_NOPIPE=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s8_prof -o run -- python3 tools/group_bench.py 2 2 > gpurun_out/s8.log 2>&1 || exit 1
echo ok
