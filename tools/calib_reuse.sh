set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/cal3
timeout -k 10 60 tools/calib_fetch > gpurun_out/cal3/plain.json
timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/cal3/hit -o run -- tools/calib_fetch > gpurun_out/cal3/hit.log 2>&1
echo ok
