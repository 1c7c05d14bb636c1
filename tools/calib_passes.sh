set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/cal2
timeout -k 10 60 tools/calib_fetch > gpurun_out/cal2/plain.json
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/cal2/fetch -o run -- tools/calib_fetch > gpurun_out/cal2/fetch.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/cal2/hit -o run -- tools/calib_fetch > gpurun_out/cal2/hit.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/cal2/write -o run -- tools/calib_fetch > gpurun_out/cal2/write.log 2>&1
echo ok
