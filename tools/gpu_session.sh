# One GPU call: GPU tests, the default bench line, and its rocprofv3 kernel
# stats (csv).  bash tools/gpu_session.sh TAG
set -o pipefail
tag=${1:-run}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo tests failed; exit 1; }
timeout -k 10 180 python bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { echo bench failed; exit 1; }
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run -- python bench.py --no-cpu-baseline > gpurun_out/${tag}_prof.log 2>&1 || { echo prof failed; exit 1; }
echo done
