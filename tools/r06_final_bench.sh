#!/bin/bash
# the driver's bench command line + a rocprofv3 kernel-trace --stats run of the same bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/r06ah
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail $out/bench.err; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $out/bench_prof.json 2> $out/bench_prof.err || { tail $out/bench_prof.err; exit 1; }
