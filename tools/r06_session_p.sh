#!/bin/bash
# final-tree bench (driver's default command line) + rocprofv3 kernel-trace stats of a bench run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/r06p
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py > $out/bench_default.json 2> $out/bench_default.err || { tail $out/bench_default.err; exit 1; }
tail -c 600 $out/bench_default.json; echo
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/bench_prof.json 2> $out/bench_prof.err || { tail $out/bench_prof.err; exit 1; }
ls $out/prof
