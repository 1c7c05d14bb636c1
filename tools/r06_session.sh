#!/bin/bash
# Round-6 GPU session: the -m gpu suite, then the 1-GPU bench (driver
# command line).  Usage: bash tools/r06_session.sh TAG [pytest args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
tag=${1:-a}; shift
out=gpurun_out/r06$tag
mkdir -p "$out"
export TMPDIR=/tmp
sel=("$@"); [ ${#sel[@]} -eq 0 ] && sel=(tests)
timeout -k 10 900 python3 -u -m pytest "${sel[@]}" -x -q -m gpu --timeout 300 --timeout-method thread > "$out/gpu_tests.txt" 2>&1
rc=$?
tail -3 "$out/gpu_tests.txt"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$out/bench.json" 2> "$out/bench.err"
rc=$?
cut -c1-600 "$out/bench.json"
exit $rc
