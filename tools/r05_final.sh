#!/bin/bash
# Round-5 final GPU session (gpurun): the whole GPU suite, smoke, bench x3,
# rocprof stats of one bench.  Each step under its own limit; the first
# failure ends the session.   bash tools/r05_final.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
tag=${1:-r05final}
out=gpurun_out/$tag
mkdir -p "$out"
step() {  # name limit cmd...
  local name=$1 lim=$2
  shift 2
  echo "== $name" >&2
  timeout -k 10 "$lim" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name: exit $rc" >&2; tail -20 "$out/$name.log" >&2; exit $rc; fi
}
step tests 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread
tail -1 "$out/tests.log" >&2
step smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
tail -1 "$out/smoke.log" >&2
for i in 1 2 3; do step bench$i 300 python3 bench.py; tail -1 "$out/bench$i.log" | cut -c1-200 >&2; done
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline
echo "session $tag done" >&2
