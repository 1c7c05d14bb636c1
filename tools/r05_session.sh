#!/bin/bash
# Round-5 measurement session (gpurun): bench x3, rocprof stats of one bench,
# the PLANES PMC passes, and kernel traces of the staged shard groups on ONE
# stream (every key alone on the GPU: the per-key durations the pipeline model
# takes).  Each GPU step under its own limit; the first failure ends it.
#   bash tools/r05_session.sh TAG [what...]   what: bench prof pmc stage rows
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
tag=${1:-r05g}
shift
what=${*:-bench prof pmc stage}
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
for w in $what; do
  case $w in
    bench)
      for i in 1 2 3; do step bench$i 240 python3 bench.py; tail -1 "$out/bench$i.log" >&2; done ;;
    prof)
      step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline ;;
    pmc)
      step pmc 700 bash tools/pmc_passes.sh "$out/pmc"
      python3 tools/pmc_summary.py "$out/pmc" k_plane k_rk > "$out/pmc_summary.txt" 2>&1 || true ;;
    stage)
      for wk in "2 1" "2 2" "4 1" "4 2" "4 3" "8 1" "8 2" "8 3"; do
        set -- $wk
        GM_PLANE_STAGE_K=$2 step stage_w$1_k$2 240 rocprofv3 --kernel-trace --output-format csv \
          -d "$out/stage_w$1_k$2" -o run -- python3 tools/group_planes.py "$1" 2
      done ;;
    rows)  # the row deal's bench shapes (bench.heaps_for), one stream
      for w in 2 4 8; do
        step rows_w$w 240 rocprofv3 --kernel-trace --output-format csv -d "$out/rows_w$w" -o run -- \
          python3 tools/group_planes.py "$w" 2
      done ;;
  esac
done
echo "session $tag done" >&2
