#!/bin/bash
# One GPU call, as a list of steps (each under its own time limit; the
# script stops at the first failure and prints the tail of that step's log).
#   bash tools/gpu_session.sh TAG step [step ...]
# steps:
#   tests[:EXPR]   python -m pytest tests -m gpu (-k EXPR)       -> TAG_gpu_tests.log
#   smoke          __graft_entry__.smoke()                        -> TAG_smoke.log
#   bench          python bench.py --steps 20 --warmup 5          -> TAG_bench.json
#   prof           rocprofv3 --kernel-trace --stats of a short bench -> TAG_prof/
#   pmc            the PMC passes of one bench step (tools/pmc_passes.sh) -> TAG_pmc/, TAG_pmc_traffic.json
#   atomics        toot 6x4 atomic counters (tools/pmc_atomics.sh)    -> TAG_atomics.json
#   groups         per-shard PLANES group timings, N = 2 4 8 (tools/group_planes.py)
#   keyed[:B]      toot B (default 6x4) md5 group timings, N = 1 2 4 (tools/group_keyed_time.py)
# Replaces the round-by-round session scripts (tools/gpu_r0*.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
tag=${1:?usage: gpu_session.sh TAG step...}
shift
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/$tag
fail() { echo "$1 failed"; tail -30 "$2"; exit 1; }
for step in "$@"; do
  case "$step" in
    tests|tests:*)
      k=()
      [ "$step" != tests ] && k=(-k "${step#tests:}")
      timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${k[@]}" \
        > ${o}_gpu_tests.log 2>&1 || fail tests ${o}_gpu_tests.log
      tail -1 ${o}_gpu_tests.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > ${o}_smoke.log 2>&1 \
        || fail smoke ${o}_smoke.log
      tail -1 ${o}_smoke.log ;;
    bench)
      timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > ${o}_bench.json 2> ${o}_bench.err \
        || fail bench ${o}_bench.err
      cat ${o}_bench.json ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${o}_prof -o run \
        -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > ${o}_prof.log 2>&1 || fail prof ${o}_prof.log
      python3 tools/kstats.py $(find ${o}_prof -name '*kernel_stats.csv' | head -1) | head -20 ;;
    pmc)  # + the per-launch traffic bench.py reads (copy it to profiles/pmc_traffic.json)
      bash tools/pmc_passes.sh ${o}_pmc > ${o}_pmc.log 2>&1 || fail pmc ${o}_pmc.log
      python3 tools/pmc_summary.py --traffic "sum_four_to_one heaps=31:31:31:31:31:31" ${o}_pmc_traffic.json \
        ${o}_pmc > /dev/null || fail pmc-summary ${o}_pmc.log
      tail -3 ${o}_pmc.log ;;
    atomics)  # keyed toot 6x4 atomic counters -> TAG_atomics.json (copy to profiles/keyed_atomics.json)
      bash tools/pmc_atomics.sh ${o}_atomics > ${o}_atomics.log 2>&1 || fail atomics ${o}_atomics.log
      python3 tools/pmc_atomics_summary.py ${o}_atomics > ${o}_atomics.json || fail atomics-summary ${o}_atomics.log
      python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['total'])" ${o}_atomics.json ;;
    groups)
      for w in 2 4 8; do
        timeout -k 10 300 python -u tools/group_planes.py $w 3 > ${o}_group$w.jsonl 2>&1 \
          || fail "group $w" ${o}_group$w.jsonl
        tail -1 ${o}_group$w.jsonl
      done ;;
    keyed|keyed:*)
      b=6x4
      [ "$step" != keyed ] && b=${step#keyed:}
      for w in 1 2 4; do
        timeout -k 10 400 python -u tools/group_keyed_time.py toot_and_otto_bitstring \
          "length=${b%x*},height=${b#*x}" $w 2 > ${o}_keyed_${b}_w$w.jsonl 2>&1 || fail "keyed $w" ${o}_keyed_${b}_w$w.jsonl
        tail -1 ${o}_keyed_${b}_w$w.jsonl
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo session $tag done
