#!/bin/bash
# pad_lab session (GPU box): timings of the padded-stride placement against
# the natural one, diagnostics, and PMC passes.  Output in gpurun_out/pad_<tag>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
tag=${1:-a}
out=gpurun_out/pad_$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run() {  # name, args...
  local n=$1; shift
  echo "== pad_lab $*" | tee -a "$out/log.txt"
  timeout -k 10 120 ./tools/pad_lab "$@" >> "$out/log.txt" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "pad_lab $*: exit $rc" | tee -a "$out/log.txt"; exit $rc; fi
}
run t0 0 10 1 1 0
run t1 1 10 1 1 0
run t2 2 10 0 1 0
run t3 5 10 0 1 0
run t4 0 10 1 0 1
run t5 0 10 1 0 2
run t6 0 10 1 0 3
for p in 0 1; do
  for c in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "WRITE_SIZE"; do
    f=$(echo $c | tr ' ' _)
    timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --stats -d $out/pmc_${p}_$f -o run -- ./tools/pad_lab $p 3 0 0 0 > $out/pmc_${p}_$f.log 2>&1 || { echo "pmc $p $c failed"; exit 3; }
  done
done
cat $out/log.txt
