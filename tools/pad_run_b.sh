#!/bin/bash
# pad_lab session b: plain vs write-through row stores (time + PMC), and the
# per-launch anatomy of single levels.  Output in gpurun_out/pad_b/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/pad_${1:-b}
mkdir -p "$out"
run() {
  echo "== pad_lab $*" >> "$out/log.txt"
  timeout -k 10 120 ./tools/pad_lab "$@" >> "$out/log.txt" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "pad_lab $*: exit $rc" >> "$out/log.txt"; cat "$out/log.txt"; exit $rc; fi
}
run 0 10 1 1 0 1
run 0 10 0 0 0 0
for s in 4 10 20 40 62; do
  for d in 0 2 4 5; do run 0 1 0 0 $d 0 $s; done
  run -1 1 0 0 0 0 $s
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for c in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "WRITE_SIZE"; do
  f=$(echo $c | tr ' ' _)
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --stats -d $out/pmc_plain_$f -o run -- ./tools/pad_lab 0 3 0 0 0 1 > $out/pmc_plain_$f.log 2>&1 || { echo "pmc $c failed"; exit 3; }
done
cat $out/log.txt
