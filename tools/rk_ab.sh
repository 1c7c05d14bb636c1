#!/bin/bash
# A/B of a RANKED kernel knob on toot 6x4 (GPU box), each value twice:
#   bash tools/rk_ab.sh TAG [VAR [VALUES...]]   (default GM_RK_SLICED 0 1)
#   -> gpurun_out/TAG_rk_<VAR><value>.jsonl
# e.g. bash tools/rk_ab.sh r04zf GM_RK_SLICED 0 1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
tag=$1
var=${2:-GM_RK_SLICED}
shift 2 2>/dev/null
vals=("$@")
[ ${#vals[@]} -eq 0 ] && vals=(0 1)
for rep in 1 2; do
  for v in "${vals[@]}"; do
    env "$var=$v" timeout -k 10 300 python -u tools/solve_once.py toot_and_otto_bitstring "length=6,height=4" ranked 3 \
      >> gpurun_out/${tag}_rk_$var$v.jsonl 2>&1 || { echo "$var=$v failed"; tail -20 gpurun_out/${tag}_rk_$var$v.jsonl; exit 1; }
  done
done
for v in "${vals[@]}"; do
  echo "$var=$v"
  grep -o '"ms_forward": [0-9.]*, "ms_backward": [0-9.]*' gpurun_out/${tag}_rk_$var$v.jsonl
done
