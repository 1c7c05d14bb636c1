#!/bin/bash
# Per-shard PLANES group timings for several staged key skews (GM_PLANE_STAGE_K):
#   bash tools/stage_k_sweep.sh TAG "WORLDS" "KS"   e.g. r04j "4 8" "2 3 4 5"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
tag=$1; worlds=${2:-"4 8"}; ks=${3:-"2 3 4 5"}
mkdir -p gpurun_out
for w in $worlds; do
  for k in $ks; do
    GM_PLANE_STAGE_K=$k timeout -k 10 300 python -u tools/group_planes.py $w 3 > gpurun_out/${tag}_w${w}_k${k}.jsonl 2>&1 \
      || { echo "w $w k $k failed"; tail -5 gpurun_out/${tag}_w${w}_k${k}.jsonl; exit 1; }
    echo "w $w k $k: $(tail -1 gpurun_out/${tag}_w${w}_k${k}.jsonl)"
  done
done
