#!/bin/bash
# A/B of the RANKED backward's entries per pass on toot 6x4 (GPU box):
#   bash tools/rk_ab.sh TAG   -> gpurun_out/TAG_rk_u{2,4}.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for u in 2 4 2 4; do
  GM_RK_UNROLL=$u timeout -k 10 300 python -u tools/solve_once.py toot_and_otto_bitstring "length=6,height=4" ranked 3 \
    >> gpurun_out/$1_rk_u$u.jsonl 2>&1 || { echo "u=$u failed"; tail -20 gpurun_out/$1_rk_u$u.jsonl; exit 1; }
done
for u in 2 4; do echo "u=$u"; grep -o '"ms_backward": [0-9.]*' gpurun_out/$1_rk_u$u.jsonl; done
