#!/bin/bash
# PMC passes on the final tree: the bench (PLANES k_plane_flow + keyed toot 6x4) and one RANKED toot 6x4 solve
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/r06q
mkdir -p $out
export TMPDIR=/tmp
bash tools/pmc_passes.sh $out/pmc --steps 2 --warmup 1 --no-cpu-baseline || exit 1
bash tools/pmc_ranked.sh $out/pmc_ranked || exit 1
