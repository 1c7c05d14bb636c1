set -o pipefail
export TMPDIR=/tmp
bash tools/ab_sweep.sh gpurun_out/ab7.jsonl "GM_GROUP_TILE=0" "GM_GROUP_TILE=128" "GM_GROUP_TILE=256" "GM_GROUP_TILE=-1" || exit 1
GM_GROUP_TILE=256 bash tools/pmc_quick.sh gpurun_out/pmc_tile256 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/q7_prof -o run -- python3 tools/group_bench.py 2 2 > gpurun_out/q7.log 2>&1 || exit 1
echo ok
