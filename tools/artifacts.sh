set -o pipefail
# PMC passes first (they feed profiles/pmc_traffic.json), then the session
bash tools/pmc_passes.sh gpurun_out/pmc_art || exit 1
bash tools/gpu_session.sh art || exit 1
