set -o pipefail
bash tools/gpu_session.sh r01s4 && bash tools/pmc_passes.sh gpurun_out/pmc_r01s4
