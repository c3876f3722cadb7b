set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 bash tools/profile_round.sh r03k > gpurun_out/profile_round.log 2>&1 && \
timeout -k 10 600 bash tools/pmc_mfma.sh r03k > gpurun_out/pmc_mfma.log 2>&1
