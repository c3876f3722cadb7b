set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 1000 bash tools/profile_round.sh r03i > gpurun_out/profile_round.log 2>&1 && \
timeout -k 10 600 bash tools/pmc_mfma.sh r03i > gpurun_out/pmc_mfma.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1
