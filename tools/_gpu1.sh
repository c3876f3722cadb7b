set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 && \
timeout -k 10 300 python -u tools/train_kernels_ab.py --steps 300 --timed 50 --rounds 3 --settings "" "mlp_train_schedule=2" > gpurun_out/train_ab.log 2>&1 && \
timeout -k 10 1000 bash tools/profile_round.sh r03h > gpurun_out/profile_round.log 2>&1 && \
timeout -k 10 600 bash tools/pmc_mfma.sh r03h > gpurun_out/pmc_mfma.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1
