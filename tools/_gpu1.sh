set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_distributed.py -x -v --timeout 300 --timeout-method thread > gpurun_out/scan_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/train_kernels_ab.py --steps 300 --timed 50 --rounds 3 > gpurun_out/train_ab.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1
