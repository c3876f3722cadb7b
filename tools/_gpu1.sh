set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_testbed.py -x -v --timeout 300 --timeout-method thread -k "render or 1080p" > gpurun_out/compact_tests.log 2>&1 && \
timeout -k 10 400 python -u tools/render_ab.py --rounds 4 --frames 5 "" "render_slot_compaction=2" > gpurun_out/render_ab.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1
