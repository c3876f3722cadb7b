set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_testbed.py tests/test_gpu_render_modes.py -x -v --timeout 300 --timeout-method thread -k "render or 1080p or normal" > gpurun_out/tail_tests.log 2>&1 && \
timeout -k 10 500 python -u tools/render_ab.py --rounds 4 --frames 5 "" "render_tail_rays=1" "render_tail_rays=262144" > gpurun_out/render_ab.log 2>&1
