set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 && \
timeout -k 10 600 python -u tools/render_ab.py --scene synthetic --rounds 4 --frames 10 "" "render_pass_samples=4194304" "render_pass_samples=6291456" > gpurun_out/render_ab_surface.log 2>&1
