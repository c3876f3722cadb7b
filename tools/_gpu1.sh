set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/render_ab.py --rounds 4 --frames 5 "" "render_pass_samples=5242880" "render_pass_samples=6291456" "render_pass_samples=8388608" "render_pass_samples=6291456 render_lanes=6291456" > gpurun_out/render_ab.log 2>&1
