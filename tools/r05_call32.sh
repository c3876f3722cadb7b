#!/bin/bash
# Round 5, call 32: schedule / launch-shape sweep on the closing kernels (fire and surface scenes, render() to host memory).
set -o pipefail
mkdir -p gpurun_out/r05ad
S=("" "render_pass_samples=4194304" "render_pass_samples=6291456" "render_pass_samples=8388608" "render_lanes=2097152" \
   "render_lanes=8388608" "render_max_steps=48" "render_max_steps=24" "mlp_workgroups_per_cu=6" "render_composite_block=1024" \
   "render_lag=4" "render_first_steps=4")
timeout -k 10 600 python -u tools/render_ab.py --host --rounds 4 --frames 5 "${S[@]}" > gpurun_out/r05ad/fire.txt 2>&1 \
  || { echo "rc=$?"; tail -20 gpurun_out/r05ad/fire.txt; exit 1; }
grep "ms/frame" gpurun_out/r05ad/fire.txt
S2=("" "render_pass_samples=4194304" "render_pass_samples=8388608" "render_lanes=2097152" "render_lanes=8388608" \
    "render_max_steps=16" "render_first_steps=2" "render_first_steps=8" "render_composite_block=1024" "mlp_workgroups_per_cu=6")
timeout -k 10 600 python -u tools/render_ab.py --scene synthetic --host --rounds 4 --frames 5 "${S2[@]}" > gpurun_out/r05ad/surface.txt 2>&1 \
  || { echo "rc=$?"; tail -20 gpurun_out/r05ad/surface.txt; exit 1; }
grep "ms/frame" gpurun_out/r05ad/surface.txt
echo "== done $(date +%T)"
