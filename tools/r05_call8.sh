#!/bin/bash
# Round 5, call 8: wave-priority A/B of the render kernels (fire scene, then the surface scene).
set -o pipefail
mkdir -p gpurun_out/r05g
echo "== fire $(date +%T)"
timeout -k 10 400 python -u tools/render_ab.py --rounds 4 --frames 5 "" "render_priority=16" "render_priority=48" "render_priority=12" \
  "render_priority=3" "render_priority=28" "render_priority=60" > gpurun_out/r05g/fire.txt 2> gpurun_out/r05g/fire.err \
  || { echo "ab rc=$?"; tail -20 gpurun_out/r05g/fire.err; exit 1; }
cat gpurun_out/r05g/fire.txt
echo "== surface $(date +%T)"
timeout -k 10 400 python -u tools/render_ab.py --scene synthetic --rounds 4 --frames 10 "" "render_priority=16" "render_priority=48" \
  "render_priority=12" "render_priority=3" > gpurun_out/r05g/surface.txt 2> gpurun_out/r05g/surface.err \
  || { echo "ab rc=$?"; tail -20 gpurun_out/r05g/surface.err; exit 1; }
cat gpurun_out/r05g/surface.txt
echo "== done $(date +%T)"
