#!/bin/bash
# Round 5, call 26: fused march at 8 waves per SIMD (64 VGPRs, small spill) -- fire / surface render A/B.
set -o pipefail
mkdir -p gpurun_out/r05x
timeout -k 10 500 python -u tools/render_ab.py --host --rounds 4 --frames 5 "" "render_fused_march=1" \
  > gpurun_out/r05x/fire_ab.txt 2>&1 || { echo "ab rc=$?"; tail -20 gpurun_out/r05x/fire_ab.txt; exit 1; }
tail -2 gpurun_out/r05x/fire_ab.txt
timeout -k 10 500 python -u tools/render_ab.py --scene synthetic --host --rounds 4 --frames 5 "" "render_fused_march=1" \
  > gpurun_out/r05x/surface_ab.txt 2>&1 || { echo "ab rc=$?"; tail -20 gpurun_out/r05x/surface_ab.txt; exit 1; }
tail -2 gpurun_out/r05x/surface_ab.txt
echo "== done $(date +%T)"
