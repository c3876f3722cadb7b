#!/bin/bash
# Round 5, call 24: fused composite + march (ngp_tuning.render_fused_march) -- frame identity tests, render A/B on the fire and
# surface scenes.
set -o pipefail
mkdir -p gpurun_out/r05v
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_testbed.py -k "fused or 1080p or streams" \
  > gpurun_out/r05v/tests.txt 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/r05v/tests.txt; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/r05v/tests.txt; tail -1 gpurun_out/r05v/tests.txt
timeout -k 10 500 python -u tools/render_ab.py --host --rounds 5 --frames 5 "" "render_fused_march=1" \
  > gpurun_out/r05v/fire_ab.txt 2>&1 || { echo "ab rc=$?"; tail -20 gpurun_out/r05v/fire_ab.txt; exit 1; }
tail -3 gpurun_out/r05v/fire_ab.txt
timeout -k 10 500 python -u tools/render_ab.py --scene synthetic --host --rounds 5 --frames 5 "" "render_fused_march=1" \
  > gpurun_out/r05v/surface_ab.txt 2>&1 || { echo "ab rc=$?"; tail -20 gpurun_out/r05v/surface_ab.txt; exit 1; }
tail -3 gpurun_out/r05v/surface_ab.txt
echo "== done $(date +%T)"
