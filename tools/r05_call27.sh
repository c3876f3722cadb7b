#!/bin/bash
# Round 5, call 27: k_generate / k_composite bodies factored into march_ray / composite_ray (no fused kernel) -- render and
# retire tests, then HEAD (ab_old/) vs the working tree on the fire scene, same box.
set -o pipefail
mkdir -p gpurun_out/r05y
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_testbed.py tests/test_gpu_render_modes.py \
  > gpurun_out/r05y/tests.txt 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/r05y/tests.txt; exit 1; }
grep -E "FAILED" gpurun_out/r05y/tests.txt; tail -1 gpurun_out/r05y/tests.txt
for pkg in old new; do
  if [ $pkg = old ]; then P=(--pkg ab_old); else P=(); fi
  timeout -k 10 400 python -u tools/render_ab.py "${P[@]}" --host --rounds 4 --frames 5 "" > gpurun_out/r05y/ab_$pkg.txt 2>&1 \
    || { echo "ab rc=$?"; tail -20 gpurun_out/r05y/ab_$pkg.txt; exit 1; }
  echo "== $pkg"; tail -1 gpurun_out/r05y/ab_$pkg.txt
done
echo "== done $(date +%T)"
