#!/bin/bash
# Round 5, call 34: the new schedule defaults (6 M / 3 M pass budgets, 6 render-MLP workgroups per CU) against the old ones.
set -o pipefail
mkdir -p gpurun_out/r05af
timeout -k 10 600 python -u tools/render_ab.py --host --rounds 6 --frames 5 "" "render_pass_samples=5242880 mlp_workgroups_per_cu=8" \
  > gpurun_out/r05af/fire.txt 2>&1 || { echo "rc=$?"; tail -20 gpurun_out/r05af/fire.txt; exit 1; }
grep "ms/frame" gpurun_out/r05af/fire.txt
timeout -k 10 600 python -u tools/render_ab.py --scene synthetic --host --rounds 6 --frames 5 "" "render_pass_samples=5242880 mlp_workgroups_per_cu=8" \
  "render_pass_samples=2097152" > gpurun_out/r05af/surface.txt 2>&1 || { echo "rc=$?"; tail -20 gpurun_out/r05af/surface.txt; exit 1; }
grep "ms/frame" gpurun_out/r05af/surface.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_testbed.py -k "1080p or streams or retires" \
  > gpurun_out/r05af/tests.txt 2>&1 || { echo "tests rc=$?"; tail -20 gpurun_out/r05af/tests.txt; exit 1; }
tail -1 gpurun_out/r05af/tests.txt
echo "== done $(date +%T)"
