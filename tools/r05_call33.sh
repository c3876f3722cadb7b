#!/bin/bash
# Round 5, call 33: confirmation of the sweep's candidates (pass budget per scene kind, MLP workgroups per CU), 6 rounds.
set -o pipefail
mkdir -p gpurun_out/r05ae
timeout -k 10 600 python -u tools/render_ab.py --host --rounds 6 --frames 5 "" "render_pass_samples=6291456" "render_pass_samples=7340032" \
  "mlp_workgroups_per_cu=6" "render_pass_samples=6291456 mlp_workgroups_per_cu=6" > gpurun_out/r05ae/fire.txt 2>&1 \
  || { echo "rc=$?"; tail -20 gpurun_out/r05ae/fire.txt; exit 1; }
grep "ms/frame" gpurun_out/r05ae/fire.txt
timeout -k 10 600 python -u tools/render_ab.py --scene synthetic --host --rounds 6 --frames 5 "" "render_pass_samples=4194304" \
  "render_pass_samples=3145728" > gpurun_out/r05ae/surface.txt 2>&1 || { echo "rc=$?"; tail -20 gpurun_out/r05ae/surface.txt; exit 1; }
grep "ms/frame" gpurun_out/r05ae/surface.txt
echo "== done $(date +%T)"
