#!/bin/bash
# Round 5, call 40: confirmation of read-back lag 2 (and with the exit cap off), 6 rounds, both scenes.
set -o pipefail
mkdir -p gpurun_out/r05ak
timeout -k 10 600 python -u tools/render_ab.py --host --rounds 6 --frames 5 "" "render_lag=2" "render_lag=2 render_exit_cap=2" "render_exit_cap=2" \
  > gpurun_out/r05ak/fire.txt 2>&1 || { echo "rc=$?"; tail -20 gpurun_out/r05ak/fire.txt; exit 1; }
grep "ms/frame" gpurun_out/r05ak/fire.txt
timeout -k 10 600 python -u tools/render_ab.py --scene synthetic --host --rounds 6 --frames 5 "" "render_lag=2" "render_lag=2 render_exit_cap=2" \
  > gpurun_out/r05ak/surface.txt 2>&1 || { echo "rc=$?"; tail -20 gpurun_out/r05ak/surface.txt; exit 1; }
grep "ms/frame" gpurun_out/r05ak/surface.txt
echo "== done $(date +%T)"
