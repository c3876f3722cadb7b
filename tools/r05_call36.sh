#!/bin/bash
# Round 5, call 36: surface-scene candidates (per-pass cap 24, budget headroom 1.25), 6 rounds.
set -o pipefail
mkdir -p gpurun_out/r05ah
timeout -k 10 600 python -u tools/render_ab.py --scene synthetic --host --rounds 6 --frames 5 "" "render_max_steps=24" "render_budget_scale=1.25" \
  "render_max_steps=24 render_budget_scale=1.25" "render_max_steps=16 render_budget_scale=1.25" "render_max_steps=24 render_budget_scale=1.5" \
  > gpurun_out/r05ah/surface.txt 2>&1 || { echo "rc=$?"; tail -20 gpurun_out/r05ah/surface.txt; exit 1; }
grep "ms/frame" gpurun_out/r05ah/surface.txt
echo "== done $(date +%T)"
