#!/bin/bash
# Round 5, call 18: ray pipelines started out of phase (ngp_tuning.render_stagger) -- fire-scene render() A/B, then
# one kernel trace of the best setting's frame.
set -o pipefail
mkdir -p gpurun_out/r05q
timeout -k 10 500 python -u tools/render_ab.py --host --rounds 5 --frames 5 "" "render_stagger=1" "render_stagger=2" \
  "render_stagger=3" > gpurun_out/r05q/stagger_ab.txt 2>&1 || { echo "ab rc=$?"; tail -20 gpurun_out/r05q/stagger_ab.txt; exit 1; }
tail -5 gpurun_out/r05q/stagger_ab.txt
echo "== done $(date +%T)"
