#!/bin/bash
# Round 5, call 39: third sweep on the re-swept defaults (encoder variants, pipelines, exit cap, unfilled-tile skip, MLP tile).
set -o pipefail
mkdir -p gpurun_out/r05aj
S=("" "encode_xcd_regions=1" "encode_streaming=1" "render_skip_unfilled=2" "render_exit_cap=2" "render_pipelines=3" \
   "encode_dense_records=1" "mlp_workgroups_per_cu=5" "render_composite_block=256" "render_mlp_tile=2" "render_lag=2")
timeout -k 10 600 python -u tools/render_ab.py --host --rounds 4 --frames 5 "${S[@]}" > gpurun_out/r05aj/fire.txt 2>&1 \
  || { echo "rc=$?"; tail -20 gpurun_out/r05aj/fire.txt; exit 1; }
grep "ms/frame" gpurun_out/r05aj/fire.txt
S2=("" "encode_xcd_regions=1" "encode_streaming=1" "render_skip_unfilled=2" "render_exit_cap=2" "render_pipelines=2" \
    "encode_dense_records=1" "render_composite_block=256" "render_lag=2" "render_first_steps=3")
timeout -k 10 600 python -u tools/render_ab.py --scene synthetic --host --rounds 4 --frames 5 "${S2[@]}" > gpurun_out/r05aj/surface.txt 2>&1 \
  || { echo "rc=$?"; tail -20 gpurun_out/r05aj/surface.txt; exit 1; }
grep "ms/frame" gpurun_out/r05aj/surface.txt
echo "== done $(date +%T)"
