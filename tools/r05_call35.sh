#!/bin/bash
# Round 5, call 35: second sweep on the new defaults (march budget headroom, lane budget, first-pass cap, block shapes).
set -o pipefail
mkdir -p gpurun_out/r05ag
S=("" "render_first_steps=16" "render_budget_scale=1.25" "render_budget_scale=0.8" "render_generate_block=256" \
   "render_lanes=3145728" "render_lanes=6291456" "render_max_steps=40" "render_pass_samples=7340032" "mlp_workgroups_per_cu=5")
timeout -k 10 600 python -u tools/render_ab.py --host --rounds 4 --frames 5 "${S[@]}" > gpurun_out/r05ag/fire.txt 2>&1 \
  || { echo "rc=$?"; tail -20 gpurun_out/r05ag/fire.txt; exit 1; }
grep "ms/frame" gpurun_out/r05ag/fire.txt
S2=("" "render_budget_scale=1.25" "render_budget_scale=0.8" "render_lanes=3145728" "render_lanes=6291456" "render_mlp_tile=4" \
    "mlp_workgroups_per_cu=6" "mlp_workgroups_per_cu=10" "render_generate_block=256" "render_max_steps=24")
timeout -k 10 600 python -u tools/render_ab.py --scene synthetic --host --rounds 4 --frames 5 "${S2[@]}" > gpurun_out/r05ag/surface.txt 2>&1 \
  || { echo "rc=$?"; tail -20 gpurun_out/r05ag/surface.txt; exit 1; }
grep "ms/frame" gpurun_out/r05ag/surface.txt
echo "== done $(date +%T)"
