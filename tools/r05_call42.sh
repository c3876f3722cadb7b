#!/bin/bash
# Round 5, call 42: fourth sweep on the lag-2 defaults (pass budgets, MLP workgroups, budget headroom, lanes, caps).
set -o pipefail
mkdir -p gpurun_out/r05am
S=("" "render_pass_samples=5242880" "render_pass_samples=7340032" "render_pass_samples=8388608" "mlp_workgroups_per_cu=5" "mlp_workgroups_per_cu=7" \
   "render_budget_scale=0.8" "render_lanes=5242880" "render_max_steps=40" "render_first_steps=6")
timeout -k 10 600 python -u tools/render_ab.py --host --rounds 4 --frames 5 "${S[@]}" > gpurun_out/r05am/fire.txt 2>&1 \
  || { echo "rc=$?"; tail -20 gpurun_out/r05am/fire.txt; exit 1; }
grep "ms/frame" gpurun_out/r05am/fire.txt
S2=("" "render_pass_samples=2097152" "render_pass_samples=4194304" "render_max_steps=20" "render_max_steps=28" "render_budget_scale=1.25" \
    "render_lanes=3145728" "render_first_steps=3" "render_first_steps=6" "mlp_workgroups_per_cu=6")
timeout -k 10 600 python -u tools/render_ab.py --scene synthetic --host --rounds 4 --frames 5 "${S2[@]}" > gpurun_out/r05am/surface.txt 2>&1 \
  || { echo "rc=$?"; tail -20 gpurun_out/r05am/surface.txt; exit 1; }
grep "ms/frame" gpurun_out/r05am/surface.txt
echo "== done $(date +%T)"
