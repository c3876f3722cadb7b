#!/bin/bash
# Round 5, call 54: hash-grid backward workgroups per level (ngp_tuning.train_bwd_chunks; 0 = one per 128-sample chunk,
# 2048 per level at 2^18 samples): the train_encode_bwd timer and the step wall time, round-robin on one model.
set -o pipefail
mkdir -p gpurun_out/r05ax
for scene in synthetic data/nerf/test/dataset/transforms_all.json; do
  echo "== $scene $(date +%T)"
  timeout -k 10 300 python -u tools/train_kernels_ab.py --scene $scene --steps 300 --timed 100 --rounds 3 \
    --settings "" "train_bwd_chunks=1024" "train_bwd_chunks=512" "train_bwd_chunks=256" "train_bwd_chunks=128" \
    > gpurun_out/r05ax/ab_$(basename $scene).log 2>&1 || { echo "ab rc=$?"; tail -5 gpurun_out/r05ax/ab_$(basename $scene).log; exit 1; }
  grep -E "^##|step_wall|train_encode_bwd" gpurun_out/r05ax/ab_$(basename $scene).log
done
echo "== done $(date +%T)"
