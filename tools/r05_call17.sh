#!/bin/bash
# Round 5, call 17: the training sampler with G lanes per ray -- oracle parity per lane count, then the training
# step per lane count on the surface and fire scenes.
set -o pipefail
mkdir -p gpurun_out/r05p
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_pipeline.py \
  -k "sampler or train_step_matches_oracle or chunked" > gpurun_out/r05p/tests.txt 2>&1 \
  || { echo "tests rc=$?"; tail -30 gpurun_out/r05p/tests.txt; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/r05p/tests.txt | tail -20; tail -1 gpurun_out/r05p/tests.txt
for sc in synthetic fire; do
  if [ $sc = fire ]; then SC=(); else SC=(--scene synthetic); fi
  timeout -k 10 400 python -u tools/train_kernels_ab.py "${SC[@]}" --steps 400 --timed 100 --rounds 3 --settings "" \
    "train_sampler_lanes=32" "train_sampler_lanes=16" "train_sampler_lanes=8" > gpurun_out/r05p/ab_$sc.txt 2>&1 \
    || { echo "ab rc=$?"; tail -20 gpurun_out/r05p/ab_$sc.txt; exit 1; }
  echo "== $sc"; grep -E "^##|step_wall|train_sampler" gpurun_out/r05p/ab_$sc.txt
done
echo "== done $(date +%T)"
