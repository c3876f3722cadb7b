#!/bin/bash
# Round 5, call 13: training-step launch fusions (sampler clamp into k_sample_write; clamp + gather + rollover +
# loss sum in one launch; Adam bias-correction table filled ahead) and 16 chunk lanes -- parity tests, then the
# training step of HEAD (ab_old/) vs the working tree on the surface and fire scenes.
set -o pipefail
mkdir -p gpurun_out/r05l
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pipeline.py \
  tests/test_gpu_kernels.py tests/test_gpu_distributed.py > gpurun_out/r05l/tests.txt 2>&1 \
  || { echo "tests rc=$?"; tail -30 gpurun_out/r05l/tests.txt; exit 1; }
tail -3 gpurun_out/r05l/tests.txt
for sc in synthetic fire; do
  if [ $sc = fire ]; then SC=(); else SC=(--scene synthetic); fi
  timeout -k 10 300 python -u tools/train_kernels_ab.py --pkg ab_old "${SC[@]}" --steps 400 --timed 100 --rounds 3 --settings "" \
    > gpurun_out/r05l/ab_old_$sc.txt 2>&1 || { echo "ab rc=$?"; tail -20 gpurun_out/r05l/ab_old_$sc.txt; exit 1; }
  timeout -k 10 300 python -u tools/train_kernels_ab.py "${SC[@]}" --steps 400 --timed 100 --rounds 3 --settings "" "train_chunk_lanes=4" \
    > gpurun_out/r05l/ab_new_$sc.txt 2>&1 || { echo "ab rc=$?"; tail -20 gpurun_out/r05l/ab_new_$sc.txt; exit 1; }
  echo "== $sc old"; grep -E "^##|step_wall|train_" gpurun_out/r05l/ab_old_$sc.txt
  echo "== $sc new"; grep -E "^##|step_wall|train_" gpurun_out/r05l/ab_new_$sc.txt
done
echo "== done $(date +%T)"
