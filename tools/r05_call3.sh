#!/bin/bash
# Round 5, call 3: four seeds per reference scene at 35k steps, masks kept for the offline statistics.
set -o pipefail
mkdir -p gpurun_out/r05c
for sc in test2 test; do
echo "== probe $sc $(date +%T)"
timeout -k 10 400 python -u tools/density_slices_probe.py --scene $sc --seeds 1337 42 7 2024 --steps 35000 \
  --out gpurun_out/r05c/ds_${sc}.json --masks gpurun_out/r05c/masks_${sc}.npz > gpurun_out/r05c/ds_${sc}.log 2>&1 \
  || { echo "probe rc=$?"; tail -20 gpurun_out/r05c/ds_${sc}.log; exit 1; }
grep -v "^Wrote\|#lattice" gpurun_out/r05c/ds_${sc}.log | cut -c1-250
done
echo "== done $(date +%T)"
echo "== camera / exposure / extra-dims tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s -k "extrinsic or exposure or cam_gradient or extra_dims or deterministic or config_e_trains" \
  --timeout 300 --timeout-method thread > gpurun_out/r05c/cam_tests.log 2>&1 \
  || { echo "tests rc=$?"; grep -E "pose error|PASS|FAIL|Error" gpurun_out/r05c/cam_tests.log | tail -20; exit 1; }
grep -E "pose error|config E|passed|failed" gpurun_out/r05c/cam_tests.log | tail -5
echo "== 8-rank DP tests $(date +%T)"
timeout -k 10 700 python -u -m pytest tests/test_gpu_distributed.py -v -s -k "8-lego" --timeout 600 --timeout-method thread \
  > gpurun_out/r05c/dp8_tests.log 2>&1 || { echo "tests rc=$?"; grep -E "world|passed|failed|Error" gpurun_out/r05c/dp8_tests.log | tail -20; exit 1; }
grep -E "world|batch|passed|failed" gpurun_out/r05c/dp8_tests.log | tail -12
echo "== done $(date +%T)"
