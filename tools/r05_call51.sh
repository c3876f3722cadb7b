#!/bin/bash
# Round 5, call 51: bucketed cell sort for the density-grid update (ngp_tuning.grid_unsorted 0) vs the full radix sort (2)
# and drawing order (1): the pipeline tests, then the grid_update timer and step wall time, round-robin on one model.
set -o pipefail
mkdir -p gpurun_out/r05au
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r05au/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05au/tests.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" gpurun_out/r05au/tests.log | head; exit $rc; }
for scene in synthetic data/nerf/test/dataset/transforms_all.json; do
  echo "== $scene $(date +%T)"
  timeout -k 10 300 python -u tools/train_kernels_ab.py --scene $scene --steps 300 --timed 160 --rounds 3 \
    --settings "" "grid_unsorted=2" "grid_unsorted=1" > gpurun_out/r05au/ab_$(basename $scene).log 2>&1 \
    || { echo "ab rc=$?"; tail -5 gpurun_out/r05au/ab_$(basename $scene).log; exit 1; }
  grep -E "^##|step_wall|grid_update" gpurun_out/r05au/ab_$(basename $scene).log
done
echo "== done $(date +%T)"
