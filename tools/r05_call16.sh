#!/bin/bash
# Round 5, call 16: the sampler without its duplicated 16-B position rows -- pipeline tests, training step of HEAD
# (ab_old/) vs the working tree; surface-scene render() with one vs two ray pipelines.
set -o pipefail
mkdir -p gpurun_out/r05o
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_pipeline.py \
  > gpurun_out/r05o/pipeline_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r05o/pipeline_tests.txt; exit 1; }
tail -1 gpurun_out/r05o/pipeline_tests.txt
for sc in synthetic fire; do
  if [ $sc = fire ]; then SC=(); else SC=(--scene synthetic); fi
  timeout -k 10 300 python -u tools/train_kernels_ab.py --pkg ab_old "${SC[@]}" --steps 400 --timed 100 --rounds 3 --settings "" \
    > gpurun_out/r05o/ab_old_$sc.txt 2>&1 || { echo "ab rc=$?"; tail -20 gpurun_out/r05o/ab_old_$sc.txt; exit 1; }
  timeout -k 10 300 python -u tools/train_kernels_ab.py "${SC[@]}" --steps 400 --timed 100 --rounds 3 --settings "" \
    > gpurun_out/r05o/ab_new_$sc.txt 2>&1 || { echo "ab rc=$?"; tail -20 gpurun_out/r05o/ab_new_$sc.txt; exit 1; }
  echo "== $sc old"; grep -E "step_wall|train_sampler" gpurun_out/r05o/ab_old_$sc.txt
  echo "== $sc new"; grep -E "step_wall|train_sampler" gpurun_out/r05o/ab_new_$sc.txt
done
timeout -k 10 400 python -u tools/render_ab.py --scene synthetic --host --rounds 4 --frames 5 "" "render_pipelines=2" \
  > gpurun_out/r05o/surface_pipes.txt 2>&1 || { echo "render ab rc=$?"; tail -20 gpurun_out/r05o/surface_pipes.txt; exit 1; }
tail -6 gpurun_out/r05o/surface_pipes.txt
echo "== done $(date +%T)"
