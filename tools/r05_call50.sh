#!/bin/bash
# Round 5, call 50: the step counters zeroed by k_sample_count instead of a memset dispatch:
# training tests, then per-step wall time of this build vs the previous one (ab_old/), alternating.
set -o pipefail
mkdir -p gpurun_out/r05at
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_testbed.py tests/test_gpu_distributed.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r05at/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05at/tests.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" gpurun_out/r05at/tests.log | head; exit $rc; }
for scene in synthetic data/nerf/test/dataset/transforms_all.json; do
  k=0
  for b in new old new old; do
    k=$((k+1))
    echo "== $scene $b $(date +%T)"
    pkg=""; [ $b = old ] && pkg="--pkg ab_old"
    timeout -k 10 240 python -u tools/train_kernels_ab.py $pkg --scene $scene --steps 300 --timed 100 --rounds 3 \
      > gpurun_out/r05at/ab_$(basename $scene)_${b}$k.log 2>&1 || { echo "ab rc=$?"; tail -5 gpurun_out/r05at/ab_$(basename $scene)_${b}$k.log; exit 1; }
    grep -E "step_wall" gpurun_out/r05at/ab_$(basename $scene)_${b}$k.log
  done
done
echo "== done $(date +%T)"
