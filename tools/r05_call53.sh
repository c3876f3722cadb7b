#!/bin/bash
# Round 5, call 53: the fine levels' optimizer overlapped with the coarse levels' hash-grid backward (ngp_tuning.train_overlap
# 0) vs in sequence (1): training tests incl. the bit-identity test, then step wall time round-robin on one model.
set -o pipefail
mkdir -p gpurun_out/r05aw
echo "== tests $(date +%T)"
timeout -k 10 700 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_pipeline.py tests/test_gpu_testbed.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r05aw/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05aw/tests.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" gpurun_out/r05aw/tests.log | head; exit $rc; }
for scene in synthetic data/nerf/test/dataset/transforms_all.json; do
  echo "== $scene $(date +%T)"
  timeout -k 10 300 python -u tools/train_kernels_ab.py --scene $scene --steps 300 --timed 100 --rounds 5 \
    --settings "" "train_overlap=1" > gpurun_out/r05aw/ab_$(basename $scene).log 2>&1 \
    || { echo "ab rc=$?"; tail -5 gpurun_out/r05aw/ab_$(basename $scene).log; exit 1; }
  grep -E "^##|step_wall" gpurun_out/r05aw/ab_$(basename $scene).log
done
echo "== done $(date +%T)"
