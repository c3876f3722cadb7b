#!/bin/bash
# GPU box: the tests fixed after r04b, then the measurement session.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_testbed.py -m gpu -v -s \
  -k "world_times or extrinsic" --timeout 200 --timeout-method thread > gpurun_out/r04c_tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed|window loss|pose error" gpurun_out/r04c_tests.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "tests rc=$rc"; exit $rc; }
tools/r04_measure.sh r04
