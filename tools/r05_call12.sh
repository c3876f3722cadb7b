#!/bin/bash
# Round 5, call 12: sampler resume point + k_train_chunk lanes per ray -- pipeline parity tests, per-kernel
# training A/B (surface and fire scenes), one surface step's kernel timeline.
set -o pipefail
mkdir -p gpurun_out/r05k
REPO=$PWD
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_pipeline.py \
  > gpurun_out/r05k/pipeline_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r05k/pipeline_tests.txt; exit 1; }
tail -3 gpurun_out/r05k/pipeline_tests.txt
timeout -k 10 400 python -u tools/train_kernels_ab.py --scene synthetic --steps 400 --timed 100 --rounds 3 \
  --settings "" "train_chunk_lanes=8" "train_chunk_lanes=16" "train_chunk_lanes=32" > gpurun_out/r05k/chunk_ab_surface.txt 2>&1 \
  || { echo "ab rc=$?"; tail -20 gpurun_out/r05k/chunk_ab_surface.txt; exit 1; }
grep -E "^##|step_wall|train_chunk|sampler|TRAIN" gpurun_out/r05k/chunk_ab_surface.txt
timeout -k 10 300 python -u tools/train_kernels_ab.py --steps 400 --timed 100 --rounds 3 \
  --settings "" "train_chunk_lanes=32" "train_chunk_lanes=16" > gpurun_out/r05k/chunk_ab_fire.txt 2>&1 \
  || { echo "ab rc=$?"; tail -20 gpurun_out/r05k/chunk_ab_fire.txt; exit 1; }
grep -E "^##|step_wall" gpurun_out/r05k/chunk_ab_fire.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$REPO/gpurun_out/r05k/kt" -o run -- python3 "$REPO/bench.py" --scene synthetic \
  --pretrain 300 --deterministic-pretrain 0 --steps 6 --warmup 3 --cpu-baseline 0 --surface-scene 0 --config-e 0 --render-in-hbm 0 \
  > "$REPO/gpurun_out/r05k/timeline.log" 2>&1 || { echo "rc=$?"; tail -5 "$REPO/gpurun_out/r05k/timeline.log"; exit 1; }
F=$(find "$REPO/gpurun_out/r05k/kt" -name '*kernel_trace.csv' | head -n 1)
python3 "$REPO/tools/step_timeline.py" "$F" "$REPO/gpurun_out/r05k/timeline_synthetic.txt" > /dev/null
find "$REPO/gpurun_out/r05k/kt" -name '*.csv' -delete
sed -n 1,30p "$REPO/gpurun_out/r05k/timeline_synthetic.txt"
echo "== done $(date +%T)"
