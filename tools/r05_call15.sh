#!/bin/bash
# Round 5, call 15: training batch samples per ray vs chunk schedules (surface and fire scenes).
set -o pipefail
mkdir -p gpurun_out/r05n
for sc in synthetic fire; do
  timeout -k 10 300 python -u tools/probe_train_chunks.py $sc 1500 > gpurun_out/r05n/chunks_$sc.txt 2>&1 \
    || { echo "probe rc=$?"; tail -20 gpurun_out/r05n/chunks_$sc.txt; exit 1; }
  echo "== $sc"; grep -E "^\[train\]|^stats" gpurun_out/r05n/chunks_$sc.txt
done
