#!/bin/bash
# Round 5, call 11: one training step's kernel timeline (surface and fire scenes).
set -o pipefail
mkdir -p gpurun_out/r05j
REPO=$PWD
cd /tmp && export TMPDIR=/tmp
for sc in synthetic fire; do
  if [ $sc = fire ]; then SC=(); else SC=(--scene synthetic); fi
  echo "== $sc $(date +%T)"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$REPO/gpurun_out/r05j/kt_$sc" -o run -- python3 "$REPO/bench.py" "${SC[@]}" \
    --pretrain 300 --deterministic-pretrain 0 --steps 6 --warmup 3 --cpu-baseline 0 --surface-scene 0 --config-e 0 --render-in-hbm 0 \
    > "$REPO/gpurun_out/r05j/$sc.log" 2>&1 || { echo "rc=$?"; tail -5 "$REPO/gpurun_out/r05j/$sc.log"; exit 1; }
  F=$(find "$REPO/gpurun_out/r05j/kt_$sc" -name '*kernel_trace.csv' | head -n 1)
  python3 "$REPO/tools/step_timeline.py" "$F" "$REPO/gpurun_out/r05j/timeline_$sc.txt" > /dev/null
  find "$REPO/gpurun_out/r05j/kt_$sc" -name '*.csv' -delete
  grep -E "^step|per kernel" -A40 "$REPO/gpurun_out/r05j/timeline_$sc.txt" | head -45
done
echo "== done $(date +%T)"
