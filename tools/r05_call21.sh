#!/bin/bash
# Round 5, call 21: idle gaps between a frame's kernels with the kernel timers off / on (surface scene, one pipeline).
set -o pipefail
mkdir -p gpurun_out/r05s
REPO=$PWD
cd /tmp && export TMPDIR=/tmp
for t in 0 -1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$REPO/gpurun_out/r05s/kt_$t" -o run -- python3 "$REPO/tools/probe_gaps.py" --timers $t \
    > "$REPO/gpurun_out/r05s/probe_$t.log" 2>&1 || { echo "rc=$?"; tail -5 "$REPO/gpurun_out/r05s/probe_$t.log"; exit 1; }
  F=$(find "$REPO/gpurun_out/r05s/kt_$t" -name '*kernel_trace.csv' | head -n 1)
  echo "== timers $t"; grep "ms per frame" "$REPO/gpurun_out/r05s/probe_$t.log"
  python3 "$REPO/tools/gap_summary.py" "$F" 2 | tee "$REPO/gpurun_out/r05s/gaps_$t.txt" | head -12
  find "$REPO/gpurun_out/r05s/kt_$t" -name '*.csv' -delete
done
echo "== done $(date +%T)"
