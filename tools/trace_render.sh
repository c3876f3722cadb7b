#!/bin/bash
# Kernel trace of a few rendered frames after a short training run; prints one frame's timeline.
OUT=$PWD/gpurun_out/trace_render
mkdir -p "$OUT"
REPO=$PWD
export TMPDIR=/tmp
cd /tmp
CAPS=32 TIMER_MASK=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt" -o run -- \
  python3 "$REPO/tools/probe_render.py" 1500 > "$OUT/probe.log" 2>&1 || exit $?
cd "$REPO"
F=$(find "$OUT/kt" -name '*kernel_trace.csv' | head -n 1)
python3 tools/frame_timeline.py "$F" "$OUT/timeline.txt" > /dev/null || exit $?
find "$OUT" -name '*.csv' -delete
tail -n 5 "$OUT/timeline.txt"
