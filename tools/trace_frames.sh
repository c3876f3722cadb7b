#!/bin/bash
# Kernel trace of rendered frames (tools/render_ab.py, one setting) -> per-launch listing of one
# frame (tools/frame_passes.py) and the overlap summary (tools/render_timeline.py).
# Usage (GPU box, repo root): tools/trace_frames.sh <label> [render_ab setting]
L=${1:-trace}; SET=${2:-}
OUT=$PWD/gpurun_out/trace_$L
mkdir -p "$OUT"
REPO=$PWD
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt" -o run -- \
  python3 "$REPO/tools/render_ab.py" --rounds 1 --frames 3 "$SET" > "$OUT/run.log" 2>&1 || exit $?
cd "$REPO"
F=$(find "$OUT/kt" -name '*kernel_trace.csv' | head -n 1)
python3 tools/frame_passes.py "$F" "$OUT/frame.txt" > /dev/null || exit $?
python3 tools/render_timeline.py "$F" 2 "$OUT/overlap.txt" > /dev/null || exit $?
find "$OUT" -name '*.csv' -delete
head -n 3 "$OUT/frame.txt"; cat "$OUT/overlap.txt" | head -40
