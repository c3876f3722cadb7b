#!/bin/bash
# Kernel trace of render_ab.py frames -> tools/render_timeline.py overlap summary (diagnostic).
# Usage (GPU box, repo root): tools/render_trace.sh <label> "<setting>"
LABEL=$1; SETTING=$2
OUT=$PWD/gpurun_out/$LABEL
mkdir -p "$OUT"
REPO=$PWD
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt" -o run -- \
  python3 "$REPO/tools/render_ab.py" --rounds 1 --frames 4 "$SETTING") > "$OUT/run.log" 2>&1 || { tail -n 20 "$OUT/run.log"; exit 1; }
F=$(find "$OUT/kt" -name '*kernel_trace.csv' | head -n 1)
python3 tools/render_timeline.py "$F" 3 "$OUT/timeline.txt" || exit 1
find "$OUT/kt" -name '*.csv' -delete
