#!/bin/bash
# Kernel trace of a short bench run; prints one train+render step's timeline (tools/step_timeline.py).
# Usage (GPU box, repo root): tools/trace_step.sh [label]
L=${1:-step}
EXTRA=${2:-}
OUT=$PWD/gpurun_out/trace_$L
mkdir -p "$OUT"
REPO=$PWD
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt" -o run -- \
  python3 "$REPO/bench.py" --steps 4 --warmup 2 --cpu-baseline 0 $EXTRA > "$OUT/bench.log" 2>&1 || exit $?
cd "$REPO"
F=$(find "$OUT/kt" -name '*kernel_trace.csv' | head -n 1)
python3 tools/step_timeline.py "$F" "$OUT/timeline.txt" > /dev/null || exit $?
find "$OUT" -name '*.csv' -delete
tail -n 45 "$OUT/timeline.txt"
