#!/bin/bash
# Round 5, call 25: why the fused march is slower -- march statistics per setting and a kernel trace of fused frames.
set -o pipefail
mkdir -p gpurun_out/r05w
REPO=$PWD
timeout -k 10 300 python -u tools/render_ab.py --stats --rounds 1 --frames 2 "" "render_fused_march=1" > gpurun_out/r05w/stats.txt 2>&1 \
  || { echo "rc=$?"; tail -20 gpurun_out/r05w/stats.txt; exit 1; }
grep -E "stats|\[render\]|ms/frame" gpurun_out/r05w/stats.txt | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/gpurun_out/r05w/kt" -o run -- python3 "$REPO/tools/render_ab.py" --rounds 1 --frames 3 "render_fused_march=1" \
  > "$REPO/gpurun_out/r05w/kt.log" 2>&1 || { echo "rc=$?"; tail -5 "$REPO/gpurun_out/r05w/kt.log"; exit 1; }
F=$(find "$REPO/gpurun_out/r05w/kt" -name '*kernel_stats.csv' | head -n 1)
python3 - "$F" <<'PY'
import csv, sys
for r in sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{r["Name"].split("(")[0][:70]:70s} {int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:9.1f} us')
PY
find "$REPO/gpurun_out/r05w/kt" -name '*trace.csv' -delete
echo "== done $(date +%T)"
