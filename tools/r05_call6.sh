#!/bin/bash
# Round 5, call 6: where config E's frame goes (probe + kernel-trace stats).
set -o pipefail
mkdir -p gpurun_out/r05e
echo "== probe $(date +%T)"
timeout -k 10 300 python -u tools/probe_config_e.py 500 > gpurun_out/r05e/probe.log 2>&1 || { echo "probe rc=$?"; tail -20 gpurun_out/r05e/probe.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05e/probe.log
echo "== kernel trace $(date +%T)"
REPO=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/gpurun_out/r05e/kt" -o run -- python3 "$REPO/tools/probe_config_e.py" 300 \
  > "$REPO/gpurun_out/r05e/kt.log" 2>&1 || { echo "kt rc=$?"; tail -20 "$REPO/gpurun_out/r05e/kt.log"; exit 1; }
cd "$REPO"
find gpurun_out/r05e/kt -name '*kernel_trace.csv' -delete
F=$(find gpurun_out/r05e/kt -name '*kernel_stats.csv' | head -n 1)
head -25 "$F" | cut -c1-160
echo "== done $(date +%T)"
