#!/bin/bash
# Round 5, call 46: kernel trace of 8 surface-scene training steps (timers off): per-kernel busy time and idle gaps.
set -o pipefail
mkdir -p gpurun_out/r05ap
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "== trace $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05ap/tr -o tr -- python3 -u tools/probe_gaps.py --train \
  > gpurun_out/r05ap/probe.log 2>&1 || { echo "probe rc=$?"; tail -20 gpurun_out/r05ap/probe.log; exit 1; }
grep "training step" gpurun_out/r05ap/probe.log
f=$(find gpurun_out/r05ap/tr -name "*kernel_trace.csv" | head -1)
python3 tools/gap_summary.py "$f" 4 k_sample_count > gpurun_out/r05ap/gaps.txt && cat gpurun_out/r05ap/gaps.txt
echo "== done $(date +%T)"
