#!/bin/bash
# Round 5, call 49: HIP API + kernel trace of 8 surface-scene training steps (timers off): the host's share of the
# step-start gap.
set -o pipefail
mkdir -p gpurun_out/r05as
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "== trace $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace --output-format csv -d gpurun_out/r05as/tr -o tr -- \
  python3 -u tools/probe_gaps.py --train > gpurun_out/r05as/probe.log 2>&1 || { echo "probe rc=$?"; tail -20 gpurun_out/r05as/probe.log; exit 1; }
grep "training step" gpurun_out/r05as/probe.log
python3 tools/host_gap_summary.py gpurun_out/r05as/tr 3 > gpurun_out/r05as/host_gaps.txt; cat gpurun_out/r05as/host_gaps.txt
python3 tools/gap_summary.py gpurun_out/r05as/tr/tr_kernel_trace.csv 4 k_sample_count | head -3
rm -rf gpurun_out/r05as/tr
echo "== done $(date +%T)"
