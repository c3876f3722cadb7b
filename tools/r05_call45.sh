#!/bin/bash
# Round 5, call 45: config-E (aabb 64, T=2^22) render schedule sweep, frame times without timer events.
set -o pipefail
mkdir -p gpurun_out/r05ao
echo "== probe $(date +%T)"
timeout -k 10 400 python -u tools/probe_config_e.py 500 > gpurun_out/r05ao/config_e.log 2>&1 \
  || { echo "probe rc=$?"; tail -20 gpurun_out/r05ao/config_e.log; exit 1; }
cat gpurun_out/r05ao/config_e.log | grep -v "^ *$" | tail -60
echo "== done $(date +%T)"
