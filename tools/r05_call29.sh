#!/bin/bash
# Round 5, call 29: spread of the reference-mosaic statistics over seeds, nondeterministic vs deterministic training.
set -o pipefail
mkdir -p gpurun_out/r05aa
timeout -k 10 1100 python -u tools/probe_mosaic_stats.py > gpurun_out/r05aa/stats.txt 2>&1 || { echo "rc=$?"; tail -20 gpurun_out/r05aa/stats.txt; exit 1; }
cat gpurun_out/r05aa/stats.txt | grep -v "^Wrote\|lattice"
echo "== done $(date +%T)"
