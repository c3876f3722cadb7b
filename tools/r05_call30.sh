#!/bin/bash
# Round 5, call 30: training trajectory of the collapsing test2 seeds.
set -o pipefail
mkdir -p gpurun_out/r05ab
timeout -k 10 300 python -u tools/probe_collapse.py 2024 0 > gpurun_out/r05ab/s2024.txt 2>&1 || { echo "rc=$?"; tail -20 gpurun_out/r05ab/s2024.txt; exit 1; }
cat gpurun_out/r05ab/s2024.txt | grep -v "^Wrote"
timeout -k 10 300 python -u tools/probe_collapse.py 1337 0 > gpurun_out/r05ab/s1337.txt 2>&1 || { echo "rc=$?"; tail -20 gpurun_out/r05ab/s1337.txt; exit 1; }
cat gpurun_out/r05ab/s1337.txt | grep -v "^Wrote"
echo "== done $(date +%T)"
