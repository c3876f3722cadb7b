#!/bin/bash
# Round 5, call 5: round profile sets of the headline and of the surface scene (kernel-trace stats, PMC traffic).
set -o pipefail
echo "== headline profile $(date +%T)"
tools/profile_round.sh r05 > gpurun_out/r05_profile.log 2>&1 || { echo "profile rc=$?"; tail -20 gpurun_out/r05_profile.log; exit 1; }
tail -8 gpurun_out/prof_r05/pmc_traffic.txt
echo "== surface profile $(date +%T)"
SKIP_CALIB=1 BENCH_EXTRA="--scene synthetic" tools/profile_round.sh r05_surface > gpurun_out/r05_surface_profile.log 2>&1 \
  || { echo "profile rc=$?"; tail -20 gpurun_out/r05_surface_profile.log; exit 1; }
tail -12 gpurun_out/prof_r05_surface/pmc_traffic.txt
echo "== done $(date +%T)"
