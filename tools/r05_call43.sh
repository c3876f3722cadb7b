#!/bin/bash
# Round 5, call 43: closing profile sets of the headline and the surface scene (kernel-trace stats, PMC traffic) on the
# final training and render kernels.
set -o pipefail
echo "== headline profile $(date +%T)"
tools/profile_round.sh r05h > gpurun_out/r05h_profile.log 2>&1 || { echo "profile rc=$?"; tail -20 gpurun_out/r05h_profile.log; exit 1; }
tail -8 gpurun_out/prof_r05h/pmc_traffic.txt
echo "== surface profile $(date +%T)"
SKIP_CALIB=1 BENCH_EXTRA="--scene synthetic" tools/profile_round.sh r05h_surface > gpurun_out/r05h_surface_profile.log 2>&1 \
  || { echo "profile rc=$?"; tail -20 gpurun_out/r05h_surface_profile.log; exit 1; }
tail -12 gpurun_out/prof_r05h_surface/pmc_traffic.txt
echo "== done $(date +%T)"
