#!/bin/bash
# Round-4 closing measurements (GPU box, repo root): the round profile set (kernel-trace stats, FETCH_SIZE
# calibration, PMC FETCH / WRITE traffic of the bench) and one default bench line.
set -o pipefail
mkdir -p gpurun_out
echo "== profile $(date +%T)"
tools/profile_round.sh r04 > gpurun_out/r04_profile.log 2>&1 || { echo "profile rc=$?"; tail -20 gpurun_out/r04_profile.log; exit 1; }
tail -5 gpurun_out/prof_r04/pmc_traffic.txt
echo "== bench $(date +%T)"
timeout -k 10 200 python -u bench.py --traffic-json gpurun_out/prof_r04/pmc_traffic.json > gpurun_out/r04_final_bench.json 2> gpurun_out/r04_final_bench.err \
  || { echo "bench rc=$?"; tail -20 gpurun_out/r04_final_bench.err; exit 1; }
echo "== done $(date +%T)"
