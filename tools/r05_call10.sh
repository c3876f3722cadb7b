#!/bin/bash
# Round 5, call 10: render() into host memory -- streamed pixels vs one read-back vs the frame kept in HBM.
set -o pipefail
mkdir -p gpurun_out/r05i
for sc in fire synthetic; do
  if [ $sc = fire ]; then SC=(); else SC=(--scene synthetic); fi
  echo "== $sc $(date +%T)"
  timeout -k 10 400 python -u tools/render_ab.py "${SC[@]}" --host --rounds 4 --frames 10 "" "render_host_frame=2" "hbm" \
    > gpurun_out/r05i/$sc.txt 2> gpurun_out/r05i/$sc.err || { echo "ab rc=$?"; tail -20 gpurun_out/r05i/$sc.err; exit 1; }
  cat gpurun_out/r05i/$sc.txt
done
echo "== done $(date +%T)"
