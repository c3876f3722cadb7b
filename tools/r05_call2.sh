#!/bin/bash
# Round 5, call 2: reference-mosaic probe with and without random background colours, slice previews.
set -o pipefail
mkdir -p gpurun_out
for sc in test test2; do for bg in 1 0; do
echo "== probe $sc bg=$bg $(date +%T)"
timeout -k 10 300 python -u tools/density_slices_probe.py --scene $sc --random-bg $bg --seeds 1337 42 --steps 1000 5000 35000 \
  --out gpurun_out/r05b_ds_${sc}_bg${bg}.json --save gpurun_out/r05b_prev > gpurun_out/r05b_ds_${sc}_bg${bg}.log 2>&1 \
  || { echo "probe rc=$?"; tail -20 gpurun_out/r05b_ds_${sc}_bg${bg}.log; exit 1; }
grep -v "^Wrote\|#lattice" gpurun_out/r05b_ds_${sc}_bg${bg}.log | cut -c1-330
done; done
echo "== done $(date +%T)"
