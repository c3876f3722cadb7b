#!/bin/bash
# Round 5, call 3: four seeds per reference scene at 35k steps, masks kept for the offline statistics.
set -o pipefail
mkdir -p gpurun_out/r05c
for sc in test2 test; do
echo "== probe $sc $(date +%T)"
timeout -k 10 400 python -u tools/density_slices_probe.py --scene $sc --seeds 1337 42 7 2024 --steps 35000 \
  --out gpurun_out/r05c/ds_${sc}.json --masks gpurun_out/r05c/masks_${sc}.npz > gpurun_out/r05c/ds_${sc}.log 2>&1 \
  || { echo "probe rc=$?"; tail -20 gpurun_out/r05c/ds_${sc}.log; exit 1; }
grep -v "^Wrote\|#lattice" gpurun_out/r05c/ds_${sc}.log | cut -c1-250
done
echo "== done $(date +%T)"
