#!/bin/bash
# GPU box: DP retry probe, then a longer render-MLP tile A/B on the fire scene.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/dp_retry_probe.py > gpurun_out/r04f_probe.txt 2> gpurun_out/r04f_probe.err
rc=$?; cat gpurun_out/r04f_probe.txt; [ $rc -eq 0 ] || { echo "probe rc=$rc"; tail -20 gpurun_out/r04f_probe.err; exit $rc; }
timeout -k 10 300 python -u tools/render_ab.py --rounds 6 --frames 5 "" "render_mlp_tile=2" "render_mlp_tile=4" \
  > gpurun_out/r04f_fire_tile.txt 2> gpurun_out/r04f_fire_tile.err || { echo "render_ab rc=$?"; tail -20 gpurun_out/r04f_fire_tile.err; exit 1; }
cat gpurun_out/r04f_fire_tile.txt
