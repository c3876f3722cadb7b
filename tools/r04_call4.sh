#!/bin/bash
# GPU box: full -m gpu suite, smoke, bench, and A/Bs of the new defaults.
set -o pipefail
mkdir -p gpurun_out
tools/gpu_check.sh r04e; rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/r04e_bench.json 2> gpurun_out/r04e_bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/r04e_bench.err; exit 1; }
python3 -c "
import json;d=json.loads(open('gpurun_out/r04e_bench.json').read().strip().split('\n')[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['split'], d['surface_scene'])"
timeout -k 10 300 python -u tools/render_ab.py --rounds 3 --frames 4 "" "render_mlp_tile=4" \
  > gpurun_out/r04e_fire_ab.txt 2> gpurun_out/r04e_fire_ab.err || { echo "render_ab rc=$?"; tail -20 gpurun_out/r04e_fire_ab.err; exit 1; }
cat gpurun_out/r04e_fire_ab.txt
timeout -k 10 300 python -u tools/render_ab.py --scene synthetic --rounds 3 --frames 4 "" "render_pipelines=2" "render_pipelines=2 render_mlp_tile=4" \
  > gpurun_out/r04e_surface_ab.txt 2> gpurun_out/r04e_surface_ab.err || { echo "render_ab rc=$?"; tail -20 gpurun_out/r04e_surface_ab.err; exit 1; }
cat gpurun_out/r04e_surface_ab.txt
