#!/bin/bash
# Round 5, call 37: surface default cap 24 vs 32; fire unchanged; frame identity under schedules; bench.
set -o pipefail
mkdir -p gpurun_out/r05ai
timeout -k 10 600 python -u tools/render_ab.py --scene synthetic --host --rounds 6 --frames 5 "" "render_max_steps=32" \
  > gpurun_out/r05ai/surface.txt 2>&1 || { echo "rc=$?"; tail -20 gpurun_out/r05ai/surface.txt; exit 1; }
grep "ms/frame" gpurun_out/r05ai/surface.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_testbed.py tests/test_gpu_pipeline.py -k "1080p or streams or retires or render" \
  > gpurun_out/r05ai/tests.txt 2>&1 || { echo "tests rc=$?"; tail -20 gpurun_out/r05ai/tests.txt; exit 1; }
tail -1 gpurun_out/r05ai/tests.txt
timeout -k 10 400 python -u bench.py > gpurun_out/r05ai/bench.json 2> gpurun_out/r05ai/bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/r05ai/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r05ai/bench.json'))
print('value',d['value'],'ms',d['ms_per_step'],'roof',d['roofline']['frac'],d['roofline']['us_per_launch'],'split',d['split'])
print('surface',d['surface_scene']['Mrays_s'],d['surface_scene']['train_ms_per_step'],d['surface_scene']['render_ms_per_frame'],d['surface_scene']['roofline']['frac'])
print('config_e',d['config_e']['Mrays_s'],d['config_e']['render_ms_per_frame'],'hbm',d['render_in_hbm']['ms_per_frame'])"
echo "== done $(date +%T)"
