#!/bin/bash
# Round 5, call 41: read-back lag 2 and no exit cap as defaults -- A/B against the previous defaults, render tests, bench.
set -o pipefail
mkdir -p gpurun_out/r05al
timeout -k 10 600 python -u tools/render_ab.py --host --rounds 6 --frames 5 "" "render_lag=3 render_exit_cap=1" \
  > gpurun_out/r05al/fire.txt 2>&1 || { echo "rc=$?"; tail -20 gpurun_out/r05al/fire.txt; exit 1; }
grep "ms/frame" gpurun_out/r05al/fire.txt
timeout -k 10 600 python -u tools/render_ab.py --scene synthetic --host --rounds 6 --frames 5 "" "render_lag=3 render_exit_cap=1" \
  > gpurun_out/r05al/surface.txt 2>&1 || { echo "rc=$?"; tail -20 gpurun_out/r05al/surface.txt; exit 1; }
grep "ms/frame" gpurun_out/r05al/surface.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_testbed.py tests/test_gpu_pipeline.py tests/test_gpu_render_modes.py -k "render or 1080p or streams or retires or frame" \
  > gpurun_out/r05al/tests.txt 2>&1 || { echo "tests rc=$?"; tail -20 gpurun_out/r05al/tests.txt; exit 1; }
tail -1 gpurun_out/r05al/tests.txt
timeout -k 10 400 python -u bench.py > gpurun_out/r05al/bench.json 2> gpurun_out/r05al/bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/r05al/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r05al/bench.json'))
print('value',d['value'],'ms',d['ms_per_step'],'roof',d['roofline']['frac'],d['roofline']['us_per_launch'],'split',d['split'])
print('surface',d['surface_scene']['Mrays_s'],d['surface_scene']['train_ms_per_step'],d['surface_scene']['render_ms_per_frame'],d['surface_scene']['roofline']['frac'])
print('config_e',d['config_e']['Mrays_s'],d['config_e']['render_ms_per_frame'],'hbm',d['render_in_hbm']['ms_per_frame'])"
echo "== done $(date +%T)"
