#!/bin/bash
# Round 5, call 9: pixels streamed to host memory by the render kernels -- parity tests, then bench.
set -o pipefail
mkdir -p gpurun_out/r05h
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_testbed.py tests/test_gpu_runpy.py -m gpu -v --timeout 300 --timeout-method thread \
  -k "render or runpy or run_py or snapshot" > gpurun_out/r05h/tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/r05h/tests.log | tail -15
[ $rc -eq 0 ] || { echo "tests rc=$rc"; grep -E "Error|assert" gpurun_out/r05h/tests.log | head -20; exit $rc; }
echo "== bench $(date +%T)"
timeout -k 10 400 python -u bench.py --cpu-baseline 0 --config-e 0 > gpurun_out/r05h/bench.json 2> gpurun_out/r05h/bench.err \
  || { echo "bench rc=$?"; tail -20 gpurun_out/r05h/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r05h/bench.json'))
print('value',d['value'],'ms',d['ms_per_step'],'split',{k:v for k,v in d['split'].items() if k!='note'}, 'hbm', d['render_in_hbm'])
s=d['surface_scene']; print('surface',s['Mrays_s'],s['ms_per_step'],s['train_ms_per_step'],s['render_ms_per_frame'])"
echo "== done $(date +%T)"
