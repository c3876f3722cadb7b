#!/bin/bash
# Round 5, call 7: loss kernels with G lanes per ray -- training parity tests, then the bench's train split.
set -o pipefail
mkdir -p gpurun_out/r05f
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_golden.py tests/test_gpu_testbed.py tests/test_gpu_distributed.py \
  -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r05f/tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/r05f/tests.log | tail -15
[ $rc -eq 0 ] || { echo "tests rc=$rc"; exit $rc; }
echo "== bench $(date +%T)"
timeout -k 10 400 python -u bench.py --cpu-baseline 0 --config-e 0 > gpurun_out/r05f/bench.json 2> gpurun_out/r05f/bench.err \
  || { echo "bench rc=$?"; tail -20 gpurun_out/r05f/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r05f/bench.json'))
print('value',d['value'],'ms',d['ms_per_step'],'split',{k:v for k,v in d['split'].items() if k!='note'})
s=d['surface_scene']; print('surface',s['Mrays_s'],s['ms_per_step'],s['train_ms_per_step'],s['render_ms_per_frame'])
for leg,kc in (('headline',d['kernels_calibration']),('surface',s['kernels_calibration'])):
  print(leg,{k:round(v['ms_total']/3*1000,1) for k,v in kc.items() if k.startswith('train') or k in ('optimizer','grid_update')})"
echo "== done $(date +%T)"
