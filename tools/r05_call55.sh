#!/bin/bash
# Round 5, call 55: the full -m gpu suite, smoke(), one default bench line.
set -o pipefail
mkdir -p gpurun_out/r05ay
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r05ay/tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/r05ay/tests.log | tail -15
grep -E "test2: corr" gpurun_out/r05ay/tests.log
[ $rc -eq 0 ] || { echo "tests rc=$rc"; exit $rc; }
echo "== smoke $(date +%T)"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05ay/smoke.log 2>&1 \
  || { echo "smoke rc=$?"; tail -20 gpurun_out/r05ay/smoke.log; exit 1; }
tail -2 gpurun_out/r05ay/smoke.log
echo "== bench $(date +%T)"
timeout -k 10 400 python -u bench.py > gpurun_out/r05ay/bench.json 2> gpurun_out/r05ay/bench.err \
  || { echo "bench rc=$?"; tail -20 gpurun_out/r05ay/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r05ay/bench.json'))
print('value',d['value'],'ms',d['ms_per_step'],'roof',d['roofline']['frac'],d['roofline']['us_per_launch'],'split',d['split'])
print('surface',{k:v for k,v in d['surface_scene'].items() if k!='kernels_calibration'})
print('config_e',{k:v for k,v in d['config_e'].items() if k!='kernels_calibration'})
print('hbm',d['render_in_hbm'])"
echo "== done $(date +%T)"
