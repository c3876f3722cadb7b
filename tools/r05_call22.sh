#!/bin/bash
# Round 5, call 22: kernel-timer events without the system-scope fence -- idle gaps with every timer on (surface scene),
# the timing tests, then the default bench line.
set -o pipefail
mkdir -p gpurun_out/r05t
REPO=$PWD
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests -k "kernel_timers or train_step_matches_oracle" \
  > gpurun_out/r05t/tests.txt 2>&1 || { echo "tests rc=$?"; tail -20 gpurun_out/r05t/tests.txt; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/r05t/tests.txt; tail -1 gpurun_out/r05t/tests.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$REPO/gpurun_out/r05t/kt" -o run -- python3 "$REPO/tools/probe_gaps.py" --timers -1 \
  > "$REPO/gpurun_out/r05t/probe.log" 2>&1 || { echo "rc=$?"; tail -5 "$REPO/gpurun_out/r05t/probe.log"; exit 1; }
F=$(find "$REPO/gpurun_out/r05t/kt" -name '*kernel_trace.csv' | head -n 1)
grep "ms per frame" "$REPO/gpurun_out/r05t/probe.log"
python3 "$REPO/tools/gap_summary.py" "$F" 2 | tee "$REPO/gpurun_out/r05t/gaps.txt" | head -8
find "$REPO/gpurun_out/r05t/kt" -name '*.csv' -delete
cd "$REPO"
timeout -k 10 400 python -u bench.py > gpurun_out/r05t/bench.json 2> gpurun_out/r05t/bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/r05t/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r05t/bench.json'))
print('value',d['value'],'ms',d['ms_per_step'],'roof',d['roofline']['frac'],d['roofline']['us_per_launch'],'split',d['split'])
print('surface',d['surface_scene']['Mrays_s'],d['surface_scene']['train_ms_per_step'],d['surface_scene']['render_ms_per_frame'],d['surface_scene']['roofline']['frac'])
print('config_e',d['config_e']['Mrays_s'],'hbm',d['render_in_hbm'])"
echo "== done $(date +%T)"
