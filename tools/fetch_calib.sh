#!/bin/bash
# FETCH_SIZE calibration (tools/fetch_calib.hip) under one rocprofv3 --pmc pass; summary in
# gpurun_out/fetch_calib/fetch_calib.json.  Usage (GPU box, repo root): tools/fetch_calib.sh
OUT=$PWD/gpurun_out/fetch_calib
mkdir -p "$OUT"
[ -x tools/fetch_calib ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o tools/fetch_calib tools/fetch_calib.hip || exit $?
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/raw" -o run -- "$PWD/tools/fetch_calib" > "$OUT/run.log" 2>&1 || exit $?
F=$(find "$OUT/raw" -name '*counter_collection.csv' | head -n 1)
python3 tools/fetch_calib.py "$F" "$OUT/run.log" "$OUT/fetch_calib.json" || exit $?
find "$OUT/raw" -name '*.csv' -delete
cat "$OUT/fetch_calib.json"
