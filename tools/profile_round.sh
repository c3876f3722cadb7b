#!/bin/bash
# Round profile set: bench line, kernel-trace stats, FETCH_SIZE calibration, PMC HBM traffic
# (separate FETCH / WRITE passes), MFMA counters.  Usage (GPU box, repo root): tools/profile_round.sh r02
# Extra bench.py arguments (e.g. the surface scene: BENCH_EXTRA="--scene synthetic") come from $BENCH_EXTRA;
# SKIP_CALIB=1 reuses an existing FETCH calibration (gpurun_out/fetch_calib/fetch_calib.json).
# BENCH_SCRIPT=tools/config_e_leg.py profiles the config-E leg alone (default: bench.py).
R=${1:-r02}
OUT=$PWD/gpurun_out/prof_$R
mkdir -p "$OUT"
REPO=$PWD
export TMPDIR=/tmp
SCRIPT=${BENCH_SCRIPT:-bench.py}
STEPS="--steps 10 --warmup 3 --pretrain 1500 --cpu-baseline 0 --surface-scene 0 --config-e 0 --render-in-hbm 0 --mlp-microbench 0 $BENCH_EXTRA"
if [ "${SKIP_CALIB:-0}" != 1 ] || [ ! -f gpurun_out/fetch_calib/fetch_calib.json ]; then
  tools/fetch_calib.sh > "$OUT/fetch_calib.log" 2>&1 || exit $?
fi
cp gpurun_out/fetch_calib/fetch_calib.json "$OUT/fetch_calib.json"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- \
  python3 "$REPO/$SCRIPT" $STEPS > "$OUT/kt.log" 2>&1 || exit $?
timeout -s KILL 500 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pf" -o run -- \
  python3 "$REPO/$SCRIPT" $STEPS > "$OUT/pf.log" 2>&1 || exit $?
timeout -s KILL 500 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pw" -o run -- \
  python3 "$REPO/$SCRIPT" $STEPS > "$OUT/pw.log" 2>&1 || exit $?
cd "$REPO"
F=$(find "$OUT/pf" -name '*counter_collection.csv' | head -n 1)
W=$(find "$OUT/pw" -name '*counter_collection.csv' | head -n 1)
python3 tools/pmc_traffic.py "$F" "$W" "$OUT/pmc_traffic.json" "$OUT/pf.log" "$OUT/fetch_calib.json" > "$OUT/pmc_traffic.txt" || exit $?
# keep only the summaries (the per-dispatch CSVs are far above the gpurun_out cap)
find "$OUT" -name '*kernel_trace.csv' -delete
find "$OUT" -name '*counter_collection.csv' -delete
find "$OUT" -name '*agent_info.csv' -delete
ls -laR "$OUT" | head -n 40
