#!/bin/bash
# Bench under several environment settings (diagnostic), one run each, one summary line per run.
# Usage (GPU box, repo root): tools/sweep_env.sh "" "A=1 B=2" "A=3" ...   ("" = defaults)
# Extra bench flags: BENCH_ARGS="--steps 10".  DEBUG=1 adds the per-frame pass statistics (NGP_RENDER_DEBUG: slow).
OUT=$PWD/gpurun_out/sweep
mkdir -p "$OUT"
ARGS=${BENCH_ARGS:---steps 10 --warmup 3 --cpu-baseline 0}
i=0
for SET in "$@"; do
  i=$((i + 1))
  timeout -k 10 150 env ${DEBUG:+NGP_RENDER_DEBUG=1} $SET python3 bench.py $ARGS > "$OUT/s$i.log" 2>&1 || { echo "run $i ($SET) rc=$?"; tail -5 "$OUT/s$i.log"; exit 1; }
  python3 - "$OUT/s$i.log" "${SET:-default}" <<'PY'
import json, sys
lines = open(sys.argv[1]).read().splitlines()
d = json.loads([l for l in lines if l.startswith('{"metric"')][-1]); k = d["kernels_calibration"]
def us(n): return k.get(n, {}).get("us_per_launch", 0)
def ms(n): return k.get(n, {}).get("ms_total", 0) / 3
print(f"{sys.argv[2]:40s} value {d['value']:8.2f} train {d['split']['train_ms_per_step']:.3f} render {d['split']['render_ms_per_frame']:.3f} "
      f"| per frame: march {ms('render_march'):.2f} enc {ms('render_encode'):.2f} mlp {ms('render_mlp'):.2f} ms"
      f" | enc {us('render_encode'):.1f}us/launch")
dbg = [l for l in lines if l.startswith("[render]")]
if dbg: print("    " + dbg[-1])
PY
done
