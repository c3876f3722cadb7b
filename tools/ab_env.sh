#!/bin/bash
# A/B of an environment setting on the bench (diagnostic): alternates runs without / with it.
# Usage (GPU box, repo root): tools/ab_env.sh "NAME=value" [rounds]
SET=$1; N=${2:-2}
OUT=$PWD/gpurun_out/ab
mkdir -p "$OUT"
summ() {
  python3 - "$1" "$2" <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1]
d = json.loads(line); k = d["kernels_calibration"]
def us(n): return k.get(n, {}).get("us_per_launch", 0)
print(f"{sys.argv[2]:24s} value {d['value']:8.2f} train {d['split']['train_ms_per_step']:.3f} render {d['split']['render_ms_per_frame']:.3f} "
      f"| render_enc {us('render_encode'):7.2f}us train_enc {us('train_encode'):7.2f}us enc_bwd {us('train_encode_bwd'):7.2f}us mlp {us('render_mlp'):6.2f}us")
PY
}
for r in $(seq 1 $N); do
  timeout -k 10 120 python3 bench.py --steps 10 --warmup 3 --cpu-baseline 0 > "$OUT/a$r.log" 2>&1 || exit $?
  summ "$OUT/a$r.log" "base#$r"
  timeout -k 10 120 env $SET python3 bench.py --steps 10 --warmup 3 --cpu-baseline 0 > "$OUT/b$r.log" 2>&1 || exit $?
  summ "$OUT/b$r.log" "$SET#$r"
done
