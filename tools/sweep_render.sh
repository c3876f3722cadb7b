#!/bin/bash
# Render-schedule sweep (diagnostic): bench lines for per-ray budget headroom and the per-pass
# sample cap, plus the kernel timer on/off.  Usage (GPU box, repo root): tools/sweep_render.sh
OUT=$PWD/gpurun_out/sweep
mkdir -p "$OUT"
run() {  # label, env..., -- bench args
  local label=$1; shift
  timeout -k 10 120 env "$@" python3 bench.py --steps 10 --warmup 3 --cpu-baseline 0 > "$OUT/$label.log" 2>&1 || return $?
  python3 - "$OUT/$label.log" "$label" <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1]
d = json.loads(line)
print(f"{sys.argv[2]:28s} value {d['value']:8.2f}  train {d['split']['train_ms_per_step']:.3f} ms  render {d['split']['render_ms_per_frame']:.3f} ms")
PY
}
run base NGP_X=0 || exit $?
timeout -k 10 120 python3 bench.py --steps 10 --warmup 3 --cpu-baseline 0 --kernel-timer 0 > "$OUT/timer_off.log" 2>&1 && grep -h metric "$OUT/timer_off.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(\"timer_off\", d[\"value\"], d[\"split\"][\"render_ms_per_frame\"])"
for b in 1.0 1.25 2.0 off; do run budget_$b NGP_RENDER_BUDGET=$b || exit $?; done
for c in 8 12 24 32; do run steps_$c NGP_RENDER_STEPS_PER_PASS=$c || exit $?; done
run base2 NGP_X=0 || exit $?
