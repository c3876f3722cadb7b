#!/bin/bash
# Per-kernel average durations (rocprofv3 --stats) of a short bench run without / with an
# environment setting, alternating (diagnostic).  Usage (GPU box, repo root):
#   tools/prof_ab.sh "NAME=value" [rounds]
SET=$1; N=${2:-1}
OUT=$PWD/gpurun_out/prof_ab
mkdir -p "$OUT"
REPO=$PWD
export TMPDIR=/tmp
run() {  # $1 label, $2 env assignment or empty
  cd /tmp
  if [ -n "$2" ]; then export "$2"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$1" -o run -- \
    python3 "$REPO/bench.py" --steps 10 --warmup 3 --cpu-baseline 0 > "$OUT/$1.log" 2>&1
  local rc=$?
  if [ -n "$2" ]; then unset "${2%%=*}"; fi
  cd "$REPO"
  [ $rc -eq 0 ] || exit $rc
  F=$(find "$OUT/$1" -name '*kernel_stats.csv' | head -n 1)
  python3 - "$F" "$1" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"== {sys.argv[2]}: total {tot/1e6:.2f} ms")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f"  {float(r['TotalDurationNs'])/1e6:7.3f} ms {int(r['Calls']):6d} x {float(r['AverageNs'])/1e3:8.2f} us  {r['Name'][:90]}")
PY
  find "$OUT/$1" -name '*trace.csv' -delete
}
for r in $(seq 1 $N); do
  run "base$r" ""
  run "set$r" "$SET"
done
