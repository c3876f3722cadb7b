#!/bin/bash
# rocprofv3 --kernel-trace --stats of a python command; per-kernel totals in gpurun_out/<label>/stats.txt
# Usage (GPU box, repo root): tools/kstats.sh <label> <python args...>
LABEL=$1; shift
OUT=$PWD/gpurun_out/$LABEL
mkdir -p "$OUT"
REPO=$PWD
ARGS=("$@")
[ -f "$REPO/${ARGS[0]}" ] && ARGS[0]="$REPO/${ARGS[0]}"
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 "${ARGS[@]}") > "$OUT/run.log" 2>&1 || { tail -n 20 "$OUT/run.log"; exit 1; }
F=$(find "$OUT/kt" -name '*kernel_stats.csv' | head -n 1)
python3 - "$F" "$OUT/stats.txt" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
with open(sys.argv[2], "w") as f:
    for r in rows[:30]:
        f.write(f'{float(r["TotalDurationNs"])/1e6:10.3f} ms {int(r["Calls"]):7d} calls {float(r["AverageNs"])/1e3:9.2f} us  {r["Name"][:110]}\n')
PY
cp "$F" "$OUT/kernel_stats.csv"
find "$OUT/kt" -name '*.csv' -delete
cat "$OUT/stats.txt"
