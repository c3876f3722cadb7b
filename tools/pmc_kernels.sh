#!/bin/bash
# PMC counters per kernel for any python command (diagnostic).  Each counter set is its own
# rocprofv3 --pmc run; per-kernel means land in gpurun_out/<label>/p<i>.txt.
# Usage (GPU box, repo root): tools/pmc_kernels.sh <label> <kernel-name regex> "<counter set>" ["<counter set>" ...] -- <python args...>
LABEL=$1; PATTERN=$2; shift 2
SETS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do SETS+=("$1"); shift; done
shift
OUT=$PWD/gpurun_out/$LABEL
mkdir -p "$OUT"
REPO=$PWD
ARGS=("$@")
[ -f "$REPO/${ARGS[0]}" ] && ARGS[0]="$REPO/${ARGS[0]}"
export TMPDIR=/tmp
i=0
for ctrs in "${SETS[@]}"; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 240 rocprofv3 --pmc $ctrs --output-format csv -d "$OUT/p$i" -o run -- python3 "${ARGS[@]}") > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i ($ctrs) rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 5 "$OUT/p$i.log"; exit $rc; fi
  F=$(find "$OUT/p$i" -name '*counter_collection.csv' | head -n 1)
  [ -n "$F" ] || continue
  python3 - "$F" "$OUT/p$i.txt" "$PATTERN" <<'PY'
import csv, re, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if re.search(sys.argv[3], name):
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
with open(sys.argv[2], "w") as f:
    for k, d in sorted(acc.items()):
        f.write(k + " " + " ".join(f"{c}={sum(v)/len(v):.4g}(n={len(v)})" for c, v in d.items()) + "\n")
PY
  find "$OUT/p$i" -name '*.csv' -delete
done
cat "$OUT"/p*.txt
