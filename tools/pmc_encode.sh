#!/bin/bash
# PMC counters of the render/train hash-grid kernels (diagnostic). Each pass is its own rocprofv3 run.
OUT=$PWD/gpurun_out/pmc_enc
mkdir -p "$OUT"
REPO=$PWD
export TMPDIR=/tmp
cd /tmp
rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1 || true
i=0
for ctrs in "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "SQ_INSTS_VALU SQ_INSTS_VMEM_RD" "TA_BUSY_avr TA_TA_BUSY_sum" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  CAPS=32 TIMER_MASK=0 timeout -k 10 240 rocprofv3 --pmc $ctrs --output-format csv -d "$OUT/p$i" -o run -- \
    python3 "$REPO/tools/probe_render.py" 400 > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i ($ctrs) rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  F=$(find "$OUT/p$i" -name '*counter_collection.csv' | head -n 1)
  if [ -n "$F" ]; then
    python3 - "$F" "$OUT/p$i.txt" <<'PY'
import csv, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if "hashgrid" in name or "mlp_infer" in name or "k_generate" in name or "k_composite" in name:
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
with open(sys.argv[2], "w") as f:
    for k, d in acc.items():
        f.write(k + " " + " ".join(f"{c}={sum(v)/len(v):.4g}(n={len(v)})" for c, v in d.items()) + "\n")
PY
    find "$OUT/p$i" -name '*.csv' -delete
  fi
done
cat "$OUT"/p*.txt
