#!/bin/bash
# Builder-side helper: submit one gpurun command, re-submitting only while the pod has no GPU slot or box free
# (nothing ran, nothing charged).  Any run that reached a box -- pass or fail -- is final.
# Usage: tools/gpurun_retry.sh OUTFILE TIMEOUT 'command'
OUT=$1; TO=$2; CMD=$3
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$OUT" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient rc=None charged=0.0s" "$OUT"; then
    echo "[retry $i: no slot] $(date +%T)" >> "$OUT.retries"; sleep 90; continue
  fi
  echo "rc=$rc" >> "$OUT"; exit $rc
done
echo "gave up" >> "$OUT"; exit 3
