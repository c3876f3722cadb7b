#!/bin/bash
# Runs GPU steps in order; stops at the first step that faults, aborts, segfaults or times out.
# Usage: tools/gpu_session.sh "<label>:<seconds>:<command>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  label="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$label] ($secs s) $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$label.log" 2>&1
  rc=$?
  echo "=== [$label] rc=$rc"; tail -n 25 "gpurun_out/$label.log"
  case $rc in
    0|1|5) ;;  # pass / test failures / no tests: keep going
    *) echo "=== stopping after rc=$rc"; exit $rc ;;
  esac
done
