#!/bin/bash
# GPU box, repo root: the full -m gpu suite, smoke() and one default bench line, each under its own limit.
# Usage: tools/gpu_check.sh TAG [pytest -k expression]
set -o pipefail
TAG=${1:-check}
K=${2:-}
mkdir -p gpurun_out
echo "== tests $(date +%T)"
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 780 python -u -m pytest tests -m gpu -v "${KARG[@]}" --timeout 200 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed|Error" gpurun_out/${TAG}_tests.log | tail -15
[ $rc -eq 0 ] || { echo "tests rc=$rc"; exit $rc; }
echo "== smoke $(date +%T)"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
  || { echo "smoke rc=$?"; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -2 gpurun_out/${TAG}_smoke.log
echo "== done $(date +%T)"
