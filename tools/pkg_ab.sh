#!/bin/bash
# Frame-time A/B of two builds on one box and one snapshot: the working tree's pyngp against
# ab_old/ (tools/ab_build_old.sh), alternating processes (diagnostic, GPU box, repo root).
# Usage: tools/pkg_ab.sh [rounds] [frames] [setting ...]
N=${1:-3}; F=${2:-5}; shift 2
OUT=gpurun_out/pkg_ab; mkdir -p "$OUT"
SNAP=/tmp/pkg_ab_snapshot.ingp
timeout -k 10 300 python3 tools/render_ab.py --rounds 1 --frames 2 --snapshot "$SNAP" "" > "$OUT/train.log" 2>&1 || exit $?
for r in $(seq 1 "$N"); do
  for pkg in ab_old new; do
    arg=""; [ "$pkg" = ab_old ] && arg="--pkg ab_old"
    timeout -k 10 200 python3 tools/render_ab.py --rounds 1 --frames "$F" --snapshot "$SNAP" $arg "" "$@" > "$OUT/$pkg.$r.log" 2>&1 || exit $?
    echo "[$pkg round $r]"; grep -v '^#' "$OUT/$pkg.$r.log"
  done
done
