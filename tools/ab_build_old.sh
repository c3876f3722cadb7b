#!/bin/bash
# Builds the HIP library + pyngp of an older revision into ab_old/ (git-ignored; travels to the
# GPU box) so tools/render_ab.py --pkg ab_old can time it beside the working tree's build.
# Usage (build container): tools/ab_build_old.sh <rev>
set -e
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=$(mktemp -d /tmp/ngp_ab.XXXXXX)
git -C "$ROOT" worktree add --detach "$WT" "$REV" > /dev/null
make -C "$WT/instant-ngp-rendering_amd" -j8 > "$WT/build.log" 2>&1 || { tail -20 "$WT/build.log"; exit 1; }
rm -rf "$ROOT/ab_old" && mkdir -p "$ROOT/ab_old"
cp "$WT"/instant-ngp-rendering_amd/*.so "$ROOT/ab_old/"
git -C "$ROOT" worktree remove --force "$WT"
echo "ab_old/ <- $(git -C "$ROOT" rev-parse --short "$REV")"
