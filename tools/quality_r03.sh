#!/bin/bash
# Held-out quality (scripts/run.py:178-268 protocol: n_steps of training, spp-8 renders, black
# background, min transmittance 1e-4, linear_to_srgb PSNR / SSIM) on static scenes with a true split:
#  * data/nerf/fox: every 8th frame held out (tools/split_scene.py), base.json (the fork's default);
#  * the procedural lego-shaped scene: 100 train / 200 test views (tools/make_synthetic_scene.py),
#    lego_L16F2.json (BASELINE config B).
# Usage (GPU box, repo root): tools/quality_r03.sh [n_steps] [tag]
N=${1:-35000}
OUT=gpurun_out/quality_${2:-r03}
T=${TMPDIR:-/tmp}
mkdir -p "$OUT"
python3 tools/split_scene.py data/nerf/fox/transforms.json 8 "$T/fox_split" 2> "$OUT/split.log" || exit $?
timeout -k 10 400 python3 instant-ngp-rendering_amd/run.py --scene "$T/fox_split/transforms_train.json" --network base.json \
  --n_steps $N --test_transforms "$T/fox_split/transforms_test.json" > "$OUT/fox_heldout.json" 2> "$OUT/fox_heldout.log" || exit $?
timeout -k 10 300 python3 tools/make_synthetic_scene.py "$T/synth" > "$OUT/synth_make.log" 2>&1 || exit $?
timeout -k 10 600 python3 instant-ngp-rendering_amd/run.py --scene "$T/synth/transforms_train.json" --network lego_L16F2.json \
  --n_steps $N --test_transforms "$T/synth/transforms_test.json" > "$OUT/synth_heldout.json" 2> "$OUT/synth_heldout.log" || exit $?
cat "$OUT"/*.json
