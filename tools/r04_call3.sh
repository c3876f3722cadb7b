#!/bin/bash
# GPU box: bit-identity of the new render-MLP tile variants + the DP retry test, then render A/Bs.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_distributed.py -m gpu -v -s \
  -k "config_e_full or 4-lego" --timeout 300 --timeout-method thread > gpurun_out/r04d_tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed|window loss" gpurun_out/r04d_tests.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "tests rc=$rc"; exit $rc; }
timeout -k 10 300 python -u tools/render_ab.py --rounds 3 --frames 4 "" "render_mlp_tile=2" "render_mlp_tile=3" \
  > gpurun_out/r04d_tile_fire.txt 2> gpurun_out/r04d_tile_fire.err || { echo "render_ab rc=$?"; tail -20 gpurun_out/r04d_tile_fire.err; exit 1; }
cat gpurun_out/r04d_tile_fire.txt
timeout -k 10 300 python -u tools/render_ab.py --scene synthetic --rounds 3 --frames 4 "" "render_pipelines=1" \
  "render_pipelines=1 render_pass_samples=8388608" "render_pipelines=1 render_pass_samples=4194304" "render_mlp_tile=3" \
  "render_pipelines=1 render_mlp_tile=3" "render_pipelines=1 render_first_steps=8" \
  > gpurun_out/r04d_surface.txt 2> gpurun_out/r04d_surface.err || { echo "render_ab rc=$?"; tail -20 gpurun_out/r04d_surface.err; exit 1; }
cat gpurun_out/r04d_surface.txt
tools/pmc_kernels.sh r04d_pmc 'k_mlp_infer_rf' "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVES SQ_INSTS_LDS" \
  -- tools/render_ab.py --rounds 1 --frames 2 --pretrain 300 "render_mlp_tile=3" || exit 1
