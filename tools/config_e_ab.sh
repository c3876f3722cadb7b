mkdir -p gpurun_out/r06ae /tmp/fox64
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_kernels.py tests/test_gpu_config_e.py tests/test_gpu_render_modes.py -m gpu -x -q --timeout 300 --timeout-method thread -k "render or march or config_e or lens or cascade" > gpurun_out/r06ae/tests.log 2>&1 || exit 1
S=$(python3 -c "import sys; sys.path.insert(0,'tests'); from test_gpu_config_e import fox_aabb64; print(fox_aabb64('/tmp/fox64'))")
C=instant-ngp-rendering_amd/configs/nerf/bicycle_L16F2T22.json
timeout -k 10 300 python3 tools/render_ab.py --rounds 1 --frames 2 --pretrain 500 --scene "$S" --config "$C" --snapshot /tmp/e.ingp "" > gpurun_out/r06ae/train.log 2>&1 || exit 2
for r in 1 2 3; do
  for pkg in ab_old new; do
    arg=""; [ "$pkg" = ab_old ] && arg="--pkg ab_old"
    timeout -k 10 200 python3 tools/render_ab.py --rounds 1 --frames 4 --scene "$S" --config "$C" --snapshot /tmp/e.ingp $arg "" > gpurun_out/r06ae/$pkg.$r.log 2>&1 || exit 3
    echo "[$pkg round $r] $(grep -v '^#' gpurun_out/r06ae/$pkg.$r.log)"
  done
done
