#!/bin/bash
# Round-4 GPU session (GPU box, repo root): tests, then the A/Bs named in DESIGN.md.  Every GPU step has its
# own time limit; test failures (rc 1) go on to the A/Bs, anything else (timeout, crash) ends the session.
set -o pipefail
mkdir -p gpurun_out
step() { echo "== $1 $(date +%T)"; }
ok_or_fail() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
step tests
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_pipeline.py tests/test_gpu_render_modes.py \
  tests/test_gpu_distributed.py -k "2-lego or hashgrid_backward or deterministic or glow or train_step_matches" \
  -v -s --timeout 300 --timeout-method thread > gpurun_out/r04_tests_b.log 2>&1
rc=$?; grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/r04_tests_b.log | tail -12; grep "within 1 fp16\|dL/dout rel" gpurun_out/r04_tests_b.log
ok_or_fail $rc || { echo "tests rc=$rc"; exit 1; }
step train_ab
timeout -k 10 400 python -u tools/train_kernels_ab.py --steps 300 --timed 50 --rounds 3 --settings "" "encode_bwd_binned=1" "encode_bwd_binned=2" \
  > gpurun_out/r04_bwd_ab.txt 2> gpurun_out/r04_bwd_ab.err || { echo "train_ab rc=$?"; tail -20 gpurun_out/r04_bwd_ab.err; exit 1; }
cat gpurun_out/r04_bwd_ab.txt
step render_ab
timeout -k 10 400 python -u tools/render_ab.py --rounds 3 --frames 4 "" "render_exit_cap=2" "render_mlp_tile=1" \
  > gpurun_out/r04_exitcap_ab.txt 2> gpurun_out/r04_exitcap_ab.err || { echo "render_ab rc=$?"; tail -20 gpurun_out/r04_exitcap_ab.err; exit 1; }
cat gpurun_out/r04_exitcap_ab.txt
step done
