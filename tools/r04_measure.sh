#!/bin/bash
# Round-4 measurement session (GPU box, repo root): the default bench line, the same bench under
# rocprofv3 --kernel-trace --stats, and same-box A/Bs of the render exit cap (fire and surface scene)
# and of the binned hash-grid backward.  Every GPU step has its own time limit; the first failure ends it.
set -o pipefail
T=${1:-r04}
mkdir -p gpurun_out
R=$PWD
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
step bench
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err \
  || { echo "bench rc=$?"; tail -20 gpurun_out/${T}_bench.err; exit 1; }
tail -c 600 gpurun_out/${T}_bench.json
step rocprof
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_kt -o run -- \
  python3 $R/bench.py --steps 10 --warmup 3 --cpu-baseline 0 --surface-scene 0 --render-to-cpu 0 \
  > $R/gpurun_out/${T}_bench_under_rocprof.json 2> $R/gpurun_out/${T}_kt.err || { echo "rocprof rc=$?"; exit 1; }
cd $R
find gpurun_out/${T}_kt -name '*kernel_trace.csv' -delete
find gpurun_out/${T}_kt -name '*agent_info.csv' -delete
step render_ab_fire
timeout -k 10 300 python -u tools/render_ab.py --rounds 3 --frames 4 "" "render_exit_cap=2" \
  > gpurun_out/${T}_exitcap_fire.txt 2> gpurun_out/${T}_exitcap_fire.err || { echo "render_ab rc=$?"; tail -20 gpurun_out/${T}_exitcap_fire.err; exit 1; }
cat gpurun_out/${T}_exitcap_fire.txt
step render_ab_surface
timeout -k 10 300 python -u tools/render_ab.py --scene synthetic --rounds 3 --frames 4 "" "render_exit_cap=2" \
  "render_pass_samples=4194304" "render_pass_samples=8388608" "render_pipelines=1" "render_first_steps=2" \
  > gpurun_out/${T}_surface_ab.txt 2> gpurun_out/${T}_surface_ab.err || { echo "render_ab rc=$?"; tail -20 gpurun_out/${T}_surface_ab.err; exit 1; }
cat gpurun_out/${T}_surface_ab.txt
step train_ab
timeout -k 10 300 python -u tools/train_kernels_ab.py --steps 300 --timed 50 --rounds 3 --settings "" "encode_bwd_binned=2" "encode_bwd_binned=3" \
  > gpurun_out/${T}_bwd_ab.txt 2> gpurun_out/${T}_bwd_ab.err || { echo "train_ab rc=$?"; tail -20 gpurun_out/${T}_bwd_ab.err; exit 1; }
cat gpurun_out/${T}_bwd_ab.txt
step pmc_mlp
timeout -k 10 600 tools/pmc_kernels.sh ${T}_pmc_mlp 'k_mlp' \
  "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES" \
  "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAVES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_WAIT_INST_LDS SQ_WAVE_CYCLES" \
  -- bench.py --steps 5 --warmup 3 --pretrain 300 --cpu-baseline 0 --surface-scene 0 --render-to-cpu 0 || { echo "pmc rc=$?"; exit 1; }
step trace
timeout -k 10 400 tools/trace_frames.sh ${T} > gpurun_out/${T}_trace.txt 2>&1 || { echo "trace rc=$?"; tail -5 gpurun_out/${T}_trace.txt; exit 1; }
tail -30 gpurun_out/${T}_trace.txt
step done
