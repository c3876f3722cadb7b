#!/bin/bash
# Round 5, call 23: SQ counters of the render march kernels (k_generate, k_composite) and the render encoder / MLP in the
# bench frame (fire scene).
set -o pipefail
timeout -k 10 700 tools/pmc_kernels.sh r05u "k_generate|k_composite|k_hashgrid_fwd<2u, 1|k_mlp_infer_rf<.*true>$" \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD" \
  "SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM" \
  -- bench.py --steps 3 --warmup 2 --pretrain 300 --cpu-baseline 0 --surface-scene 0 --config-e 0 --render-in-hbm 0 \
  > gpurun_out/r05u.log 2>&1 || { echo "rc=$?"; tail -20 gpurun_out/r05u.log; exit 1; }
cat gpurun_out/r05u/p*.txt | cut -c1-600
echo "== done $(date +%T)"
