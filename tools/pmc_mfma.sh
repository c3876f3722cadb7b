#!/bin/bash
# MFMA / LDS counters of the fused MLP kernels (k_mlp_train, k_mlp_infer_rf) over a short bench
# run: one rocprofv3 --pmc pass (7 SQ + 1 GRBM counters), summarised per kernel by
# tools/pmc_mfma.py.  Usage (GPU box, repo root): tools/pmc_mfma.sh r02 [extra bench args]
R=${1:-r02}; shift
OUT=$PWD/gpurun_out/pmc_mfma_$R
mkdir -p "$OUT"
REPO=$PWD
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_LDS SQ_WAIT_INST_LDS \
  SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/raw" -o run -- \
  python3 "$REPO/bench.py" --steps 5 --warmup 3 --pretrain 300 --cpu-baseline 0 "$@" > "$OUT/bench.log" 2>&1 || exit $?
cd "$REPO"
F=$(find "$OUT/raw" -name '*counter_collection.csv' | head -n 1)
python3 tools/pmc_mfma.py "$F" "$OUT/pmc_mfma.json" > "$OUT/pmc_mfma.txt" || exit $?
find "$OUT/raw" -name '*.csv' -delete
cat "$OUT/pmc_mfma.txt"
