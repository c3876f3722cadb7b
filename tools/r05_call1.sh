#!/bin/bash
# Round 5, call 1 (GPU box, repo root): density-slice parity tests, the reference-mosaic probe on both scenes,
# one default bench line.
set -o pipefail
mkdir -p gpurun_out
echo "== tests $(date +%T)"
timeout -k 10 400 python -u -m pytest tests/test_gpu_density_slices.py -v --timeout 300 --timeout-method thread \
  > gpurun_out/r05a_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/r05a_tests.log; exit 1; }
tail -3 gpurun_out/r05a_tests.log
echo "== probe test $(date +%T)"
timeout -k 10 400 python -u tools/density_slices_probe.py --scene test --seeds 1337 42 --steps 1000 3000 10000 35000 \
  --out gpurun_out/r05a_ds_test.json --save gpurun_out/r05a_slices > gpurun_out/r05a_ds_test.log 2>&1 \
  || { echo "probe rc=$?"; tail -20 gpurun_out/r05a_ds_test.log; exit 1; }
grep -v "^Wrote\|#lattice" gpurun_out/r05a_ds_test.log
echo "== probe test2 $(date +%T)"
timeout -k 10 500 python -u tools/density_slices_probe.py --scene test2 --seeds 1337 42 --steps 1000 3000 10000 35000 \
  --out gpurun_out/r05a_ds_test2.json --save gpurun_out/r05a_slices > gpurun_out/r05a_ds_test2.log 2>&1 \
  || { echo "probe rc=$?"; tail -20 gpurun_out/r05a_ds_test2.log; exit 1; }
grep -v "^Wrote\|#lattice" gpurun_out/r05a_ds_test2.log
echo "== bench $(date +%T)"
timeout -k 10 300 python -u bench.py > gpurun_out/r05a_bench.json 2> gpurun_out/r05a_bench.err \
  || { echo "bench rc=$?"; tail -20 gpurun_out/r05a_bench.err; exit 1; }
cat gpurun_out/r05a_bench.json | cut -c1-600
echo "== done $(date +%T)"
