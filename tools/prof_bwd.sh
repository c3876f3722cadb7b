set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bwd2 -o run -- python3 $R/tools/train_kernels_ab.py --steps 100 --timed 30 --rounds 1 --settings "encode_bwd_binned=2" > $R/gpurun_out/prof_bwd2.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bwd2d -o run -- python3 $R/tools/train_kernels_ab.py --deterministic --steps 100 --timed 30 --rounds 1 --settings "encode_bwd_binned=2" "encode_bwd_binned=1" > $R/gpurun_out/prof_bwd2d.txt 2>&1
rc=$?
cd $R
for d in prof_bwd2 prof_bwd2d; do f=$(find gpurun_out/$d -name '*kernel_stats.csv' | head -1); echo "## $d"; python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in rows:
    n=r['Name']
    if any(k in n for k in ('bwd','scan','hashgrid')): print(n[:90], r['Calls'], r['AverageNs'], r['TotalDurationNs'])
"; done
exit $rc
