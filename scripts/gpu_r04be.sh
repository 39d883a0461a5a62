#!/bin/bash
# kernel trace of the C3-sized continuous fit
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04be}
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 scripts/bench_continuous.py > $OUT/trace.log 2>&1 || { echo "trace rc=$?"; tail -30 $OUT/trace.log; exit 1; }
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/kernel_stats.csv; head -14 "$f" | cut -c1-150
rm -rf $OUT/trace
echo "gpu_r04be done"
