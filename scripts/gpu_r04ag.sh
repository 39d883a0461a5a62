#!/bin/bash
# GBM 10M x 100 kernel trace
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04ag}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 scripts/bench_gbm.py --synthetic --rows 10000000 --features 100 --depth 5 --learners 3 > $OUT/trace.log 2>&1 || { echo "trace rc=$?"; tail -30 $OUT/trace.log; exit 1; }
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1); head -20 "$f" | cut -c1-150
echo "gpu_r04ag done"
