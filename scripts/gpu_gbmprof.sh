#!/bin/bash
set -u
OUT=gpurun_out/${RUN:-gbmprof}
mkdir -p $OUT
export TMPDIR=/tmp
for n in 100000 1000000; do
  timeout -k 10 300 python -u scripts/gbm_probe.py $n > $OUT/probe_$n.log 2>&1 || { echo "probe rc=$?"; tail -30 $OUT/probe_$n.log; exit 1; }
  tail -1 $OUT/probe_$n.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 scripts/gbm_probe.py 1000000 > $OUT/trace.log 2>&1 || { echo "trace rc=$?"; tail -30 $OUT/trace.log; exit 1; }
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1); head -14 "$f" | cut -c1-160
echo "gpu_gbmprof done"
