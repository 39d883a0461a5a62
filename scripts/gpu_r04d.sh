#!/bin/bash
# fp64 engine breakdown: serialized probe with per-level trace, and a kernel trace
set -u
OUT=gpurun_out/${RUN:-r04d}
mkdir -p $OUT
export TMPDIR=/tmp
SBAG_OVERLAP=0 SBAG_LEVEL_TRACE=1 timeout -k 10 300 python -u scripts/f64_probe.py > $OUT/probe_trace.log 2>&1 || { echo "probe rc=$?"; tail -30 $OUT/probe_trace.log; exit 1; }
grep "f64 level\|fit_ms" $OUT/probe_trace.log | tail -12
SBAG_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 scripts/f64_probe.py > $OUT/trace.log 2>&1 || { echo "trace rc=$?"; tail -30 $OUT/trace.log; exit 1; }
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1); head -20 "$f"
echo "gpu_r04d done"
