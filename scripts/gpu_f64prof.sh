#!/bin/bash
# fp64 engine: parity tests, serialized probe with per-level trace, kernel trace
set -u
OUT=gpurun_out/${RUN:-f64prof}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_f64.py tests/test_gpu_gbm.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
SBAG_OVERLAP=0 SBAG_LEVEL_TRACE=1 timeout -k 10 300 python -u scripts/f64_probe.py > $OUT/probe_trace.log 2>&1 || { echo "probe rc=$?"; tail -30 $OUT/probe_trace.log; exit 1; }
grep "f64 level\|fit_ms" $OUT/probe_trace.log | tail -10
timeout -k 10 300 python -u scripts/f64_probe.py > $OUT/probe.log 2>&1 || { echo "probe rc=$?"; tail -30 $OUT/probe.log; exit 1; }
cat $OUT/probe.log
SBAG_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 scripts/f64_probe.py > $OUT/trace.log 2>&1 || { echo "trace rc=$?"; tail -30 $OUT/trace.log; exit 1; }
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1); head -12 "$f" | cut -c1-160
echo "gpu_f64prof done"
