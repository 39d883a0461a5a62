#!/bin/bash
# fp64 chains: labels exploded into LDS per stage (no per-entry count loop)
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04p}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_f64.py tests/test_gpu_gbm.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
SBAG_OVERLAP=0 SBAG_LEVEL_TRACE=1 timeout -k 10 300 python -u scripts/f64_probe.py > $OUT/probe_trace.log 2>&1 || { echo "probe rc=$?"; tail -30 $OUT/probe_trace.log; exit 1; }
grep "ms: hist\|fit_ms" $OUT/probe_trace.log | tail -10
timeout -k 10 300 python -u scripts/f64_probe.py > $OUT/probe.log 2>&1 || { echo "probe rc=$?"; tail -30 $OUT/probe.log; exit 1; }
echo "overlapped: $(tail -1 $OUT/probe.log)"
timeout -k 10 300 python -u scripts/bench_gbm.py > $OUT/bench_gbm.log 2>&1 || { echo "bench_gbm rc=$?"; tail -20 $OUT/bench_gbm.log; exit 1; }
cat $OUT/bench_gbm.log
SBAG_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ftrace -o trace -- python3 scripts/f64_probe.py > $OUT/ftrace.log 2>&1 || { echo "ftrace rc=$?"; tail -30 $OUT/ftrace.log; exit 1; }
f=$(find $OUT/ftrace -name "*kernel_stats.csv" | head -1); head -12 "$f" | cut -c1-160
echo "gpu_r04p done"
