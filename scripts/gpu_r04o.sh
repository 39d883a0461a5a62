#!/bin/bash
# fp64: bins saved by the count pass; then HEAD profiles (C3, C4) for bench.py's traffic
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04o}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_f64.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
SBAG_OVERLAP=0 SBAG_LEVEL_TRACE=1 timeout -k 10 300 python -u scripts/f64_probe.py > $OUT/probe_trace.log 2>&1 || { echo "probe rc=$?"; tail -30 $OUT/probe_trace.log; exit 1; }
grep "ms: hist\|fit_ms" $OUT/probe_trace.log | tail -10
timeout -k 10 300 python -u scripts/f64_probe.py > $OUT/probe.log 2>&1 || { echo "probe rc=$?"; tail -30 $OUT/probe.log; exit 1; }
echo "overlapped: $(tail -1 $OUT/probe.log)"
RUN=${RUN:-r04o} bash scripts/gpu_r04n.sh || exit 1
echo "gpu_r04o done"
