#!/bin/bash
# fp64 engine: exact fallback split by node size (walk small flagged nodes, chain big ones)
set -u
OUT=gpurun_out/${RUN:-r04j}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_f64.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
SBAG_OVERLAP=0 SBAG_LEVEL_TRACE=1 timeout -k 10 300 python -u scripts/f64_probe.py > $OUT/probe_trace.log 2>&1 || { echo "probe rc=$?"; tail -30 $OUT/probe_trace.log; exit 1; }
grep "f64 level\|fit_ms" $OUT/probe_trace.log | tail -40
for m in default chain; do
  if [ $m = chain ]; then export SBAG_F64_FALLBACK=chain; fi
  SBAG_OVERLAP=0 timeout -k 10 300 python -u scripts/f64_probe.py > $OUT/probe_$m.log 2>&1 || { echo "probe $m rc=$?"; tail -30 $OUT/probe_$m.log; exit 1; }
  echo "$m: $(tail -1 $OUT/probe_$m.log)"
done
unset SBAG_F64_FALLBACK
timeout -k 10 300 python -u scripts/f64_probe.py > $OUT/probe.log 2>&1 || { echo "probe rc=$?"; tail -30 $OUT/probe.log; exit 1; }
echo "overlapped: $(tail -1 $OUT/probe.log)"
echo "gpu_r04j done"
