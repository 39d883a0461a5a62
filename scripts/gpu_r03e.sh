#!/bin/bash
# fp64 histogram: parity (default and always-split) + probe per split threshold
set -u
OUT=gpurun_out/r03e
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_f64.py > $OUT/f64_tests.log 2>&1 || { echo "f64 tests rc=$?"; tail -30 $OUT/f64_tests.log; exit 1; }
tail -1 $OUT/f64_tests.log
SBAG_F64_SPLIT=1000000000 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_f64.py > $OUT/f64_tests_split.log 2>&1 || { echo "f64 split tests rc=$?"; tail -30 $OUT/f64_tests_split.log; exit 1; }
tail -1 $OUT/f64_tests_split.log
for sp in ${SPLITS:-1024 1000000000}; do
  SBAG_F64_SPLIT=$sp SBAG_OVERLAP=0 SBAG_LEVEL_TRACE=1 timeout -k 10 300 python -u scripts/f64_probe.py > $OUT/probe_split$sp.log 2>&1 || { echo "probe rc=$?"; tail -20 $OUT/probe_split$sp.log; exit 1; }
  echo "split $sp"; grep "f64 level" $OUT/probe_split$sp.log | head -8 | tr '\n' ' '; echo; tail -1 $OUT/probe_split$sp.log
done
echo "gpu_r03e done"
