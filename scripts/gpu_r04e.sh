#!/bin/bash
# Booster through the screened engine: GBM parity + C driver, GBM bench A/B, fp64 profile
set -u
OUT=gpurun_out/${RUN:-r04e}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gbm.py tests/test_gpu_c_abi.py tests/test_gpu_f64.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -u scripts/bench_gbm.py > $OUT/bench_gbm.log 2>&1 || { echo "bench_gbm rc=$?"; tail -20 $OUT/bench_gbm.log; exit 1; }
cat $OUT/bench_gbm.log
SBAG_BOOSTER_ENGINE=bt timeout -k 10 300 python -u scripts/bench_gbm.py > $OUT/bench_gbm_bt.log 2>&1 || { echo "bench_gbm bt rc=$?"; tail -20 $OUT/bench_gbm_bt.log; exit 1; }
cat $OUT/bench_gbm_bt.log
SBAG_OVERLAP=0 SBAG_LEVEL_TRACE=1 timeout -k 10 300 python -u scripts/f64_probe.py > $OUT/probe_trace.log 2>&1 || { echo "probe rc=$?"; tail -30 $OUT/probe_trace.log; exit 1; }
grep "f64 level\|fit_ms" $OUT/probe_trace.log | tail -12
SBAG_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 scripts/f64_probe.py > $OUT/trace.log 2>&1 || { echo "trace rc=$?"; tail -30 $OUT/trace.log; exit 1; }
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1); head -24 "$f" | cut -c1-200
echo "gpu_r04e done"
