#!/bin/bash
# chainx double-buffered stages; gap sampler loads kept in flight (raw ring, unrolled chunk loop, rows buffered in LDS);
# fp64 suite incl. the full-size engines-agree test; split-sample parity; GBM lines
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04az}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_f64.py tests/test_gpu_gbm.py tests/test_gpu_random.py tests/test_gpu_parity.py -m gpu -x -q --timeout 400 --timeout-method thread -k "f64 or nondyadic or sample or split or gbm or booster or gap" > $OUT/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python3 -u scripts/bench_gbm.py --synthetic --rows 10000000 --features 100 --depth 5 --learners 5 > $OUT/bench_gbm_10m.log 2>&1 || { echo "gbm rc=$?"; tail -20 $OUT/bench_gbm_10m.log; exit 1; }
tail -1 $OUT/bench_gbm_10m.log
timeout -k 10 300 python3 -u scripts/bench_gbm.py > $OUT/bench_gbm.log 2>&1 || { echo "gbm rc=$?"; tail -20 $OUT/bench_gbm.log; exit 1; }
grep rows $OUT/bench_gbm.log
echo "gpu_r04az done"
SBAG_OVERLAP=0 SBAG_LEVEL_TRACE=1 timeout -k 10 300 python -u scripts/f64_probe.py > $OUT/probe.log 2>&1 || { echo "probe rc=$?"; tail -30 $OUT/probe.log; exit 1; }
grep 'ms: hist' $OUT/probe.log | tail -8 | cut -c1-120; tail -1 $OUT/probe.log | cut -c1-200
echo "gpu_r04az probe done"
