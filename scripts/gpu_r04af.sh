#!/bin/bash
# gap sampler: 4096-row chunks in aligned 16-byte loads; split-sample / GBM parity; GBM benches
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04af}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random.py tests/test_gpu_gbm.py tests/test_gpu_f64.py -m gpu -x -q --timeout 300 --timeout-method thread -k "sample or split or gbm or booster or partition or f64 or nondyadic" > $OUT/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 400 python3 -u scripts/bench_gbm.py --synthetic --rows 10000000 --features 100 --depth 5 --learners 5 > $OUT/bench_gbm_10m.log 2>&1 || { echo "gbm10m rc=$?"; tail -20 $OUT/bench_gbm_10m.log; exit 1; }
cat $OUT/bench_gbm_10m.log
timeout -k 10 300 python3 -u scripts/bench_gbm.py > $OUT/bench_gbm.log 2>&1 || { echo "gbm rc=$?"; tail -20 $OUT/bench_gbm.log; exit 1; }
cat $OUT/bench_gbm.log
echo "gpu_r04af done"
