#!/bin/bash
# gap sampler over several waves per (replica, partition): parity, fuzz, GBM lines
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04bm}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_gbm.py tests/test_gpu_random.py tests/test_gpu_parity.py tests/test_gpu_f64.py -m gpu -x -q --timeout 400 --timeout-method thread -k "sample or split or gbm or booster or gap or nondyadic or f64" > $OUT/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 200 python3 -u scripts/fuzz_parity.py --minutes 2 --start 97000 --booster > $OUT/fuzz_booster.log 2>&1 || { echo "fuzz booster rc=$?"; grep -v "^ok" $OUT/fuzz_booster.log | head -20 | cut -c1-250; exit 1; }
tail -1 $OUT/fuzz_booster.log
timeout -k 10 200 python3 -u scripts/fuzz_parity.py --minutes 2 --start 98000 > $OUT/fuzz.log 2>&1 || { echo "fuzz rc=$?"; grep -v "^ok" $OUT/fuzz.log | head -20 | cut -c1-250; exit 1; }
tail -1 $OUT/fuzz.log
timeout -k 10 300 python3 -u scripts/bench_gbm.py --synthetic --rows 10000000 --features 100 --depth 5 --learners 5 > $OUT/bench_gbm_10m.log 2>&1 || { echo "gbm rc=$?"; tail -20 $OUT/bench_gbm_10m.log; exit 1; }
tail -1 $OUT/bench_gbm_10m.log
timeout -k 10 300 python3 -u scripts/bench_gbm.py > $OUT/bench_gbm.log 2>&1 || { echo "gbm rc=$?"; tail -20 $OUT/bench_gbm.log; exit 1; }
grep rows $OUT/bench_gbm.log
echo "gpu_r04bm done"
