#!/bin/bash
# gap sampler resolving a chunk's items in parallel: split-sample parity, GBM lines
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04as}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_gbm.py tests/test_gpu_random.py tests/test_gpu_parity.py -m gpu -x -q -k "sample or split or gbm or booster" --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
SBAG_PROFILE_HOST=1 timeout -k 10 300 python3 -u scripts/bench_gbm.py --synthetic --rows 10000000 --features 100 --depth 5 --learners 5 > $OUT/bench_gbm_10m.log 2>&1 || { echo "gbm rc=$?"; tail -20 $OUT/bench_gbm_10m.log; exit 1; }
grep "booster host" $OUT/bench_gbm_10m.log | tail -2; tail -1 $OUT/bench_gbm_10m.log
timeout -k 10 300 python3 -u scripts/bench_gbm.py > $OUT/bench_gbm.log 2>&1 || { echo "gbm rc=$?"; tail -20 $OUT/bench_gbm.log; exit 1; }
grep rows $OUT/bench_gbm.log
echo "gpu_r04as done"
