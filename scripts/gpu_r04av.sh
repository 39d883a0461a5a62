#!/bin/bash
# gap sampler tail fix: regression seeds, split-sample / GBM parity, then the fuzz again
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04av}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_random.py tests/test_gpu_gbm.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "sample or split or gbm or booster or gap" > $OUT/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 420 python3 -u scripts/fuzz_parity.py --minutes 5 --start 81000 > $OUT/fuzz.log 2>&1 || { echo "fuzz rc=$?"; grep -v "^ok" $OUT/fuzz.log | head -20 | cut -c1-250; tail -2 $OUT/fuzz.log; exit 1; }
tail -1 $OUT/fuzz.log
timeout -k 10 300 python3 -u scripts/fuzz_parity.py --minutes 3 --start 82000 --booster > $OUT/fuzz_booster.log 2>&1 || { echo "fuzz booster rc=$?"; grep -v "^ok" $OUT/fuzz_booster.log | head -20 | cut -c1-250; exit 1; }
tail -1 $OUT/fuzz_booster.log
timeout -k 10 300 python3 -u scripts/fuzz_parity.py --minutes 2 --start 83000 --big > $OUT/fuzz_big.log 2>&1 || { echo "fuzz big rc=$?"; grep -v "^ok" $OUT/fuzz_big.log | head -20 | cut -c1-250; exit 1; }
tail -1 $OUT/fuzz_big.log
echo "gpu_r04av done"
