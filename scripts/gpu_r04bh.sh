#!/bin/bash
# per-replica bins by code cuts searched in LDS: parity, then the continuous fit (cuts / LUT)
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04bh}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_random.py tests/test_gpu_parity.py tests/test_gpu_f64.py tests/test_gpu_gbm.py tests/test_gpu_ingest.py -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 600 python3 -u scripts/bench_continuous.py > $OUT/bench_continuous.log 2>&1 || { echo "rc=$?"; tail -20 $OUT/bench_continuous.log; exit 1; }
tail -1 $OUT/bench_continuous.log
SBAG_MATERIALIZE_LUT=1 timeout -k 10 600 python3 -u scripts/bench_continuous.py > $OUT/bench_continuous_lut.log 2>&1 || { echo "rc=$?"; tail -20 $OUT/bench_continuous_lut.log; exit 1; }
tail -1 $OUT/bench_continuous_lut.log | cut -c1-260
timeout -k 10 300 python3 -u scripts/fuzz_parity.py --minutes 3 --start 93000 > $OUT/fuzz.log 2>&1 || { echo "fuzz rc=$?"; grep -v "^ok" $OUT/fuzz.log | head -20 | cut -c1-250; exit 1; }
tail -1 $OUT/fuzz.log
echo "gpu_r04bh done"
