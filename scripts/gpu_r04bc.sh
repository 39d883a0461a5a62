#!/bin/bash
# per-replica bins: coalesced materialization + up-front learner-range split; parity of the
# per-replica binning tests, then the C3-sized continuous fit
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04bc}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_random.py tests/test_gpu_parity.py tests/test_gpu_f64.py tests/test_gpu_bench_configs.py -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 900 python3 -u scripts/bench_continuous.py > $OUT/bench_continuous.log 2>&1 || { echo "rc=$?"; tail -20 $OUT/bench_continuous.log; exit 1; }
tail -1 $OUT/bench_continuous.log
echo "gpu_r04bc done"
