#!/bin/bash
set -u
OUT=gpurun_out/${RUN:-r04h}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random.py tests/test_gpu_gbm.py -m gpu -x -q --timeout 300 --timeout-method thread -k "sampled or split_sample or gbm or booster or max_bins" > $OUT/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
RUN=${RUN:-r04h}_f64 bash scripts/gpu_f64prof.sh || exit 1
RUN=${RUN:-r04h}_gbm bash scripts/gpu_gbmprof.sh || exit 1
