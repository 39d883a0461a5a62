#!/bin/bash
# full GPU suite at HEAD
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04z}
mkdir -p $OUT
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
echo "gpu_r04z done"
