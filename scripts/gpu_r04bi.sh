#!/bin/bash
# bin materialization with several replicas per workgroup (SBAG_MATERIALIZE_RB): parity at
# RB=4, continuous fit at RB = 1, 2, 4
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04bi}
mkdir -p $OUT
SBAG_MATERIALIZE_RB=4 timeout -k 10 900 python -u -m pytest tests/test_gpu_random.py tests/test_gpu_parity.py tests/test_gpu_ingest.py -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for rb in 1 2 4; do
  SBAG_MATERIALIZE_RB=$rb timeout -k 10 600 python3 -u scripts/bench_continuous.py > $OUT/bench_continuous_rb$rb.log 2>&1 || { echo "rc=$?"; tail -20 $OUT/bench_continuous_rb$rb.log; exit 1; }
  echo "rb=$rb $(tail -1 $OUT/bench_continuous_rb$rb.log | cut -c150-260)"
done
echo "gpu_r04bi done"
