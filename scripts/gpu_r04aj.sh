#!/bin/bash
# exploded chains with ballot prefix sums: parity for each width, GBM 10M, C3 nondyadic by width
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04aj}
mkdir -p $OUT
for c in 16 4 1; do
  SBAG_F64_CHAIN_X=1 SBAG_F64_CHAIN_C=$c timeout -k 10 600 python -u -m pytest tests/test_gpu_f64.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_c$c.log 2>&1 || { echo "tests c=$c rc=$?"; tail -60 $OUT/gpu_tests_c$c.log; exit 1; }
  echo "C=$c"; tail -1 $OUT/gpu_tests_c$c.log
done
SBAG_F64_CHAIN_X=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_gbm.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_gbm.log 2>&1 || { echo "gbm tests rc=$?"; tail -60 $OUT/gpu_tests_gbm.log; exit 1; }
tail -1 $OUT/gpu_tests_gbm.log
SBAG_F64_CHAIN_X=1 timeout -k 10 300 python3 -u scripts/bench_gbm.py --synthetic --rows 10000000 --features 100 --depth 5 --learners 5 > $OUT/gbm10m_x1.log 2>&1 || { echo "gbm rc=$?"; tail -20 $OUT/gbm10m_x1.log; exit 1; }
tail -1 $OUT/gbm10m_x1.log
for c in 16 4; do
  SBAG_F64_CHAIN_X=1 SBAG_F64_CHAIN_C=$c SBAG_OVERLAP=0 SBAG_LEVEL_TRACE=1 timeout -k 10 300 python -u scripts/f64_probe.py > $OUT/probe_c$c.log 2>&1 || { echo "probe rc=$?"; tail -30 $OUT/probe_c$c.log; exit 1; }
  echo "C=$c:"; grep 'ms: hist' $OUT/probe_c$c.log | tail -8 | cut -c1-120
  tail -1 $OUT/probe_c$c.log | cut -c1-200
done
echo "gpu_r04aj done"
