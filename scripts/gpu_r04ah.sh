#!/bin/bash
# fp64 chains with the draws exploded in LDS (k_fb_chainx, SBAG_F64_CHAIN_X=1): parity, then
# A/B on the GBM 10M line and the C3 nondyadic fit (serialized, level trace)
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04ah}
mkdir -p $OUT
SBAG_F64_CHAIN_X=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_f64.py tests/test_gpu_gbm.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_x.log 2>&1 || { echo "tests rc=$?"; tail -60 $OUT/gpu_tests_x.log; exit 1; }
tail -2 $OUT/gpu_tests_x.log
for x in 0 1; do
  SBAG_F64_CHAIN_X=$x timeout -k 10 300 python3 -u scripts/bench_gbm.py --synthetic --rows 10000000 --features 100 --depth 5 --learners 5 > $OUT/gbm10m_x$x.log 2>&1 || { echo "gbm rc=$?"; tail -20 $OUT/gbm10m_x$x.log; exit 1; }
  echo "X=$x"; tail -1 $OUT/gbm10m_x$x.log
done
for x in 0 1; do
  SBAG_F64_CHAIN_X=$x SBAG_OVERLAP=0 SBAG_LEVEL_TRACE=1 timeout -k 10 300 python -u scripts/f64_probe.py > $OUT/probe_x$x.log 2>&1 || { echo "probe rc=$?"; tail -30 $OUT/probe_x$x.log; exit 1; }
  echo "X=$x:"; grep 'ms: hist' $OUT/probe_x$x.log | tail -8 | cut -c1-120
  tail -1 $OUT/probe_x$x.log | cut -c1-300
done
echo "gpu_r04ah done"
