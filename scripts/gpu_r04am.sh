#!/bin/bash
# fp64 bucket scatter staged by bin in LDS (coalesced bucket stores): parity, A/B on the
# C3 nondyadic fit (serialized) and the GBM 10M line
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04am}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_f64.py tests/test_gpu_gbm.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for st in 0 1; do
  SBAG_F64_SCATTER_STAGE=$st SBAG_OVERLAP=0 SBAG_LEVEL_TRACE=1 timeout -k 10 300 python -u scripts/f64_probe.py > $OUT/probe_s$st.log 2>&1 || { echo "probe rc=$?"; tail -30 $OUT/probe_s$st.log; exit 1; }
  echo "stage=$st:"; grep 'ms: hist' $OUT/probe_s$st.log | tail -8 | cut -c1-120
  tail -1 $OUT/probe_s$st.log | cut -c1-200
done
timeout -k 10 300 python3 -u scripts/bench_gbm.py --synthetic --rows 10000000 --features 100 --depth 5 --learners 5 > $OUT/bench_gbm_10m.log 2>&1 || { echo "gbm rc=$?"; tail -20 $OUT/bench_gbm_10m.log; exit 1; }
tail -1 $OUT/bench_gbm_10m.log
SBAG_OVERLAP=0 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 scripts/f64_probe.py > $OUT/write.log 2>&1 || { echo "pmc write failed rc=$?"; tail -20 $OUT/write.log; exit 1; }
echo "gpu_r04am done"
