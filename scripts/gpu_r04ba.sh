#!/bin/bash
# chainx: one buffer ahead vs two fixed buffers (SBAG_F64_CHAIN_DB), same box
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04ba}
mkdir -p $OUT
SBAG_F64_CHAIN_DB=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_f64.py -m gpu -x -q --timeout 400 --timeout-method thread -k "not full" > $OUT/gpu_tests_db.log 2>&1 || { echo "tests rc=$?"; tail -60 $OUT/gpu_tests_db.log; exit 1; }
tail -1 $OUT/gpu_tests_db.log
for db in 0 1 0 1; do
  SBAG_F64_CHAIN_DB=$db SBAG_OVERLAP=0 SBAG_LEVEL_TRACE=1 timeout -k 10 300 python -u scripts/f64_probe.py > $OUT/probe_db$db.log 2>&1 || { echo "probe rc=$?"; tail -30 $OUT/probe_db$db.log; exit 1; }
  echo "db=$db: $(grep 'level 0 ms' $OUT/probe_db$db.log | cut -c1-90) | $(grep 'level 5 ms' $OUT/probe_db$db.log | cut -c20-90)"
  tail -1 $OUT/probe_db$db.log | cut -c1-90
done
echo "gpu_r04ba done"
