#!/bin/bash
# C3-sized fit on continuous features (per-replica binning at scale)
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04bb}
mkdir -p $OUT
timeout -k 10 900 python3 -u scripts/bench_continuous.py > $OUT/bench_continuous.log 2>&1 || { echo "rc=$?"; tail -20 $OUT/bench_continuous.log; exit 1; }
tail -3 $OUT/bench_continuous.log
echo "gpu_r04bb done"
