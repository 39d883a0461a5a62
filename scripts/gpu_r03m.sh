#!/bin/bash
# C5 per-level trace (histogram launches and per-level stage ms), serialized halves
set -u
OUT=gpurun_out/r03m
mkdir -p $OUT
SBAG_OVERLAP=0 SBAG_LEVEL_TRACE=1 SBAG_PROFILE_HOST=1 timeout -k 10 300 python -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/c5_trace.log 2>&1 || { echo "c5 trace rc=$?"; tail -20 $OUT/c5_trace.log; exit 1; }
grep -c sbag $OUT/c5_trace.log
echo "gpu_r03m done"
