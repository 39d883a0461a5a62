#!/bin/bash
# C4-shape fp64 probe: serialized with level trace, then default (halves as sbag_fit picks)
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04t}
mkdir -p $OUT
SBAG_OVERLAP=0 SBAG_LEVEL_TRACE=1 timeout -k 10 400 python -u scripts/f64_probe.py 100000000 64 256 > $OUT/probe_c4_trace.log 2>&1 || { echo "probe rc=$?"; tail -30 $OUT/probe_c4_trace.log; exit 1; }
grep "ms: hist\|fit_ms\|nodes.*flagged" $OUT/probe_c4_trace.log | tail -30
timeout -k 10 400 python -u scripts/f64_probe.py 100000000 64 256 > $OUT/probe_c4.log 2>&1 || { echo "probe rc=$?"; tail -30 $OUT/probe_c4.log; exit 1; }
echo "default: $(tail -1 $OUT/probe_c4.log)"
echo "gpu_r04t done"
