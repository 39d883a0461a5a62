#!/bin/bash
# fp64 chains: 64 per wave (k_fb_chain64) vs 16, C3 nondyadic serialized level trace; parity
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04y}
mkdir -p $OUT
SBAG_F64_CHAIN_C=64 timeout -k 10 600 python -u -m pytest tests/test_gpu_f64.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests64.log 2>&1 || { echo "tests rc=$?"; tail -60 $OUT/gpu_tests64.log; exit 1; }
tail -2 $OUT/gpu_tests64.log
for cw in 16 64; do
  SBAG_F64_CHAIN_C=$cw SBAG_OVERLAP=0 SBAG_LEVEL_TRACE=1 timeout -k 10 300 python -u scripts/f64_probe.py > $OUT/probe_c$cw.log 2>&1 || { echo "probe rc=$?"; tail -30 $OUT/probe_c$cw.log; exit 1; }
  echo "C=$cw:"; grep 'ms: hist' $OUT/probe_c$cw.log | tail -8 | cut -c1-100
  tail -1 $OUT/probe_c$cw.log | cut -c1-100
done
SBAG_F64_CHAIN_C=64 SBAG_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ftrace -o trace -- python3 scripts/f64_probe.py > $OUT/ftrace.log 2>&1 || { echo "ftrace rc=$?"; tail -30 $OUT/ftrace.log; exit 1; }
f=$(find $OUT/ftrace -name "*kernel_stats.csv" | head -1); head -8 "$f" | cut -c1-140
echo "gpu_r04y done"
