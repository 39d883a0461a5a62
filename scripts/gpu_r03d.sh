#!/bin/bash
# fp64-label probe: FPW 64 and 32, serialized halves, per-level trace
set -u
OUT=gpurun_out/r03d
mkdir -p $OUT
for fpw in 64 32; do
  SBAG_F64_FPW=$fpw SBAG_OVERLAP=0 SBAG_LEVEL_TRACE=1 timeout -k 10 300 python -u scripts/f64_probe.py > $OUT/f64_fpw$fpw.log 2>&1 || { echo "probe fpw $fpw rc=$?"; tail -20 $OUT/f64_fpw$fpw.log; exit 1; }
  echo "fpw $fpw"; grep "level" $OUT/f64_fpw$fpw.log | tail -10; tail -1 $OUT/f64_fpw$fpw.log
done
echo "gpu_r03d done"
