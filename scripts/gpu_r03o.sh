#!/bin/bash
# C5 histogram ablation per level (SBAG_HIST_ABLATE relaunches, timing only)
set -u
OUT=gpurun_out/r03o
mkdir -p $OUT
for v in 4096; do
SBAG_HIST_SMALL=$v SBAG_OVERLAP=0 SBAG_LEVEL_TRACE=1 SBAG_HIST_ABLATE=1 timeout -k 10 300 python -u bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline --no-nondyadic > $OUT/c5_ablate_small$v.log 2>&1 || { echo "c5 ablate rc=$?"; tail -20 $OUT/c5_ablate_small$v.log; exit 1; }
done
echo "gpu_r03o done"
