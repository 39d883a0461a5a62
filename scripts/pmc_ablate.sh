#!/bin/bash
# PMC counters of the histogram kernel per ablation mode (timing-only builds)
export TMPDIR=/tmp
for m in 0 2; do
  for grp in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES" "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU"; do
    tag=$(echo $grp | cut -d' ' -f1)
    OUT=gpurun_out/pmc/m${m}_$tag; mkdir -p $OUT
    SBAG_HIST_ABLATE=$m timeout -k 10 200 rocprofv3 --pmc $grp --output-format csv -d $OUT -o p -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --depth 1 > $OUT/log 2>&1 || { echo "mode $m $tag failed"; tail -5 $OUT/log; exit 1; }
  done
done
echo pmc done
