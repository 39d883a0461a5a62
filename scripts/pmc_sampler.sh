#!/bin/bash
# PMC pass over the Poisson sampler alone (scripts/bench_sampler.py, C3 shape).
# usage: scripts/pmc_sampler.sh <tag> [env assignments...]
set -u
TAG=$1; shift
OUT=gpurun_out/pmc_sampler_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for kv in "$@"; do export "$kv"; done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 scripts/bench_sampler.py --reps 2 > $OUT/trace.log 2>&1 || { echo "trace failed rc=$?"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/sq -o sq -- python3 scripts/bench_sampler.py --reps 1 > $OUT/sq.log 2>&1 || { echo "pmc sq failed rc=$?"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_WAIT_ANY --output-format csv -d $OUT/sq2 -o sq2 -- python3 scripts/bench_sampler.py --reps 1 > $OUT/sq2.log 2>&1 || { echo "pmc sq2 failed rc=$?"; exit 1; }
echo "pmc_sampler $TAG done"
