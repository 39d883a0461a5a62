#!/bin/bash
# Kernel trace + SQ counter passes over the sampler alone (scripts/bench_sampler.py).
# usage: scripts/profile_sampler.sh <tag> [bench_sampler args...]
set -u
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python3 scripts/bench_sampler.py --reps 1 $*"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- $CMD > $OUT/trace.log 2>&1 || { echo "trace failed rc=$?"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU --output-format csv -d $OUT/sq -o sq -- $CMD > $OUT/sq.log 2>&1 || { echo "pmc sq failed rc=$?"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_WAVES --output-format csv -d $OUT/lds -o lds -- $CMD > $OUT/lds.log 2>&1 || { echo "pmc lds failed rc=$?"; exit 1; }
echo "profile_sampler $TAG done"
