#!/bin/bash
# Profile the C3 bench on the GPU box: kernel trace + separate PMC passes
# (FETCH_SIZE, WRITE_SIZE and the LDS counters each in their own run, never with
# a trace domain).  Summarise afterwards with scripts/pmc_summary.py.
# usage: scripts/profile.sh <tag> [bench args...]
set -u
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
# kernel durations of each launch alone (the bench's roofline fit does the same)
export SBAG_OVERLAP=0
BENCH="python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-continuous --sampler-partitions 128 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- $BENCH > $OUT/trace.log 2>&1 || { echo "trace failed rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- $BENCH > $OUT/fetch.log 2>&1 || { echo "pmc fetch failed rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- $BENCH > $OUT/write.log 2>&1 || { echo "pmc write failed rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS --output-format csv -d $OUT/lds -o lds -- $BENCH > $OUT/lds.log 2>&1 || { echo "pmc lds failed rc=$?"; exit 1; }
echo "profile $TAG done"
