#!/bin/bash
# issue / wait breakdown per kernel of one serialized fit (W=c3/c4/c5, default c5)
set -u
OUT=gpurun_out/$1; shift
mkdir -p $OUT
export TMPDIR=/tmp SBAG_OVERLAP=0
BENCH="python3 bench.py --workload ${W:-c5} --steps 1 --warmup 0 --no-cpu-baseline --sampler-partitions 128"

timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS --output-format csv -d $OUT/sq -o sq -- $BENCH > $OUT/sq.log 2>&1 || { echo "pmc sq failed rc=$?"; exit 1; }
echo "pmc_c5 done"
