#!/bin/bash
# SQ counters of the fp64 engine's kernels (C3 nondyadic, serialized): issue vs waits
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04ao}
mkdir -p $OUT
export SBAG_OVERLAP=0
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/sq -o sq -- python3 scripts/f64_probe.py > $OUT/sq.log 2>&1 || { echo "pmc sq failed rc=$?"; tail -20 $OUT/sq.log; exit 1; }
echo "gpu_r04ao done"
