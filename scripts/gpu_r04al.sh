#!/bin/bash
# PMC traffic of the fp64 engine's kernels (C3 nondyadic fit, serialized): FETCH_SIZE and
# WRITE_SIZE passes, each alone
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04al}
mkdir -p $OUT
export SBAG_OVERLAP=0
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 scripts/f64_probe.py > $OUT/fetch.log 2>&1 || { echo "pmc fetch failed rc=$?"; tail -20 $OUT/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 scripts/f64_probe.py > $OUT/write.log 2>&1 || { echo "pmc write failed rc=$?"; tail -20 $OUT/write.log; exit 1; }
ls -R $OUT | head -20
echo "gpu_r04al done"
