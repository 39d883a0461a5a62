#!/bin/bash
# C3 PMC profile of the dyadic fits only (bench.py's traffic field)
set -u
export TMPDIR=/tmp
bash scripts/profile.sh ${RUN:-r04ac}_c3 --no-nondyadic || exit 1
echo "gpu_r04ac done"
