#!/bin/bash
# kernel trace only + per-dispatch listing: scripts/trace.sh <tag> [bench args]
TAG=$1; shift
OUT=gpurun_out/trace_$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o trace -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline "$@" > $OUT/trace.log 2>&1
rc=$?
python3 scripts/dispatches.py $OUT > $OUT/dispatches.txt 2>&1
echo "rc=$rc"
