#!/bin/bash
# One GPU-box pass: headline bench, the C4/C5 shard benches and the C3 profile.
# usage: scripts/gpu_round.sh <tag>
set -u
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 240 python3 bench.py --steps 10 --warmup 2 > $OUT/bench_c3.log 2>&1 || { echo "bench c3 failed rc=$?"; exit 1; }
tail -1 $OUT/bench_c3.log
timeout -k 10 240 python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_c5.log 2>&1 || { echo "bench c5 failed rc=$?"; exit 1; }
timeout -k 10 300 python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_c4.log 2>&1 || { echo "bench c4 failed rc=$?"; exit 1; }
bash scripts/profile.sh ${TAG}_c3 || exit 1
echo "gpu_round $TAG done"
