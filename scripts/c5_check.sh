#!/bin/bash
# C5 class-tile grouping: gini parity tests, then the C5 shard bench with and without
# grouping, then a C5 profile.  usage: scripts/c5_check.sh <tag>
set -u
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random.py tests/test_gpu_bench_configs.py -k "class or gini or random or c5 or vehicle or classif" -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 240 python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline --sampler-partitions 128 > $OUT/bench_c5.log 2>&1 || { echo "bench c5 failed rc=$?"; exit 1; }
SBAG_NO_TILE_GROUPING=1 timeout -k 10 240 python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline --sampler-partitions 128 > $OUT/bench_c5_nogroup.log 2>&1 || { echo "bench c5 nogroup failed rc=$?"; exit 1; }
SBAG_HIST_RL=0 timeout -k 10 240 python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline --sampler-partitions 128 > $OUT/bench_c5_norl.log 2>&1 || { echo "bench c5 norl failed rc=$?"; exit 1; }
bash scripts/profile.sh ${TAG}_c5 --workload c5 || exit 1
echo "c5_check $TAG done"
