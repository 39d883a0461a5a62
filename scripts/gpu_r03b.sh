#!/bin/bash
# Round 3 GPU pass: two-rank test, C3 bench (with the non-dyadic timing), C4 shard with the
# learner halves overlapped, C5 level trace.  Every GPU step has its own time limit; the
# first failure ends the script.
set -u
OUT=gpurun_out/r03b
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $OUT/gpu_dist.log 2>&1 || { echo "dist test rc=$?"; tail -30 $OUT/gpu_dist.log; exit 1; }
tail -3 $OUT/gpu_dist.log
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 > $OUT/bench_c3.log 2>&1 || { echo "bench c3 rc=$?"; tail -20 $OUT/bench_c3.log; exit 1; }
tail -c 2500 $OUT/bench_c3.log; echo
SBAG_OVERLAP=2 timeout -k 10 400 python -u bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline --no-nondyadic > $OUT/bench_c4_overlap.log 2>&1 || { echo "bench c4 overlap rc=$?"; tail -20 $OUT/bench_c4_overlap.log; exit 1; }
python3 -c "import json,sys; d=json.loads(open('$OUT/bench_c4_overlap.log').read().strip().splitlines()[-1]); print('c4 overlap ms/step', d['ms_per_step'], d['breakdown_ms'])"
SBAG_LEVEL_TRACE=1 SBAG_OVERLAP=0 timeout -k 10 300 python -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/bench_c5_trace.log 2>&1 || { echo "bench c5 rc=$?"; tail -20 $OUT/bench_c5_trace.log; exit 1; }
grep "level .* ms:" $OUT/bench_c5_trace.log | tail -14
echo "gpu_r03b done"
