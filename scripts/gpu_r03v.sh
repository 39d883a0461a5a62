#!/bin/bash
# Barrier waits made explicit (block_sync): determinism of fuzz seed 50680, the GPU suite,
# a fuzz pass, default bench (C3) and the C5 shard.
set -u
OUT=gpurun_out/r03v
mkdir -p $OUT
timeout -k 10 300 python3 -u scripts/fuzz_determinism.py 50680 3 none > $OUT/det.log 2>&1 || { echo "det rc=$?"; tail -5 $OUT/det.log; exit 1; }
grep -v amdgpu.ids $OUT/det.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 420 python3 -u scripts/fuzz_parity.py --start 60000 --minutes 6 > $OUT/fuzz.log 2>&1; echo "fuzz rc=$?"; tail -1 $OUT/fuzz.log; grep FAIL $OUT/fuzz.log | head -5
timeout -k 10 300 python -u bench.py > $OUT/bench_default.log 2>&1 || { echo "bench default rc=$?"; tail -20 $OUT/bench_default.log; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_default.log').read().strip().splitlines()[-1]); print('default', d['ms_per_step'], d['value'], d['roofline']['frac'], d['breakdown_ms'])"
timeout -k 10 400 python -u bench.py --workload c5 --steps 4 --warmup 1 --no-cpu-baseline > $OUT/bench_c5.log 2>&1 || { echo "bench c5 rc=$?"; tail -20 $OUT/bench_c5.log; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_c5.log').read().strip().splitlines()[-1]); print('c5', d['ms_per_step'], d['value'], d['breakdown_ms'])"
echo "gpu_r03v done"
