#!/bin/bash
# GPU suite, the default bench line, then the C3 profile (trace + PMC passes) at HEAD.
# First failure ends it.
set -u
OUT=gpurun_out/r03g
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > $OUT/bench_c3.log 2>&1 || { echo "bench c3 rc=$?"; tail -20 $OUT/bench_c3.log; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_c3.log').read().strip().splitlines()[-1]); print('c3', d['ms_per_step'], d['value'], d['roofline']['frac'], d['breakdown_ms'])"
bash scripts/profile.sh r03g_c3 --no-nondyadic || exit 1
echo "gpu_r03g done"
