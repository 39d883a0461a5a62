#!/bin/bash
# GPU suite, then C3 (with the non-dyadic timing) and C5 benches at HEAD.  First failure ends it.
set -u
OUT=gpurun_out/r03f
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_c3.log 2>&1 || { echo "bench c3 rc=$?"; tail -20 $OUT/bench_c3.log; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_c3.log').read().strip().splitlines()[-1]); print('c3', d['ms_per_step'], d['value'], 'nondyadic', d['nondyadic_labels']['ms_per_step'], d['nondyadic_labels']['breakdown_ms'])"
timeout -k 10 400 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_c5.log 2>&1 || { echo "bench c5 rc=$?"; tail -20 $OUT/bench_c5.log; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_c5.log').read().strip().splitlines()[-1]); print('c5', d['ms_per_step'], d['value'], d['breakdown_ms'])"
echo "gpu_r03f done"
