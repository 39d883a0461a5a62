#!/bin/bash
# Round 4, first pass: the multi-rank bench rehearsal (2 ranks, gloo, one GPU), the full-size
# C4 / C5 shard tests, then the default bench line.
set -u
OUT=gpurun_out/r04a
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench_multirank.py tests/test_gpu_bench_configs.py -m gpu -x -v --timeout 600 --timeout-method thread -k "multirank or full_shard or two_ranks" > $OUT/gpu_new_tests.log 2>&1 || { echo "new tests rc=$?"; tail -60 $OUT/gpu_new_tests.log; exit 1; }
tail -5 $OUT/gpu_new_tests.log
timeout -k 10 300 python -u bench.py > $OUT/bench_default.log 2>&1 || { echo "bench default rc=$?"; tail -20 $OUT/bench_default.log; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_default.log').read().strip().splitlines()[-1]); print('default', d['ms_per_step'], d['value'], d['roofline']['frac'], d['breakdown_ms']['sample_ms'], d['nondyadic_labels']['ms_per_step'])"
echo "gpu_r04a done"
