#!/bin/bash
# GPU suite, default bench (C3), C4 and C5 shard benches at HEAD.  First failure ends it.
set -u
OUT=gpurun_out/r03l
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -k "poisson or bernoulli" --timeout 120 --timeout-method thread > $OUT/sampler_tests.log 2>&1 || { echo "sampler rc=$?"; tail -30 $OUT/sampler_tests.log; exit 1; }
tail -1 $OUT/sampler_tests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > $OUT/bench_c3.log 2>&1 || { echo "bench c3 rc=$?"; tail -20 $OUT/bench_c3.log; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_c3.log').read().strip().splitlines()[-1]); print('c3', d['ms_per_step'], d['value'], d['roofline']['frac'], d['breakdown_ms']['sample_ms'], d['sampler_at_nproc_partitions'], d['nondyadic_labels']['ms_per_step'])"
timeout -k 10 400 python -u bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_c4.log 2>&1 || { echo "bench c4 rc=$?"; tail -20 $OUT/bench_c4.log; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_c4.log').read().strip().splitlines()[-1]); print('c4', d['ms_per_step'], d['value'], d['breakdown_ms'])"
timeout -k 10 400 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_c5.log 2>&1 || { echo "bench c5 rc=$?"; tail -20 $OUT/bench_c5.log; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_c5.log').read().strip().splitlines()[-1]); print('c5', d['ms_per_step'], d['value'], d['breakdown_ms'])"
echo "gpu_r03l done"
