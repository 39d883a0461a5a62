#!/bin/bash
# Round-3 pass after the barrier fix: GPU suite, default bench (C3), C4 / C5 shard benches, C3 profile.
set -u
OUT=gpurun_out/r03y
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python -u bench.py > $OUT/bench_default.log 2>&1 || { echo "bench default rc=$?"; tail -20 $OUT/bench_default.log; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_default.log').read().strip().splitlines()[-1]); print('default', d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['lds_atomic']['frac'], d['breakdown_ms']['sample_ms'], d['cpu_baseline']['value'])"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-nondyadic > $OUT/bench_c3.log 2>&1 || { echo "bench c3 rc=$?"; tail -20 $OUT/bench_c3.log; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_c3.log').read().strip().splitlines()[-1]); print('c3x10', d['ms_per_step'], d['value'])"
timeout -k 10 400 python -u bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_c4.log 2>&1 || { echo "bench c4 rc=$?"; tail -20 $OUT/bench_c4.log; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_c4.log').read().strip().splitlines()[-1]); print('c4', d['ms_per_step'], d['value'], d['breakdown_ms']['hist_ms'])"
timeout -k 10 400 python -u bench.py --workload c5 --steps 6 --warmup 1 --no-cpu-baseline > $OUT/bench_c5.log 2>&1 || { echo "bench c5 rc=$?"; tail -20 $OUT/bench_c5.log; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_c5.log').read().strip().splitlines()[-1]); print('c5', d['ms_per_step'], d['value'], d['breakdown_ms']['hist_ms'])"
bash scripts/profile.sh r03y_c3 --no-nondyadic || exit 1
bash scripts/profile.sh r03y_c5 --workload c5 || exit 1
echo "gpu_r03y done"
