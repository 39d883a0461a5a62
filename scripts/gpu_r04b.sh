#!/bin/bash
# Round 4: the screened fp64 engine -- parity first (small), then the C3-shape nondyadic
# line, then the bench.
set -u
OUT=gpurun_out/${RUN:-r04b}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_f64.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_f64.log 2>&1 || { echo "f64 tests rc=$?"; tail -60 $OUT/gpu_f64.log; exit 1; }
tail -3 $OUT/gpu_f64.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_configs.py -m gpu -x -v -s --timeout 500 --timeout-method thread -k nondyadic > $OUT/gpu_c3_f64.log 2>&1 || { echo "c3 f64 rc=$?"; tail -60 $OUT/gpu_c3_f64.log; exit 1; }
grep -E "c3 nondyadic|passed|failed" $OUT/gpu_c3_f64.log
SBAG_LEVEL_TRACE=1 timeout -k 10 300 python -u bench.py --steps 2 --no-cpu-baseline > $OUT/bench_default.log 2>&1 || { echo "bench rc=$?"; tail -30 $OUT/bench_default.log; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_default.log').read().strip().splitlines()[-1]); print('default', d['ms_per_step'], d['roofline']['frac'], 'nondyadic', d['nondyadic_labels']['ms_per_step'], d['nondyadic_labels']['breakdown_ms'])"
echo "gpu_r04b done"
