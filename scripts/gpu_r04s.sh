#!/bin/bash
# fp64 exact fallback restricted to the screen's contender features; C3 + C4 nondyadic
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04s}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_f64.py tests/test_gpu_gbm.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
SBAG_OVERLAP=0 SBAG_LEVEL_TRACE=1 timeout -k 10 300 python -u scripts/f64_probe.py > $OUT/probe_trace.log 2>&1 || { echo "probe rc=$?"; tail -30 $OUT/probe_trace.log; exit 1; }
grep "ms: hist\|fit_ms" $OUT/probe_trace.log | tail -10
timeout -k 10 300 python -u scripts/f64_probe.py > $OUT/probe.log 2>&1 || { echo "probe rc=$?"; tail -30 $OUT/probe.log; exit 1; }
echo "overlapped: $(tail -1 $OUT/probe.log)"
timeout -k 10 600 python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_c4.log 2>&1 || { echo "bench c4 rc=$?"; tail -20 $OUT/bench_c4.log; exit 1; }
tail -1 $OUT/bench_c4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('root_mfma')); print(d['nondyadic_labels'])"
echo "gpu_r04s done"
