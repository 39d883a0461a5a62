#!/bin/bash
# MFMA root with XCD-aware work order: parity, C3 bench, C4 bench (root ms)
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04ad}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma_root.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 400 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-nondyadic > $OUT/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3', d['ms_per_step'], d['roofline']['root_mfma']['frac'], d['roofline']['root_mfma']['ms_per_fit'])"
timeout -k 10 600 python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline --no-nondyadic > $OUT/bench_c4.log 2>&1 || { echo "bench c4 rc=$?"; tail -20 $OUT/bench_c4.log; exit 1; }
tail -1 $OUT/bench_c4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', d['ms_per_step'], d['roofline']['root_mfma']['frac'], d['roofline']['root_mfma']['ms_per_fit'])"
echo "gpu_r04ad done"
