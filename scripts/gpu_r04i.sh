#!/bin/bash
# MFMA root histogram parity + C3 bench A/B (k_hist_mfma vs k_hist_rl root), fp64 chain
# rework (labels gathered by the scatter), kernel trace of the default bench
set -u
OUT=gpurun_out/${RUN:-r04i}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma_root.py tests/test_gpu_f64.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > $OUT/bench.log 2>&1 || { echo "bench rc=$?"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-600
SBAG_ROOT_MFMA=0 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > $OUT/bench_lds.log 2>&1 || { echo "bench lds rc=$?"; tail -30 $OUT/bench_lds.log; exit 1; }
tail -1 $OUT/bench_lds.log | cut -c1-400
timeout -k 10 300 python -u scripts/f64_probe.py > $OUT/probe.log 2>&1 || { echo "probe rc=$?"; tail -30 $OUT/probe.log; exit 1; }
cat $OUT/probe.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 bench.py --steps 2 --warmup 1 > $OUT/trace.log 2>&1 || { echo "trace rc=$?"; tail -30 $OUT/trace.log; exit 1; }
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1); head -16 "$f" | cut -c1-200
SBAG_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ftrace -o trace -- python3 scripts/f64_probe.py > $OUT/ftrace.log 2>&1 || { echo "ftrace rc=$?"; tail -30 $OUT/ftrace.log; exit 1; }
f=$(find $OUT/ftrace -name "*kernel_stats.csv" | head -1); head -12 "$f" | cut -c1-200
echo "gpu_r04i done"
