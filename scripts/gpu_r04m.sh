#!/bin/bash
# Packed per-replica rows for subspace histograms: parity A/B, C5 bench A/B, C5 kernel trace
set -u
OUT=gpurun_out/${RUN:-r04m}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_packed_rows.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_c5.log 2>&1 || { echo "bench c5 rc=$?"; tail -20 $OUT/bench_c5.log; exit 1; }
tail -1 $OUT/bench_c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5', d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('avg_launch_ms'), d['breakdown_ms'])"
SBAG_PACK_ROWS=0 timeout -k 10 300 python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_c5_nopack.log 2>&1 || { echo "bench c5 nopack rc=$?"; tail -20 $OUT/bench_c5_nopack.log; exit 1; }
tail -1 $OUT/bench_c5_nopack.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 nopack', d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('avg_launch_ms'), d['breakdown_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/trace.log 2>&1 || { echo "trace rc=$?"; tail -30 $OUT/trace.log; exit 1; }
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1); head -14 "$f" | cut -c1-200
echo "gpu_r04m done"
