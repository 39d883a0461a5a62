#!/bin/bash
# exploded chains by default (width by wave count): f64 / gbm parity, GBM 10M + 1M, C3 nondyadic probe + trace
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04ak}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_f64.py tests/test_gpu_gbm.py tests/test_gpu_bench_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "f64 or gbm or booster or nondyadic or c3" > $OUT/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python3 -u scripts/bench_gbm.py --synthetic --rows 10000000 --features 100 --depth 5 --learners 5 > $OUT/bench_gbm_10m.log 2>&1 || { echo "gbm rc=$?"; tail -20 $OUT/bench_gbm_10m.log; exit 1; }
tail -1 $OUT/bench_gbm_10m.log
timeout -k 10 300 python3 -u scripts/bench_gbm.py > $OUT/bench_gbm.log 2>&1 || { echo "gbm rc=$?"; tail -20 $OUT/bench_gbm.log; exit 1; }
cat $OUT/bench_gbm.log | grep rows
SBAG_OVERLAP=0 SBAG_LEVEL_TRACE=1 timeout -k 10 300 python -u scripts/f64_probe.py > $OUT/probe.log 2>&1 || { echo "probe rc=$?"; tail -30 $OUT/probe.log; exit 1; }
grep 'ms: hist' $OUT/probe.log | tail -8 | cut -c1-120; tail -1 $OUT/probe.log | cut -c1-200
SBAG_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ftrace -o trace -- python3 scripts/f64_probe.py > $OUT/ftrace.log 2>&1 || { echo "ftrace rc=$?"; tail -30 $OUT/ftrace.log; exit 1; }
f=$(find $OUT/ftrace -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/kernel_stats.csv; head -8 "$f" | cut -c1-140
g=$(find $OUT/ftrace -name "*kernel_trace.csv" | head -1); python3 - "$g" > $OUT/fb_calls.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
for r in rows:
    n = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('sbag::', '')
    if 'k_fb' in n:
        print(f"{n[:24]:24s} {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6:8.2f}")
PY
rm -rf $OUT/ftrace
echo "gpu_r04ak done"
