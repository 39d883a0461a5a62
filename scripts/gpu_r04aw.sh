#!/bin/bash
# k_fb_count pieces dispatched XCD-aware (row slice of each piece): A/B
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04aw}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_f64.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for o in 0 1; do
  SBAG_F64_XCD_ORDER=$o SBAG_OVERLAP=0 SBAG_LEVEL_TRACE=1 timeout -k 10 300 python -u scripts/f64_probe.py > $OUT/probe_o$o.log 2>&1 || { echo "probe rc=$?"; tail -30 $OUT/probe_o$o.log; exit 1; }
  echo "order=$o:"; grep 'ms: hist' $OUT/probe_o$o.log | tail -8 | cut -c1-120
  tail -1 $OUT/probe_o$o.log | cut -c1-200
done
SBAG_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ftrace -o trace -- python3 scripts/f64_probe.py > $OUT/ftrace.log 2>&1 || { echo "ftrace rc=$?"; tail -30 $OUT/ftrace.log; exit 1; }
f=$(find $OUT/ftrace -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/kernel_stats.csv; head -10 "$f" | cut -c1-140
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
echo "gpu_r04aw done"
