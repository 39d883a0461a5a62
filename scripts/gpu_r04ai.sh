#!/bin/bash
# C3 nondyadic fit kernel trace with the exploded chains (k_fb_chainx)
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04ai}
mkdir -p $OUT
SBAG_F64_CHAIN_X=1 SBAG_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ftrace -o trace -- python3 scripts/f64_probe.py > $OUT/ftrace.log 2>&1 || { echo "ftrace rc=$?"; tail -30 $OUT/ftrace.log; exit 1; }
f=$(find $OUT/ftrace -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/kernel_stats.csv; head -12 "$f" | cut -c1-160
g=$(find $OUT/ftrace -name "*kernel_trace.csv" | head -1); python3 - "$g" > $OUT/chain_calls.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
for r in rows:
    n = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('sbag::', '')
    if 'k_fb' in n:
        print(f"{n[:24]:24s} {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6:8.2f}")
PY
head -60 $OUT/chain_calls.txt
echo "gpu_r04ai done"
