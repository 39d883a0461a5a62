#!/bin/bash
# default bench (C3 + nondyadic line), GBM at 10M x 100, fp64/booster fuzz parity
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04r}
mkdir -p $OUT
timeout -k 10 400 python3 bench.py > $OUT/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline'].get('root_mfma'), d['nondyadic_labels']['ms_per_step'], d['nondyadic_labels']['exact_fallbacks'], d['cpu_baseline'])"
timeout -k 10 400 python3 -u scripts/bench_gbm.py --synthetic --rows 10000000 --features 100 --depth 5 --learners 10 > $OUT/bench_gbm_10m.log 2>&1 || { echo "gbm10m rc=$?"; tail -20 $OUT/bench_gbm_10m.log; exit 1; }
cat $OUT/bench_gbm_10m.log
timeout -k 10 400 python3 -u scripts/fuzz_parity.py --minutes 4 --start 71000 > $OUT/fuzz.log 2>&1 || { echo "fuzz rc=$?"; tail -20 $OUT/fuzz.log; exit 1; }
tail -3 $OUT/fuzz.log
timeout -k 10 300 python3 -u scripts/fuzz_parity.py --minutes 2 --start 72000 --booster > $OUT/fuzz_booster.log 2>&1 || { echo "fuzz booster rc=$?"; tail -20 $OUT/fuzz_booster.log; exit 1; }
tail -3 $OUT/fuzz_booster.log
echo "gpu_r04r done"
