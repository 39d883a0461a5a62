#!/bin/bash
# GBM 10M x 100 breakdown; C4 bench with its nondyadic line (fp64-aware overlap estimate)
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04v}
mkdir -p $OUT
timeout -k 10 400 python3 -u scripts/bench_gbm.py --synthetic --rows 10000000 --features 100 --depth 5 --learners 5 > $OUT/bench_gbm_10m.log 2>&1 || { echo "gbm10m rc=$?"; tail -20 $OUT/bench_gbm_10m.log; exit 1; }
cat $OUT/bench_gbm_10m.log
timeout -k 10 700 python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_c4.log 2>&1 || { echo "bench c4 rc=$?"; tail -20 $OUT/bench_c4.log; exit 1; }
tail -1 $OUT/bench_c4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', d['ms_per_step'], d['roofline']['frac']); print(d['nondyadic_labels']['ms_per_step'], d['nondyadic_labels']['breakdown_ms'])"
echo "gpu_r04v done"
