#!/bin/bash
# GBM 10M host-side phases (SBAG_PROFILE_HOST); C4 shard bench with its nondyadic line at HEAD
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04aq}
mkdir -p $OUT
SBAG_PROFILE_HOST=1 timeout -k 10 300 python3 -u scripts/bench_gbm.py --synthetic --rows 10000000 --features 100 --depth 5 --learners 3 > $OUT/gbm_hostprof.log 2>&1 || { echo "gbm rc=$?"; tail -20 $OUT/gbm_hostprof.log; exit 1; }
grep "booster host\|host ms\|^\[sbag\] host" $OUT/gbm_hostprof.log | tail -4 | cut -c1-400; tail -1 $OUT/gbm_hostprof.log
timeout -k 10 700 python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_c4.log 2>&1 || { echo "bench c4 rc=$?"; tail -20 $OUT/bench_c4.log; exit 1; }
tail -1 $OUT/bench_c4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', d['ms_per_step'], d['roofline']['frac']); print(d['nondyadic_labels']['ms_per_step'], d['nondyadic_labels']['breakdown_ms'])"
echo "gpu_r04aq done"
