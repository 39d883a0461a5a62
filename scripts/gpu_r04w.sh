#!/bin/bash
# parallel label analysis (host), chunked fp64 buckets: label/GBM/f64 tests, GBM 10M, C4 bench
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04w}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_gpu_f64.py tests/test_gpu_gbm.py tests/test_gpu_parity.py tests/test_gpu_c_abi.py tests/test_gpu_ingest.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 400 python3 -u scripts/bench_gbm.py --synthetic --rows 10000000 --features 100 --depth 5 --learners 5 > $OUT/bench_gbm_10m.log 2>&1 || { echo "gbm10m rc=$?"; tail -20 $OUT/bench_gbm_10m.log; exit 1; }
cat $OUT/bench_gbm_10m.log
timeout -k 10 300 python3 -u scripts/bench_gbm.py > $OUT/bench_gbm.log 2>&1 || { echo "gbm rc=$?"; tail -20 $OUT/bench_gbm.log; exit 1; }
cat $OUT/bench_gbm.log
timeout -k 10 700 python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_c4.log 2>&1 || { echo "bench c4 rc=$?"; tail -20 $OUT/bench_c4.log; exit 1; }
tail -1 $OUT/bench_c4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', d['ms_per_step'], d['roofline']['frac']); print(d['nondyadic_labels']['ms_per_step'], d['nondyadic_labels']['breakdown_ms'])"
echo "gpu_r04w done"
