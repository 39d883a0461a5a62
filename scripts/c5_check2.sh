#!/bin/bash
set -u
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_parity.py tests/test_gpu_random.py tests/test_gpu_bench_configs.py -k "ingest or sparse or columnar or class or gini or random or c5 or vehicle or classif" -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for v in "" "SBAG_NO_TILE_GROUPING=1" "SBAG_HIST_GROUPED_LDS_KB=70" "SBAG_HIST_GROUPED_LDS_KB=20"; do
  n=$(echo "$v" | tr '=' '_'); n=${n:-default}
  env $v timeout -k 10 240 python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline --sampler-partitions 128 > $OUT/bench_c5_$n.log 2>&1 || { echo "bench c5 $v failed rc=$?"; exit 1; }
  python3 -c "import json;d=json.loads([l for l in open('$OUT/bench_c5_$n.log') if l.startswith('{')][-1]);print('$n', d['ms_per_step'], d['breakdown_ms']['hist_ms'])"
done
timeout -k 10 240 python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline --sampler-partitions 128 > $OUT/bench_c4.log 2>&1 || { echo "bench c4 failed rc=$?"; exit 1; }
python3 -c "import json;d=json.loads([l for l in open('$OUT/bench_c4.log') if l.startswith('{')][-1]);print('c4', d['ms_per_step'], d['breakdown_ms']['hist_ms'])"
echo "c5_check2 $TAG done"
