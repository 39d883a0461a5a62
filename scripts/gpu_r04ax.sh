#!/bin/bash
# k_partition XCD queues (XCC_ID): parity (C3/C4/C5 shapes, random), A/B on the C3 bench and
# the C4 shard (partition_ms)
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04ax}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench_configs.py tests/test_gpu_random.py tests/test_gpu_parity.py -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for x in 0 1; do
  SBAG_PART_XCD=$x timeout -k 10 700 python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline --no-nondyadic > $OUT/bench_c4_x$x.log 2>&1 || { echo "bench c4 rc=$?"; tail -20 $OUT/bench_c4_x$x.log; exit 1; }
  tail -1 $OUT/bench_c4_x$x.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4 xcd=$x', d['ms_per_step'], d['breakdown_ms']['partition_ms'], d['breakdown_ms']['hist_ms'])"
  SBAG_PART_XCD=$x timeout -k 10 400 python3 bench.py --steps 10 --no-cpu-baseline --no-nondyadic > $OUT/bench_c3_x$x.log 2>&1 || { echo "bench c3 rc=$?"; tail -20 $OUT/bench_c3_x$x.log; exit 1; }
  tail -1 $OUT/bench_c3_x$x.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 xcd=$x', d['ms_per_step'], d['breakdown_ms']['partition_ms'])"
done
echo "gpu_r04ax done"
