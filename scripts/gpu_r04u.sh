#!/bin/bash
# C4 shard: k_hist vs forced row-lane k_hist_rl (A/B, same box); C4 full-shard parity with rl
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04u}
mkdir -p $OUT
for m in default rl; do
  if [ $m = rl ]; then export SBAG_HIST_RL_FORCE=1; fi
  timeout -k 10 500 python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline --no-nondyadic > $OUT/bench_c4_$m.log 2>&1 || { echo "bench c4 $m rc=$?"; tail -20 $OUT/bench_c4_$m.log; exit 1; }
  tail -1 $OUT/bench_c4_$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m', d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['breakdown_ms']['hist_ms'])"
done
SBAG_HIST_RL_FORCE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_configs.py -m gpu -x -q --timeout 500 --timeout-method thread -k c4 > $OUT/gpu_tests_rl.log 2>&1 || { echo "tests rc=$?"; tail -40 $OUT/gpu_tests_rl.log; exit 1; }
tail -2 $OUT/gpu_tests_rl.log
echo "gpu_r04u done"
