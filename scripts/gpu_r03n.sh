#!/bin/bash
# short-segment k_hist (deep gini levels): parity (gini / C5 shapes), then C5 A/B of SBAG_HIST_SMALL
set -u
OUT=gpurun_out/r03n
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_configs.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "c5 or gini or vehicle or classes or class" > $OUT/gini_tests.log 2>&1 || { echo "gini tests rc=$?"; tail -30 $OUT/gini_tests.log; exit 1; }
tail -1 $OUT/gini_tests.log
for v in 0 4096 0 4096; do
  SBAG_HIST_SMALL=$v timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c5_small$v.log 2>&1 || { echo "c5 $v rc=$?"; tail -20 $OUT/c5_small$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/c5_small$v.log').read().strip().splitlines()[-1]); b=d['breakdown_ms']; print('small=$v', d['ms_per_step'], 'hist', b['hist_ms'], 'total', b['total_ms'])"
done
echo "gpu_r03n done"
