#!/bin/bash
# k_poisson4: sampler parity, then C3 sampler time per variant (bench breakdown, HIP events)
set -u
OUT=gpurun_out/r03i
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "poisson or bernoulli or all_ones" > $OUT/sampler_tests.log 2>&1 || { echo "sampler tests failed rc=$?"; tail -30 $OUT/sampler_tests.log; exit 1; }
tail -1 $OUT/sampler_tests.log
for v in "4 8" "4 16" "4 4"; do
  set -- $v
  F=$OUT/bench_v$1_l$2.log
  SBAG_POISSON_V=$1 SBAG_POISSON_LANES=$2 timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 \
    --no-cpu-baseline --no-nondyadic > $F 2>&1 || { echo "bench $v failed rc=$?"; tail -20 $F; exit 1; }
  echo "$v: $(tail -1 $F | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["breakdown_ms"]["sample_ms"], d["sampler_at_nproc_partitions"]["sample_ms"])')"
done
echo "gpu_r03h done"
bash scripts/pmc_sampler.sh v4l8 SBAG_POISSON_LANES=8 || exit 1
