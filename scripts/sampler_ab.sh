#!/bin/bash
# Sampler parity tests, then C3 bench A/B over the Poisson sampler variants.
# usage: scripts/sampler_ab.sh <tag> ["V SPL PAR" ...]
set -u
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "poisson or bernoulli or all_ones" > $OUT/sampler_tests.log 2>&1 || { echo "sampler tests failed rc=$?"; tail -30 $OUT/sampler_tests.log; exit 1; }
tail -1 $OUT/sampler_tests.log

for v in "$@"; do
  set -- $v
  F=$OUT/bench_v$1_s$2_p$3.log
  SBAG_POISSON_V=$1 SBAG_POISSON_SPL=$2 SBAG_POISSON_PAR=$3 timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 \
    --no-cpu-baseline > $F 2>&1 || { echo "bench $v failed rc=$?"; tail -20 $F; exit 1; }
  echo "$v: $(tail -1 $F | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["breakdown_ms"]["sample_ms"], d.get("sampler_at_nproc_partitions"))')"
done
