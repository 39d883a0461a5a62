#!/bin/bash
set -u
OUT=gpurun_out/r03j
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "poisson or bernoulli or all_ones" > $OUT/sampler_tests.log 2>&1 || { echo "sampler tests failed rc=$?"; tail -30 $OUT/sampler_tests.log; exit 1; }
tail -1 $OUT/sampler_tests.log
bash scripts/sampler_sweep.sh "$1" "$2" "$3"
