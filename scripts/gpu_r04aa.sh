#!/bin/bash
# MFMA root without the multiply-by-255: parity + C3 bench (root ms, step)
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04aa}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma_root.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 400 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['frac'], d['roofline']['root_mfma']['frac'], d['roofline']['root_mfma']['ms_per_fit'], d['nondyadic_labels']['ms_per_step'])"
echo "gpu_r04aa done"
