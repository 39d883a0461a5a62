#!/bin/bash
# A/B of bench variants on one box, optionally after a pytest selection.
# usage: scripts/ab.sh <tag> <workload> "<pytest -k expr or ->" "<ENV=v ...>" ["<ENV=v ...>" ...]
# ("-" skips the tests; "none" as a variant runs the default environment)
set -u
TAG=$1; W=$2; K=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "$K" != "-" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -k "$K" -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
fi
for v in "$@"; do
  n=$(echo "$v" | tr '= ' '__')
  e=$v; [ "$v" = "none" ] && e=""
  env $e timeout -k 10 300 python3 bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline --sampler-partitions 128 > $OUT/bench_${W}_$n.log 2>&1 || { echo "bench $W $v failed rc=$?"; tail -5 $OUT/bench_${W}_$n.log; exit 1; }
  python3 -c "import json;d=json.loads([l for l in open('$OUT/bench_${W}_$n.log') if l.startswith('{')][-1]);b=d['breakdown_ms'];print('$W $n step', d['ms_per_step'], 'hist', b['hist_ms'], 'part', b['partition_ms'], 'split', b['split_ms'], 'sample', b['sample_ms'])"
done
echo "ab $TAG done"
