#!/bin/bash
# fp64 chain width A/B (C3 nondyadic, serialized level trace) and C4 bench with 2^32 budget
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04x}
mkdir -p $OUT
for cw in 16 4 1; do
  SBAG_F64_CHAIN_C=$cw SBAG_OVERLAP=0 SBAG_LEVEL_TRACE=1 timeout -k 10 300 python -u scripts/f64_probe.py > $OUT/probe_c$cw.log 2>&1 || { echo "probe rc=$?"; tail -30 $OUT/probe_c$cw.log; exit 1; }
  echo "C=$cw: $(grep 'level 0 ms' $OUT/probe_c$cw.log | tail -1) $(grep 'level 5 ms' $OUT/probe_c$cw.log | tail -1)"
  tail -1 $OUT/probe_c$cw.log | cut -c1-120
done
timeout -k 10 700 python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_c4.log 2>&1 || { echo "bench c4 rc=$?"; tail -20 $OUT/bench_c4.log; exit 1; }
tail -1 $OUT/bench_c4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', d['ms_per_step'], d['roofline']['frac']); print(d['nondyadic_labels']['ms_per_step'], d['nondyadic_labels']['breakdown_ms'])"
echo "gpu_r04x done"
