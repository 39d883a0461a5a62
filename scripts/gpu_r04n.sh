#!/bin/bash
# HEAD profiles for bench.py's traffic field: C3 and C4 kernel trace + PMC passes; C4 bench
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04n}
mkdir -p $OUT
bash scripts/profile.sh ${RUN:-r04n}_c3 || exit 1
timeout -k 10 600 python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_c4.log 2>&1 || { echo "bench c4 rc=$?"; tail -20 $OUT/bench_c4.log; exit 1; }
tail -1 $OUT/bench_c4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('avg_launch_ms'), d['breakdown_ms'])"
bash scripts/profile.sh ${RUN:-r04n}_c4 --workload c4 || exit 1
echo "gpu_r04n done"
