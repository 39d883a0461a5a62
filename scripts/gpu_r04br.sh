#!/bin/bash
# C4 shard: histogram workgroups per CU (SBAG_HIST_WPC) sweep (one box)
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04br}
mkdir -p $OUT
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 400 python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline --no-nondyadic > $OUT/c4_$tag.log 2>&1 || { echo "c4 $tag rc=$?"; tail -5 $OUT/c4_$tag.log; exit 1; }
  echo "$tag $(tail -1 $OUT/c4_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown_ms']; print(d['ms_per_step'], 'part', b['partition_ms'], 'hist', b['hist_ms'], 'root', b['root_ms'])")"
}
run base SBAG_DUMMY=1
run wpc1 SBAG_HIST_WPC=1
run wpc3 SBAG_HIST_WPC=3
run wpc4 SBAG_HIST_WPC=4
echo "gpu_r04br done"
