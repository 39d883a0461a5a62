#!/bin/bash
# C5 shard: sweep of the engine's launch knobs (one box)
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04bk}
mkdir -p $OUT
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c5_$tag.log 2>&1 || { echo "c5 $tag rc=$?"; tail -5 $OUT/c5_$tag.log; exit 1; }
  echo "$tag $(tail -1 $OUT/c5_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown_ms']; print(d['ms_per_step'], 'hist', b['hist_ms'], 'part', b['partition_ms'], 'group', b['group_ms'], 'split', b['split_ms'])")"
}
run base SBAG_DUMMY=1
run small2k SBAG_HIST_SMALL=2048
run small8k SBAG_HIST_SMALL=8192
run wpc2 SBAG_HIST_WPC=2
run wpc8 SBAG_HIST_WPC=8
run piece16k SBAG_PART_PIECE=16384
run piece4k SBAG_PART_PIECE=4096
run planes128 SBAG_PLANES_MIN_PARENTS=128
run base2 SBAG_DUMMY=2
echo "gpu_r04bk done"
