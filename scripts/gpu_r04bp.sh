#!/bin/bash
# C4 shard: partition piece size sweep (one box): 32k, 16k, then 4k
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04bp}
mkdir -p $OUT
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 400 python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline --no-nondyadic > $OUT/c4_$tag.log 2>&1 || { echo "c4 $tag rc=$?"; tail -5 $OUT/c4_$tag.log; exit 1; }
  echo "$tag $(tail -1 $OUT/c4_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown_ms']; print(d['ms_per_step'], 'part', b['partition_ms'], 'hist', b['hist_ms'], 'sample', b['sample_ms'])")"
}
run base SBAG_DUMMY=1
run piece4k SBAG_PART_PIECE=4096
run piece4k_b SBAG_PART_PIECE=4096
run base2 SBAG_DUMMY=2
echo "gpu_r04bp done"
