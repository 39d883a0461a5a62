#!/bin/bash
# C5 shard: SBAG_HIST_SMALL repeat (one box)
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04bl}
mkdir -p $OUT
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --workload c5 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/c5_$tag.log 2>&1 || { echo "c5 $tag rc=$?"; tail -5 $OUT/c5_$tag.log; exit 1; }
  echo "$tag $(tail -1 $OUT/c5_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown_ms']; print(d['ms_per_step'], 'hist', b['hist_ms'])")"
}
run base SBAG_DUMMY=1
run small8k SBAG_HIST_SMALL=8192
run small16k SBAG_HIST_SMALL=16384
run base_b SBAG_DUMMY=2
run small8k_b SBAG_HIST_SMALL=8192
run small16k_b SBAG_HIST_SMALL=16384
echo "gpu_r04bl done"
