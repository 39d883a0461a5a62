#!/bin/bash
# time the histogram kernel with phases ablated (timing only; results are wrong)
export TMPDIR=/tmp
for m in 0 1 2 6; do
  OUT=gpurun_out/ablate/m$m; mkdir -p $OUT
  SBAG_HIST_ABLATE=$m timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT -o t -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --depth 3 "$@" > $OUT/log 2>&1 || { echo "mode $m failed"; exit 1; }
done
echo ablate done
