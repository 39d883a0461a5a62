#!/bin/bash
# randomized parity fuzz at HEAD (fits and boosters) after the fp64 engine changes
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04au}
mkdir -p $OUT
timeout -k 10 420 python3 -u scripts/fuzz_parity.py --minutes 5 --start 81000 > $OUT/fuzz.log 2>&1 || { echo "fuzz rc=$?"; tail -20 $OUT/fuzz.log; exit 1; }
tail -3 $OUT/fuzz.log
timeout -k 10 300 python3 -u scripts/fuzz_parity.py --minutes 3 --start 82000 --booster > $OUT/fuzz_booster.log 2>&1 || { echo "fuzz booster rc=$?"; tail -20 $OUT/fuzz_booster.log; exit 1; }
tail -3 $OUT/fuzz_booster.log
timeout -k 10 300 python3 -u scripts/fuzz_parity.py --minutes 2 --start 83000 --big > $OUT/fuzz_big.log 2>&1 || { echo "fuzz big rc=$?"; tail -20 $OUT/fuzz_big.log; exit 1; }
tail -3 $OUT/fuzz_big.log
echo "gpu_r04au done"
