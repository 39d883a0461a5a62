#!/bin/bash
# HEAD validation: full GPU suite, default bench, smoke, parity fuzz (fits, boosters, big)
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r04bj}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 400 python3 bench.py > $OUT/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['root_mfma']['frac'], d['nondyadic_labels']['ms_per_step'], d['nondyadic_labels']['exact_fallbacks'], d['cpu_baseline']['value'])"
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python3 -u scripts/fuzz_parity.py --minutes 3 --start 95000 > $OUT/fuzz.log 2>&1 || { echo "fuzz rc=$?"; grep -v "^ok" $OUT/fuzz.log | head -20 | cut -c1-250; exit 1; }
tail -1 $OUT/fuzz.log
timeout -k 10 200 python3 -u scripts/fuzz_parity.py --minutes 1 --start 96000 --booster > $OUT/fuzz_booster.log 2>&1 || { echo "fuzz booster rc=$?"; grep -v "^ok" $OUT/fuzz_booster.log | head -20 | cut -c1-250; exit 1; }
tail -1 $OUT/fuzz_booster.log
echo "gpu_r04bj done"
