#!/bin/bash
# Poisson sampler kernel time (rocprofv3 kernel trace) per variant and partition count,
# C3 shape (10M rows, 128 learners).  A variant is V:LANES[:EXP] (V ignored since round 6: k_poisson4 only;
# SBAG_POISSON_LANES, SBAG_POISSON_EXP).  Box-to-box clocks differ by up to ~10 %: compare
# variants within one call.  usage: scripts/sampler_sweep.sh <tag> "<variants...>" "<P...>"
set -u
TAG=$1; VARS=$2; PS=$3
OUT=gpurun_out/sweep_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for v in $VARS; do for p in $PS; do
  IFS=: read -r V L E <<< "$v"
  D=$OUT/v${V}_l${L}_e${E:-0}_p${p}
  SBAG_POISSON_V=$V SBAG_POISSON_LANES=$L SBAG_POISSON_EXP=${E:-0} timeout -s KILL 120 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $D -o t -- python3 scripts/bench_sampler.py --reps 3 --partitions $p ${SWEEP_ARGS:-} > $D.log 2>&1 || { echo "$v p=$p failed rc=$?"; exit 1; }
  python3 - "$D" "$v" "$p" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/*kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        if "poisson" in r["Name"]:
            print(f"{sys.argv[2]} P={sys.argv[3]}: {float(r['AverageNs'])/1e6:.3f} ms x{r['Calls']}")
PY
done; done
