#!/bin/bash
# issue / wait breakdown of the fp64-label kernels (one serialized fit of scripts/f64_probe.py)
set -u
OUT=gpurun_out/$1; shift
mkdir -p $OUT
export TMPDIR=/tmp SBAG_OVERLAP=0
PROBE="python3 scripts/f64_probe.py ${ROWS:-2000000} ${LEARNERS:-128}"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- $PROBE > $OUT/trace.log 2>&1 || { echo "trace failed rc=$?"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS --output-format csv -d $OUT/sq -o sq -- $PROBE > $OUT/sq.log 2>&1 || { echo "pmc sq failed rc=$?"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $OUT/lds -o lds -- $PROBE > $OUT/lds.log 2>&1 || { echo "pmc lds failed rc=$?"; exit 1; }
python3 scripts/pmc_summary.py $OUT profiles/r03/f64_pmc > /dev/null 2>&1 || true
python3 - <<PY
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob("$OUT/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_f64_hist" in r["Kernel_Name"]:
            acc[r["Counter_Name"]]["v"] += float(r["Counter_Value"])
for k, v in sorted(acc.items()):
    print(k, "%.4g" % v["v"])
PY
echo "pmc_f64 done"
