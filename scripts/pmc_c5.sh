# Three PMC passes (no trace domains) over one serialized C5 shard fit: instruction mix and
# waits of the gini split search, the tile grouping and the partition, and their HBM bytes.
# Summarise with scripts/pmc_kernels.py gpurun_out/<run>.
set -u
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r06c5pmc}
mkdir -p $O
B="python3 bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline --no-continuous --no-nondyadic"
export SBAG_OVERLAP=0
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $O/p1 -o p1 -- $B > $O/p1.log 2>&1 || { echo p1 failed; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD --output-format csv -d $O/p2 -o p2 -- $B > $O/p2.log 2>&1 || { echo p2 failed; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p3 -o p3 -- $B > $O/p3.log 2>&1 || { echo p3 failed; exit 1; }
echo done
