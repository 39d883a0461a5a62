set -u
export TMPDIR=/tmp
O=gpurun_out/r06mf
mkdir -p $O
B="python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-continuous --no-nondyadic --sampler-partitions 128"
export SBAG_OVERLAP=0
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_I8 SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU --output-format csv -d $O/p1 -o p1 -- $B > $O/p1.log 2>&1 || { echo p1 failed; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU_MFMA_MOPS_I8 --output-format csv -d $O/p2 -o p2 -- $B > $O/p2.log 2>&1 || { echo p2 failed; exit 1; }
echo done
