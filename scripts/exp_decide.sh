# decide ablations (timing only): SBAG_DECIDE_DEBUG bits 1 table, 2 nid store, 4 bits store, 8 nid load
for v in 0 1 2 4 6 7 15; do
  SBAG_DECIDE_DEBUG=$v bash scripts/trace.sh a$v > /dev/null; echo "debug $v"; grep -E "decide" gpurun_out/trace_a$v/dispatches.txt | awk '{print $NF}' | tr '\n' ' '; echo
done
