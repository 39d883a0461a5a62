# sampler ablations (timing only): SBAG_POISSON_DBG 1 = no parse (2 rows/batch... 4), 2 = no generator
for v in 0 1 2 3; do
  SBAG_POISSON_DBG=$v bash scripts/trace.sh pz$v > /dev/null; echo "dbg $v: $(grep -E 'poisson' gpurun_out/trace_pz$v/dispatches.txt | awk '{print $NF}' | tr '\n' ' ')"
done
SBAG_POISSON_V1=1 bash scripts/trace.sh pv1 > /dev/null; echo "v1: $(grep -E 'poisson' gpurun_out/trace_pv1/dispatches.txt | awk '{print $NF}' | tr '\n' ' ')"
