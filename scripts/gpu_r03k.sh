set -u
mkdir -p gpurun_out/r03k
SBAG_POISSON_EXP=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "poisson_bag_bit_exact" > gpurun_out/r03k/exp4_tests.log 2>&1 || { echo "exp4 tests failed"; tail -20 gpurun_out/r03k/exp4_tests.log; exit 1; }
tail -1 gpurun_out/r03k/exp4_tests.log
bash scripts/sampler_sweep.sh f "3:8 4:8:0 4:8:4 4:8:2 4:8:0 4:8:4" "128" || exit 1
bash scripts/pmc_sampler.sh exp4 SBAG_POISSON_EXP=4
SWEEP_ARGS="--rows 100000000 --learners 64 --reps 2" bash scripts/sampler_sweep.sh c4 "3:8 4:8 4:16 4:4" "128" || exit 1
