# Chebyshev-filtered eigen at config B: unit tests, B parity with the filter on, B bench on/off, rocprof of the filter
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -k "chebyshev or subspace" -x -q --timeout 120 --timeout-method thread > gpurun_out/ch_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/ch_tests.log; exit 1; }
tail -2 gpurun_out/ch_tests.log
SCC_EIG_SI_LOG=1 SCC_EIG_CHEB=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-pearson --no-transfers --steps 10 --warmup 2 > gpurun_out/ch_bench_b.json 2> gpurun_out/ch_bench_b.err || { echo "bench rc=$?"; tail gpurun_out/ch_bench_b.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pearson --no-transfers --steps 10 --warmup 2 > gpurun_out/ch_bench_b0.json 2> gpurun_out/ch_bench_b0.err || { echo "bench0 rc=$?"; exit 1; }
SCC_EIG_CHEB=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ch_prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-pearson --no-transfers --steps 5 --warmup 1 > gpurun_out/ch_prof.log 2>&1 || { echo "prof rc=$?"; exit 1; }
SCC_EIG_CHEB=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -k config_b -x -q --timeout 500 --timeout-method thread > gpurun_out/ch_cfgb.log 2>&1 || { echo "cfgB rc=$?"; tail -30 gpurun_out/ch_cfgb.log; exit 1; }
tail -2 gpurun_out/ch_cfgb.log
echo ALLDONE
