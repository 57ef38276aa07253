# round-end evidence on the committed tree: full GPU suite, config-B bench with CPU baseline, rocprof kernel
# stats at B, HBM traffic passes at B, C / D / E benches
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/f_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/f_tests.log; exit 1; }
tail -1 gpurun_out/f_tests.log
timeout -k 10 300 python bench.py > gpurun_out/f_bench_b.json 2> gpurun_out/f_bench_b.err || { echo "bench rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/f_prof_b -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-pearson --no-transfers --steps 5 --warmup 2 > gpurun_out/f_prof_b.log 2>&1 || { echo "prof rc=$?"; exit 1; }
true
timeout -k 10 300 python bench.py --config C --no-cpu-baseline --no-pearson --no-transfers --steps 3 --warmup 1 > gpurun_out/f_bench_c.json 2> gpurun_out/f_bench_c.err || { echo "benchC rc=$?"; exit 1; }
timeout -k 10 400 python bench.py --config D --no-cpu-baseline --no-pearson --no-transfers --steps 3 --warmup 1 > gpurun_out/f_bench_d.json 2> gpurun_out/f_bench_d.err || { echo "benchD rc=$?"; exit 1; }
timeout -k 10 400 python bench.py --config E --no-cpu-baseline --no-pearson --no-transfers --steps 3 --warmup 1 > gpurun_out/f_bench_e.json 2> gpurun_out/f_bench_e.err || { echo "benchE rc=$?"; exit 1; }
echo ALLDONE
