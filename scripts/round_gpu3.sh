# re-split slices: rank-stage GPU tests (large configs, stretches), shard timing at D, full D and B benches
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_exchange.py tests/test_gpu_large.py tests/test_gpu_de.py tests/test_gpu_grouped.py -q --timeout 300 --timeout-method thread > gpurun_out/r4_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r4_tests.log; exit 1; }
tail -1 gpurun_out/r4_tests.log
timeout -k 10 400 python scripts/shard_ingest_time.py D 8 > gpurun_out/r4_ing_d.log 2>&1 || { echo "ingD rc=$?"; tail gpurun_out/r4_ing_d.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4_ing_d.log
timeout -k 10 400 python bench.py --config D --no-cpu-baseline --no-pearson --no-transfers --steps 3 --warmup 1 > gpurun_out/r4_bench_d.json 2> gpurun_out/r4_bench_d.err || { echo "benchD rc=$?"; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pearson --no-transfers --steps 10 --warmup 2 > gpurun_out/r4_bench_b.json 2> gpurun_out/r4_bench_b.err || { echo "benchB rc=$?"; exit 1; }
echo ALLDONE
