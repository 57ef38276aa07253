# quick GPU check: distance / exchange / config tests, then the config-B bench (no CPU baseline)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_exchange.py tests/test_gpu_configs.py tests/test_gpu_shard.py -q -x --timeout 400 --timeout-method thread > gpurun_out/c_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/c_tests.log; exit 1; }
tail -1 gpurun_out/c_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pearson --no-transfers --steps 10 --warmup 2 > gpurun_out/c_bench_b.json 2> gpurun_out/c_bench_b.err || { echo "benchB rc=$?"; exit 1; }
python -c "
import json
d=json.loads(open('gpurun_out/c_bench_b.json').read().strip().splitlines()[-1])
print('B', round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['stage_ms'].items()})
"
echo ALLDONE
