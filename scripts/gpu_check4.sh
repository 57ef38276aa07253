# Gram change: distance tests, then B / C / D benches (gram stage)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_exchange.py -q -x --timeout 300 --timeout-method thread > gpurun_out/g_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/g_tests.log; exit 1; }
tail -1 gpurun_out/g_tests.log
for cfg in B C D; do
  timeout -k 10 400 python bench.py --config $cfg --no-cpu-baseline --no-pearson --no-transfers --steps 4 --warmup 1 > gpurun_out/g_bench_$cfg.json 2>/dev/null || { echo "bench $cfg rc=$?"; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/g_bench_$cfg.json').read().strip().splitlines()[-1])
s=d['stage_ms']; print('$cfg', round(d['ms_per_step'],3), 'gram', round(s['gram'],3), 'dist', round(s['dist'],3), 'gather', round(s['gather'],3))"
done
echo ALLDONE
