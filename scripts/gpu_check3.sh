# rank-stage change: DE / large / grouped / config tests, then B, D and E benches
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_de.py tests/test_gpu_large.py tests/test_gpu_grouped.py tests/test_gpu_configs.py tests/test_gpu_exchange.py -q -x --timeout 400 --timeout-method thread > gpurun_out/r_tests3.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r_tests3.log; exit 1; }
tail -1 gpurun_out/r_tests3.log
for cfg in B D E; do
  timeout -k 10 400 python bench.py --config $cfg --no-cpu-baseline --no-pearson --no-transfers --steps 4 --warmup 1 > gpurun_out/r3_bench_$cfg.json 2> gpurun_out/r3_bench_$cfg.err || { echo "bench $cfg rc=$?"; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/r3_bench_$cfg.json').read().strip().splitlines()[-1])
s=d.get('stage_ms') or d.get('stage_ms_per_step'); print('$cfg', round(d['ms_per_step'],3), 'rank', round(s['gene_rank'],3))"
done
echo ALLDONE
