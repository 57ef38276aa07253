# rank parity (bit-exact) + D / E / D SLOW timings + one shard of D
set -u
mkdir -p gpurun_out/rq
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_de.py tests/test_gpu_rank_mfma.py tests/test_gpu_streams.py tests/test_gpu_grouped.py tests/test_gpu_configs.py tests/test_gpu_large.py tests/test_gpu_shard.py tests/test_gpu_exchange.py -x -q --timeout 600 --timeout-method thread > gpurun_out/rq/tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/rq/tests.log; exit 1; }
tail -2 gpurun_out/rq/tests.log
for c in "D" "E" "D --de slow"; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-transfers --no-pearson --steps 3 --warmup 2 > gpurun_out/rq/o.json 2>/dev/null || exit 1
  echo "$c $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rq/o.json) $(grep -o '"gene_rank": [0-9.]*' gpurun_out/rq/o.json | head -1)"
done
timeout -k 10 600 python -u scripts/shard_ingest_time.py D 8 range > gpurun_out/rq/shard.log 2>&1 || exit 1
grep "range read" gpurun_out/rq/shard.log
