# range ingest: GPU tests of the exchange path, the per-rank ingest times at B and D (8 shards)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_exchange.py tests/test_gpu_shard.py tests/test_gpu_shard_ranks.py -q --timeout 300 --timeout-method thread > gpurun_out/r2_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r2_tests.log; exit 1; }
tail -1 gpurun_out/r2_tests.log
timeout -k 10 300 python scripts/shard_ingest_time.py B 8 > gpurun_out/r2_ing_b.log 2>&1 || { echo "ingB rc=$?"; tail gpurun_out/r2_ing_b.log; exit 1; }
cat gpurun_out/r2_ing_b.log
timeout -k 10 400 python scripts/shard_ingest_time.py D 8 > gpurun_out/r2_ing_d.log 2>&1 || { echo "ingD rc=$?"; tail gpurun_out/r2_ing_d.log; exit 1; }
cat gpurun_out/r2_ing_d.log
echo ALLDONE
