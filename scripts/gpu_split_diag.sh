# the split's per-gene clocks at config D (SCC_RW_DEBUG=9) and one gene
# shard's rank-stage timeline (1/8 of D)
set -u
mkdir -p gpurun_out/sd
export TMPDIR=/tmp
SCC_RW_DEBUG=9 timeout -k 10 300 python bench.py --config D --no-cpu-baseline --no-transfers --no-pearson --steps 1 --warmup 1 > gpurun_out/sd/diag.json 2> gpurun_out/sd/diag.err || exit 1
grep "split diag" gpurun_out/sd/diag.err | tail -2
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sd/tr -o run -- python3 scripts/shard_ingest_time.py D 8 range > gpurun_out/sd/shard.log 2>&1 || exit 1
python3 scripts/timeline.py gpurun_out/sd/tr/run_kernel_trace.csv k_rank_classify k_pair_test
