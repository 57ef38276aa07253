set -u
mkdir -p gpurun_out/g13
export TMPDIR=/tmp
run() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/g13/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; tail -3 gpurun_out/g13/$n.log; [ $rc -eq 0 ] || exit $rc; }
run rank 900 python -u -m pytest tests/test_gpu_de.py tests/test_gpu_rank_mfma.py tests/test_gpu_streams.py tests/test_gpu_configs.py::test_config_b_full_fast_parity tests/test_gpu_large.py -x -q --timeout 600 --timeout-method thread
run trD 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/g13/trD -o run -- python3 bench.py --config D --no-cpu-baseline --no-transfers --no-pearson --steps 2 --warmup 1
python3 scripts/timeline.py gpurun_out/g13/trD/run_kernel_trace.csv k_rank_classify k_pair_test
run benchB 300 python bench.py --no-cpu-baseline --no-transfers --no-pearson --steps 20 --warmup 5
grep -o '"gene_rank": [0-9.]*' gpurun_out/g13/benchB.log; grep -o '"ms_per_step": [0-9.]*' gpurun_out/g13/benchB.log
