set -u
mkdir -p gpurun_out/g13
export TMPDIR=/tmp
run() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/g13/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; tail -3 gpurun_out/g13/$n.log; [ $rc -eq 0 ] || exit $rc; }
run rank 900 python -u -m pytest tests/test_gpu_de.py tests/test_gpu_rank_mfma.py tests/test_gpu_streams.py tests/test_gpu_grouped.py tests/test_gpu_configs.py tests/test_gpu_large.py -x -q --timeout 600 --timeout-method thread
bash scripts/gpu_sweep_configs.sh
