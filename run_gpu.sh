#!/bin/bash
# GPU session script: each GPU step under its own time limit; stop at the first
# fault / abort / timeout (exit codes other than 0 = pass, 1 = test failures).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
mkdir -p gpurun_out
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name"
  # a heartbeat line a minute, so a long single test is not taken for a hang
  ( while sleep 60; do echo "[$name] $(date +%T) running"; done ) & local hb=$!
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  kill $hb 2>/dev/null; wait $hb 2>/dev/null
  echo "=== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 ;;
    testsall) step testsall 900 python -u -m pytest tests -m gpu -v --timeout 300 ;;
    bench) step bench 900 python bench.py ;;
    benchq) step benchq 600 python bench.py --no-cpu-baseline ;;
    stamps) SCC_STAMPS=1 step stamps 300 python scripts/diag_gpu.py B ;;
    prof) step prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 ;;
    tdist) step tdist 600 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 120 --timeout-method thread ;;
    benchev) step benchev 600 python bench.py --no-cpu-baseline --no-transfers --no-pearson --steps 20 --warmup 5 && step benchnoev 600 python bench.py --no-cpu-baseline --no-transfers --no-pearson --steps 20 --warmup 5 --no-stage-events ;;
    benchq2) step benchq2 600 python bench.py --no-cpu-baseline --no-transfers --steps 20 --warmup 5 ;;
    profq) step profq 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profq -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-transfers --no-pearson --steps 5 --warmup 2 ;;
    pmcB) step pmcB 600 bash scripts/pmc_traffic.sh B ;;
    profD) step profD 900 rocprofv3 --kernel-trace --stats -d gpurun_out/profD -o run --output-format csv -- python3 bench.py --config D --no-cpu-baseline --no-transfers --no-pearson --steps 2 --warmup 1 ;;
    profE) step profE 900 rocprofv3 --kernel-trace --stats -d gpurun_out/profE -o run --output-format csv -- python3 bench.py --config E --no-cpu-baseline --steps 2 --warmup 1 ;;
    pmcD) step pmcD 900 bash scripts/pmc_traffic.sh D ;;
    benchsplit) step benchsplit 600 python bench.py --no-cpu-baseline --no-transfers --steps 20 --warmup 5 --split-calls ;;
    cap2kB) SCC_SC_CAP=2048 step cap2kB 600 python bench.py --no-cpu-baseline --no-transfers --no-pearson --steps 20 --warmup 5 ;;
    cap3kB) SCC_SC_CAP=3072 step cap3kB 600 python bench.py --no-cpu-baseline --no-transfers --no-pearson --steps 20 --warmup 5 ;;
    cap6kB) SCC_SC_CAP=6144 step cap6kB 600 python bench.py --no-cpu-baseline --no-transfers --no-pearson --steps 20 --warmup 5 ;;
    cap2kD) SCC_SC_CAP=2048 step cap2kD 900 python bench.py --config D --no-cpu-baseline --no-transfers --no-pearson --steps 3 --warmup 2 ;;
    cap8kB) SCC_SC_CAP=8192 step cap8kB 600 python bench.py --no-cpu-baseline --no-transfers --no-pearson --steps 20 --warmup 5 ;;
    cap12kB) SCC_SC_CAP=12288 step cap12kB 600 python bench.py --no-cpu-baseline --no-transfers --no-pearson --steps 20 --warmup 5 ;;
    cap6kD) SCC_SC_CAP=6144 step cap6kD 900 python bench.py --config D --no-cpu-baseline --no-transfers --no-pearson --steps 3 --warmup 2 ;;
    cap8kD) SCC_SC_CAP=8192 step cap8kD 900 python bench.py --config D --no-cpu-baseline --no-transfers --no-pearson --steps 3 --warmup 2 ;;
    benchD) step benchD 900 python bench.py --config D --no-cpu-baseline --no-transfers --no-pearson --steps 3 --warmup 2 ;;
    benchBq) step benchBq 600 python bench.py --no-cpu-baseline --no-transfers --no-pearson --steps 20 --warmup 5 ;;
    benchC) step benchC 900 python bench.py --config C --no-cpu-baseline --no-transfers --no-pearson --steps 3 --warmup 2 ;;
    benchE) step benchE 900 python bench.py --config E --no-cpu-baseline --steps 3 --warmup 2 ;;
    benchBslow) step benchBslow 600 python bench.py --de slow --no-cpu-baseline --no-transfers --no-pearson --steps 10 --warmup 3 ;;
    benchDslow) step benchDslow 900 python bench.py --config D --de slow --no-cpu-baseline --no-transfers --no-pearson --steps 2 --warmup 1 ;;
    benchdev) SCC_BENCH_DEVICES=0,0 step benchdev 600 python bench.py --route devices --no-cpu-baseline --no-transfers --no-pearson --steps 10 --warmup 3 ;;
    dbgx) AMD_LOG_LEVEL=1 step dbgx 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_exchange.py -x -v --timeout 120 --timeout-method thread ;;
    rank) step rank 600 python -u -m pytest tests/test_gpu_rank_mfma.py tests/test_gpu_de.py -x -v --timeout 200 --timeout-method thread ;;
    rkstB) SCC_RW_DEBUG=7 step rkstB 300 python bench.py --no-cpu-baseline --no-transfers --no-pearson --steps 2 --warmup 1 ;;
    rkstD) SCC_RW_DEBUG=7 step rkstD 600 python bench.py --config D --no-cpu-baseline --no-transfers --no-pearson --steps 1 --warmup 1 ;;
    rkDslow) SCC_RW_DEBUG=7 step rkDslow 900 python bench.py --config D --de slow --no-cpu-baseline --no-transfers --no-pearson --steps 1 --warmup 1 ;;
    rkD256) SCC_RANK_MFMA_MIN=256 step rkD256 600 python bench.py --config D --no-cpu-baseline --no-transfers --no-pearson --steps 2 --warmup 1 ;;
    rkD128) SCC_RANK_MFMA_MIN=128 step rkD128 600 python bench.py --config D --no-cpu-baseline --no-transfers --no-pearson --steps 2 --warmup 1 ;;
    rkC256) SCC_RANK_MFMA_MIN=256 step rkC256 600 python bench.py --config C --no-cpu-baseline --no-transfers --no-pearson --steps 2 --warmup 1 ;;
    distt) step distt 600 python -u -m pytest tests/test_gpu_dist.py -k "kernels_agree or sizes" -x -v --timeout 200 --timeout-method thread ;;
    pca) step pca 900 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_exchange.py tests/test_gpu_devices.py tests/test_gpu_shard.py -x -v --timeout 200 --timeout-method thread ;;
    scores) step scores 600 python -u -m pytest tests/test_gpu_dist.py -k "scores or kernels_agree" -x -v --timeout 200 --timeout-method thread ;;
    gram) step gram 600 python -u -m pytest tests/test_gpu_dist.py -k "gram" -x -v --timeout 200 --timeout-method thread ;;
    rk16B) SCC_RANK_MFMA16=1 step rk16B 300 python bench.py --no-cpu-baseline --no-transfers --no-pearson --steps 10 --warmup 3 ;;
    rk16C) SCC_RANK_MFMA16=1 step rk16C 600 python bench.py --config C --no-cpu-baseline --no-transfers --no-pearson --steps 2 --warmup 1 ;;
    fsi) step fsi 600 python -u -m pytest tests/test_gpu_fsi.py tests/test_gpu_regress.py tests/test_gpu_devices.py -v --timeout 120 --timeout-method thread ;;
    fsiguard) step fsiguard 600 python -u -m pytest tests/test_gpu_dist.py -k "guard" -v --timeout 120 --timeout-method thread ;;
    benchfsi) SCC_EIG_FSI=1 SCC_EIG_SI_LOG=1 step benchfsi 600 python bench.py --no-cpu-baseline --no-transfers --no-pearson --steps 20 --warmup 5 ;;
    proffsi) SCC_EIG_FSI=1 step proffsi 600 rocprofv3 --kernel-trace --stats -d gpurun_out/proffsi -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-transfers --no-pearson --steps 5 --warmup 2 ;;
    smalleig) step smalleig 300 rocprofv3 --kernel-trace --stats -d gpurun_out/smalleig -o run --output-format csv -- python3 scripts/small_eig_bench.py ;;
    benchfsi3) SCC_EIG_FSI=1 SCC_EIG_FSI_PASSES=3 SCC_EIG_SI_LOG=1 step benchfsi3 600 python bench.py --no-cpu-baseline --no-transfers --no-pearson --steps 20 --warmup 5 ;;
    robust) step robust 600 python -u -m pytest tests/test_gpu_robust.py tests/test_gpu_fsi.py -x -v --timeout 200 --timeout-method thread ;;
    de) step de 900 python -u -m pytest tests/test_gpu_de.py tests/test_gpu_rank_mfma.py tests/test_gpu_grouped.py -x -v --timeout 300 --timeout-method thread ;;
    cfg) step cfg 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_large.py -x -v --timeout 600 --timeout-method thread ;;
    benchB) step benchB 600 python bench.py --no-cpu-baseline --steps 20 --warmup 5 ;;
    benchEq) step benchEq 900 python bench.py --config E --no-cpu-baseline --steps 2 --warmup 1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
