#!/bin/bash
# MFMA counters for k_gram_f64 / k_pearson_mfma at config B and HBM traffic
# (FETCH_SIZE, WRITE_SIZE, TCC_EA0_WRREQ) at config D, each pass its own
# rocprofv3 process (MI355X_MICROARCH.md HBM section: separate --pmc passes).
# Output: gpurun_out/pmc_mfma/<pass>/..._counter_collection.csv
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/pmc_mfma
mkdir -p $out
run() {  # name, counters, bench args
  timeout -s KILL 240 rocprofv3 --pmc $2 --output-format csv -d $out/$1 -o run -- \
    python3 bench.py --no-cpu-baseline --no-transfers --steps 2 --warmup 1 $3 > $out/$1.log 2>&1
  rc=$?; echo "pass $1 rc=$rc"
  return $rc
}
run mfma_b "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_MOPS_F32 GRBM_GUI_ACTIVE" "" || exit 1
run wrreq_b "TCC_EA0_WRREQ TCC_EA0_WRREQ_64B" "--no-pearson" || exit 1
run fetch_d "FETCH_SIZE" "--config D --no-pearson" || exit 1
run write_d "WRITE_SIZE" "--config D --no-pearson" || exit 1
python3 scripts/pmc_mfma_summary.py $out > $out/summary.json
cat $out/summary.json
