#!/bin/bash
# Issue/stall counters of k_pearson_mfma at config B (one PMC pass).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/pmc_pearson_issue
mkdir -p $out
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
  --output-format csv -d $out -o run -- python3 bench.py --no-cpu-baseline --no-transfers --steps 1 --warmup 1 > $out/pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; exit $rc
