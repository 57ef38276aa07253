#!/bin/bash
# Issue counters per kernel at a config (one PMC pass): VALU / SALU
# instructions, wave cycles, issue and wait cycles.  Output:
# gpurun_out/pmc_issue_<cfg>/
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
cfg=${1:-B}
out=gpurun_out/pmc_issue_$cfg
mkdir -p $out
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE \
  --output-format csv -d $out -o run -- python3 bench.py --config $cfg --no-cpu-baseline --no-transfers --no-pearson --steps 1 --warmup 1 > $out/pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; exit $rc
