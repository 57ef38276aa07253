#!/bin/bash
# Issue / wait breakdown (SQ counters) of every kernel of the config-B step, two
# PMC passes (each its own process), counters checked against `rocprofv3 -L` first.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/pmci
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 -L > gpurun_out/pmci/list.txt 2>&1 || true
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  ok=""
  for c in $set; do
    if grep -qw "$c" gpurun_out/pmci/list.txt; then ok="$ok $c"; else echo "pass $i: $c not listed, skipped"; fi
  done
  timeout -s KILL 120 rocprofv3 --pmc $ok --output-format csv -d gpurun_out/pmci/p$i -o run -- python3 bench.py --no-cpu-baseline --no-pearson --no-transfers --steps 2 --warmup 1 > gpurun_out/pmci/p$i.log 2>&1
  rc=$?; echo "pass $i ($ok) rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
