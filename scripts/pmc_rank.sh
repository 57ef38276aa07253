#!/bin/bash
# PMC passes over one config-B DE + distance run (each pass its own process).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
i=0
for ctr in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 scripts/diag_gpu.py B > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i ($ctr) rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
