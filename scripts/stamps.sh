#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
cfg=${1:-B}
SCC_STAMPS=1 timeout -k 10 300 python scripts/diag_gpu.py $cfg > gpurun_out/stamps_$cfg.log 2>&1
rc=$?; echo "rc=$rc"; cat gpurun_out/stamps_$cfg.log | tail -20; exit $rc
