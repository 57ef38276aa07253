#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
SCC_STAMPS=1 timeout -k 10 300 python scripts/diag_gpu.py B > gpurun_out/stamps_B.log 2>&1
rc=$?; echo "rc=$rc"; cat gpurun_out/stamps_B.log | tail -20; exit $rc
