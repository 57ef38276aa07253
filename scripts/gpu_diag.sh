#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export SCC_DEBUG_SYNC=1 AMD_SERIALIZE_KERNEL=3 PYTHONUNBUFFERED=1
SCC_CAP_SMALL=256 SCC_CAP_MEDIUM=512 SCC_CHUNK_BIG=256 SCC_SELECT_CAP=32 SCC_UNION_CAP=64 \
  timeout -k 10 240 python scripts/diag_gpu.py forced > gpurun_out/diag_forced.log 2>&1
rc=$?; echo "forced rc=$rc"; tail -n 40 gpurun_out/diag_forced.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/diag_gpu.py B > gpurun_out/diag_B.log 2>&1
rc=$?; echo "B rc=$rc"; tail -n 40 gpurun_out/diag_B.log
exit $rc
