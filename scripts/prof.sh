#!/bin/bash
# rocprofv3 kernel-trace + stats of the bench (separate from PMC passes)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -n 5 gpurun_out/prof_bench.log
find gpurun_out/prof -name "*stats*" | head
exit $rc
