#!/bin/bash
# HBM traffic per kernel from rocprofv3 PMC counters (MI355X_MICROARCH.md
# HBM section): FETCH_SIZE and WRITE_SIZE in separate passes (they cannot
# share the 4 TCC slots), each pass its own process over the same bench
# command.  Output: gpurun_out/pmc_traffic/{fetch,write}/run_counter_collection.csv
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_traffic
for ctr in FETCH_SIZE WRITE_SIZE; do
  d=gpurun_out/pmc_traffic/$ctr
  timeout -s KILL 180 rocprofv3 --pmc $ctr --output-format csv -d $d -o run -- \
    python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/pmc_traffic/$ctr.log 2>&1
  rc=$?; echo "pass $ctr rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
python3 scripts/pmc_summary.py gpurun_out/pmc_traffic > gpurun_out/pmc_traffic/summary.json
cat gpurun_out/pmc_traffic/summary.json
