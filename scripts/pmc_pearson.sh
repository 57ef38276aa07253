#!/bin/bash
# Pearson epilogue traffic: WRITE_SIZE of k_pearson_mfma with nontemporal
# stores on (default) and off (SCC_PEARSON_NT=0), one PMC pass each, plus the
# bench's Pearson time for both.  Output: gpurun_out/pmc_pearson/
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/pmc_pearson
mkdir -p $out
for nt in 1 0; do
  SCC_PEARSON_NT=$nt timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-transfers --steps 3 --warmup 2 > $out/bench_nt$nt.log 2>&1
  rc=$?; echo "bench nt=$nt rc=$rc"; [ $rc -ne 0 ] && exit $rc
  SCC_PEARSON_NT=$nt timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/nt$nt -o run -- \
    python3 bench.py --no-cpu-baseline --no-transfers --steps 1 --warmup 1 > $out/pmc_nt$nt.log 2>&1
  rc=$?; echo "pmc nt=$nt rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
