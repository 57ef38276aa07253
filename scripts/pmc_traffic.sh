#!/bin/bash
# HBM traffic per kernel from rocprofv3 PMC counters (MI355X_MICROARCH.md
# HBM section): FETCH_SIZE and WRITE_SIZE in separate passes (they cannot
# share the 4 TCC slots), each pass its own process over the same bench
# command.  Output: gpurun_out/pmc_traffic_<cfg>/{FETCH_SIZE,WRITE_SIZE}/...
# Usage: scripts/pmc_traffic.sh [config=B] [de=fast|slow]
# (slow: reclusterDEConsensus, written to pmc_traffic_<cfg>_slow; bench.py
# reads profiles/pmc_traffic_<cfg>[_slow].json for the matching --de)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
cfg=${1:-B}
de=${2:-fast}
tag=$cfg; [ "$de" = slow ] && tag=${cfg}_slow
out=gpurun_out/pmc_traffic_$tag
mkdir -p $out
for ctr in FETCH_SIZE WRITE_SIZE; do
  d=$out/$ctr
  timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d $d -o run -- \
    python3 bench.py --config $cfg --de $de --no-cpu-baseline --no-transfers --no-pearson --steps 2 --warmup 2 \
    > $out/$ctr.log 2>&1
  rc=$?; echo "pass $ctr rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
python3 scripts/pmc_summary.py $out > $out/summary.json
cat $out/summary.json
