#!/bin/bash
# One FETCH_SIZE or WRITE_SIZE pass over a bench config with extra env
# (A/B experiments on one kernel's traffic).  Usage:
#   scripts/pmc_one.sh <tag> <counter> <config> [VAR=value ...]
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=$1; ctr=$2; cfg=$3; shift 3
for kv in "$@"; do export "$kv"; done
d=gpurun_out/pmc1_$tag
mkdir -p $d
timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d $d -o run -- \
  python3 bench.py --config $cfg --no-cpu-baseline --no-transfers --no-pearson --steps 2 --warmup 2 > $d/log 2>&1
