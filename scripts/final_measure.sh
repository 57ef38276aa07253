#!/bin/bash
# Round-end measurements on one MI355X (each GPU step under its own limit,
# stop at the first failure).  Part 1: PMC traffic (B, D, E) copied where
# bench.py reads it, then the bench lines.  Part 2: rocprof kernel stats.
# Usage: scripts/final_measure.sh 1|2
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/final
run() { local t=$1; shift; timeout -k 10 "$t" "$@" || { echo "FAILED ($?): $*"; exit 1; }; }
if [ "$1" = 1 ]; then
  for c in B D E; do
    run 400 bash scripts/pmc_traffic.sh $c > gpurun_out/final/pmc_$c.log 2>&1
    cp gpurun_out/pmc_traffic_$c/summary.json profiles/pmc_traffic_$c.json
  done
  run 300 python bench.py > gpurun_out/final/bench_b.json 2> gpurun_out/final/bench_b.err
  run 300 python bench.py --config C --no-cpu-baseline > gpurun_out/final/bench_c.json 2> gpurun_out/final/bench_c.err
  run 400 python bench.py --config D --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/final/bench_d.json 2> gpurun_out/final/bench_d.err
  run 400 python bench.py --config E --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/final/bench_e.json 2> gpurun_out/final/bench_e.err
  echo "part 1 done"
else
  run 400 python bench.py --config D --de slow --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/final/bench_d_slow.json 2> gpurun_out/final/bench_d_slow.err
  run 300 python bench.py --de slow --no-cpu-baseline > gpurun_out/final/bench_b_slow.json 2> gpurun_out/final/bench_b_slow.err
  run 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/prof_b -o run -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/final/prof_b.log 2>&1
  run 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/prof_d -o run -- python3 bench.py --config D --no-cpu-baseline --no-transfers --no-pearson --steps 3 --warmup 1 > gpurun_out/final/prof_d.log 2>&1
  run 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/prof_e -o run -- python3 bench.py --config E --no-cpu-baseline --no-transfers --steps 2 --warmup 1 > gpurun_out/final/prof_e.log 2>&1
  run 600 python -u scripts/shard_ingest_time.py D 8 > gpurun_out/final/shard_d_8.log 2>&1
  echo "part 2 done"
fi
