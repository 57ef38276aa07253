#!/bin/bash
# Round-end measurements on one MI355X (each GPU step under its own limit,
# stop at the first failure).
#   1: PMC traffic (B, B slow, D slow; D and E: part 4) copied where bench.py reads it
#   2: the bench lines (B with the CPU baseline, C, D, E, D slow, B slow)
#   3: rocprof kernel stats (B, D, E, D slow)
#   4: PMC traffic D and E
# Usage: scripts/final_measure.sh 1|2|3|4
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/final
run() { local t=$1; shift; timeout -k 10 "$t" "$@" || { echo "FAILED ($?): $*"; exit 1; }; }
pmc() {  # config [slow]
  local tag=$1; [ "${2:-fast}" = slow ] && tag=${1}_slow
  run 400 bash scripts/pmc_traffic.sh "$1" "${2:-fast}" > gpurun_out/final/pmc_$tag.log 2>&1
  cp gpurun_out/pmc_traffic_$tag/summary.json profiles/pmc_traffic_$tag.json
  echo "pmc $tag done"
}
case "$1" in
1)
  pmc B; pmc B slow; pmc D slow
  ;;
4)
  pmc D; pmc E
  ;;
2)
  run 300 python bench.py > gpurun_out/final/bench_b.json 2> gpurun_out/final/bench_b.err; echo "bench B done"
  run 300 python bench.py --config C --no-cpu-baseline > gpurun_out/final/bench_c.json 2> gpurun_out/final/bench_c.err; echo "bench C done"
  run 400 python bench.py --config D --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/final/bench_d.json 2> gpurun_out/final/bench_d.err; echo "bench D done"
  run 400 python bench.py --config E --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/final/bench_e.json 2> gpurun_out/final/bench_e.err; echo "bench E done"
  run 400 python bench.py --config D --de slow --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/final/bench_d_slow.json 2> gpurun_out/final/bench_d_slow.err; echo "bench D slow done"
  run 300 python bench.py --de slow --no-cpu-baseline > gpurun_out/final/bench_b_slow.json 2> gpurun_out/final/bench_b_slow.err; echo "bench B slow done"
  ;;
3)
  run 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/prof_b -o run -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/final/prof_b.log 2>&1; echo "prof B done"
  run 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/prof_d -o run -- python3 bench.py --config D --no-cpu-baseline --no-transfers --no-pearson --steps 3 --warmup 1 > gpurun_out/final/prof_d.log 2>&1; echo "prof D done"
  run 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/prof_e -o run -- python3 bench.py --config E --no-cpu-baseline --no-transfers --steps 2 --warmup 1 > gpurun_out/final/prof_e.log 2>&1; echo "prof E done"
  run 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/prof_d_slow -o run -- python3 bench.py --config D --de slow --no-cpu-baseline --no-transfers --no-pearson --steps 2 --warmup 1 > gpurun_out/final/prof_d_slow.log 2>&1; echo "prof D slow done"
  ;;
esac
echo "part $1 done"
