# kernel timelines of one DE step (rank stage) at several configurations
set -u
mkdir -p gpurun_out/tl
export TMPDIR=/tmp
tl() { local n=$1; shift; timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl/$n -o run -- "$@" > gpurun_out/tl/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/tl/$n.log; exit 1; }; python3 scripts/timeline.py gpurun_out/tl/$n/run_kernel_trace.csv k_rank_classify k_pair_test > gpurun_out/tl/$n.txt; echo "== $n"; cat gpurun_out/tl/$n.txt; }
tl B python3 bench.py --no-cpu-baseline --no-transfers --no-pearson --steps 3 --warmup 2
tl E python3 bench.py --config E --no-cpu-baseline --steps 2 --warmup 1
tl Dslow python3 bench.py --config D --de slow --no-cpu-baseline --no-transfers --no-pearson --steps 2 --warmup 1
