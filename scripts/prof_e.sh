# rocprof kernel stats of the config-E DE (one engine run, K = 100)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_e -o run --output-format csv -- python3 bench.py --config E --no-cpu-baseline --no-pearson --no-transfers --steps 2 --warmup 1 > gpurun_out/prof_e.log 2>&1 || { echo "prof rc=$?"; tail gpurun_out/prof_e.log; exit 1; }
echo ALLDONE
