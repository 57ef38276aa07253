# rocprofv3 kernel stats of the config-E DE-only bench
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_E -o run --output-format csv -- \
  python3 bench.py --config E --steps 1 --warmup 1 > gpurun_out/prof_E.log 2>&1
rc=$?
f=$(find gpurun_out/prof_E -name '*kernel_stats.csv' | head -n 1)
[ -n "$f" ] && cp "$f" gpurun_out/kstats_E.csv
exit $rc
