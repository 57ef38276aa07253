# per-kernel times of one rank's gene shard (1/8 of D's genes, range ingest) under rocprof
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r3_prof -o run --output-format csv -- python3 scripts/shard_ingest_time.py D 8 > gpurun_out/r3_prof.log 2>&1 || { echo "prof rc=$?"; tail gpurun_out/r3_prof.log; exit 1; }
echo ALLDONE
