# rocprofv3 kernel stats of one bench config: bash scripts/prof_cfg.sh <config> [extra bench args]
set -u
cfg=$1; shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$cfg -o run --output-format csv -- \
  python3 bench.py --config "$cfg" --no-cpu-baseline --no-pearson --steps 2 --warmup 1 "$@" > gpurun_out/prof_$cfg.log 2>&1
rc=$?
f=$(find gpurun_out/prof_$cfg -name '*kernel_stats.csv' | head -n 1)
[ -n "$f" ] && cp "$f" gpurun_out/kstats_$cfg.csv && head -n 25 "$f"
exit $rc
