# re-split timing experiments at config D, as run for DESIGN §3.1 (SCC_RW_DEBUG 11..15 cut the wave
# re-split short after each phase; results invalid).  The cut points were removed from the kernel
# after the measurement: re-add them before running this again.
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for m in 0 11 12 13 14 15; do
  SCC_RW_DEBUG=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rsw_$m -o run --output-format csv -- \
    python3 bench.py --config D --no-cpu-baseline --no-pearson --steps 2 --warmup 1 > gpurun_out/rsw_$m.log 2>&1 || exit $?
  f=$(find gpurun_out/rsw_$m -name '*kernel_stats.csv' | head -n 1)
  echo "mode $m: $(grep k_rank_resplit_w $f | cut -d, -f4)"
done
