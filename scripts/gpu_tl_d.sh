# rank-stage timelines at config D FAST and SLOW (one step each)
set -u
mkdir -p gpurun_out/tl
export TMPDIR=/tmp
for c in D Dslow; do
  a="--config D"; [ $c = Dslow ] && a="--config D --de slow"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl/$c -o run -- python3 bench.py $a --no-cpu-baseline --no-transfers --no-pearson --steps 2 --warmup 1 > gpurun_out/tl/$c.log 2>&1 || exit 1
  echo "== $c"; python3 scripts/timeline.py gpurun_out/tl/$c/run_kernel_trace.csv k_rank_classify k_pair_test | tee gpurun_out/tl/$c.txt
done
