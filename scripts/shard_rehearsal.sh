# One config-C job sharded over 2 ranks that share the test box's one GPU
# (gloo carries the collectives; SCC_SHARE_GPU=1), beside the 1-rank run.
# A correctness rehearsal of the N-GPU path, not a scaling measurement.
mkdir -p gpurun_out
cfg=${1:-C}
timeout -k 10 400 python bench.py --config $cfg --mode shard --steps 2 --warmup 1 --no-pearson --no-cpu-baseline \
  > gpurun_out/shard1_$cfg.log 2>&1 || exit $?
SCC_SHARE_GPU=1 SCC_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --config $cfg --mode shard --steps 2 --warmup 1 --no-pearson \
  --no-cpu-baseline > gpurun_out/shard2_$cfg.log 2>&1 || exit $?
for f in gpurun_out/shard1_$cfg.log gpurun_out/shard2_$cfg.log; do
  grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d['ms_per_step'], d['config']['union'], d['config']['parallelism'])"
done
