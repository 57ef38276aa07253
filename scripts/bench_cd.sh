# configs C and D (device-generated inputs): bash scripts/bench_cd.sh [extra bench args]
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --config C --steps 3 --warmup 1 "$@" > gpurun_out/bench_C.log 2>&1 && \
timeout -k 10 500 python bench.py --config D --steps 3 --warmup 1 --no-pearson "$@" > gpurun_out/bench_D.log 2>&1
rc=$?
for c in C D; do grep '^{' gpurun_out/bench_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'], d['ms_per_step'], d['stage_ms'])"; done
exit $rc
