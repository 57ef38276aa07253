#!/bin/bash
# Pearson distance kernel: parity tests, then the bench (side measurement in kernels.pearson)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_shard.py -x -q --timeout 120 --timeout-method thread -m gpu -k "pearson or Pearson or shard" > gpurun_out/tpearson.log 2>&1
rc=$?; tail -3 gpurun_out/tpearson.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/bench_pearson.log 2>&1 || exit $?
python3 -c "import json;d=json.loads([l for l in open('gpurun_out/bench_pearson.log') if l.startswith('{')][0]);print(d['ms_per_step'], d['stage_ms'].get('zscore'), json.dumps(d['kernels'].get('pearson')))"
