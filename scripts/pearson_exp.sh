#!/bin/bash
# Pearson kernel: parity tests, then timings (plain / f32 output / no-store)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/pexp; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_shard.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/pexp/tests.log 2>&1
rc=$?; tail -3 gpurun_out/pexp/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 scripts/pearson_only.py B 10 || exit $?
SCC_PEARSON_F32=1 timeout -k 10 200 python3 scripts/pearson_only.py B 10 || exit $?
SCC_PEARSON_NOSTORE=1 timeout -k 10 200 python3 scripts/pearson_only.py B 10 || exit $?
