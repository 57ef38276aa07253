# distance tile width sweep (columns per tile) at B and D: bit-identity test first
set -u
mkdir -p gpurun_out/dsw
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -k "kernels_agree" -q --timeout 200 --timeout-method thread > gpurun_out/dsw/tests.log 2>&1 || { echo "tests rc=$?"; tail -20 gpurun_out/dsw/tests.log; exit 1; }
tail -1 gpurun_out/dsw/tests.log
for cfg in B D; do for c in 16 32 64 128; do
  SCC_DIST_COLS=$c timeout -k 10 400 python bench.py --config $cfg --no-cpu-baseline --no-pearson --no-transfers --steps 4 --warmup 1 > gpurun_out/dsw/$cfg$c.json 2>/dev/null || { echo "$cfg $c rc=$?"; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/dsw/$cfg$c.json').read().strip().splitlines()[-1])
print('$cfg cols $c', round(d['ms_per_step'],3), 'dist', round(d['stage_ms']['dist'],3))"
done; done
echo ALLDONE
