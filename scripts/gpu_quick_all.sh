# quick check of a rank-stage change: B kernel stats, rank stage at D / E / D SLOW / B SLOW, rank parity tests
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/qa
BIS=HEAD bash scripts/gpu_bisect_b.sh || exit 1
run() { local n=$1; shift; timeout -k 10 300 "$@" > gpurun_out/qa/$n.json 2> gpurun_out/qa/$n.err || { echo "$n failed"; tail -5 gpurun_out/qa/$n.err; exit 1; }; python3 -c "
import json,sys
for l in open('gpurun_out/qa/$n.json'):
    if l.startswith('{'):
        d=json.loads(l); st=d.get('stage_ms') or {}; print('$n', round(d['ms_per_step'],3), 'rank', round(st.get('gene_rank',0),3), 'rank(line)', round(d.get('kernels',{}).get('gene_rank',{}).get('avg_launch_ms',0),3))
"; }
run d python bench.py --config D --no-cpu-baseline --no-transfers --no-pearson --steps 3 --warmup 2
run e python bench.py --config E --no-cpu-baseline --no-transfers --steps 2 --warmup 1
run ds python bench.py --config D --de slow --no-cpu-baseline --no-transfers --no-pearson --steps 2 --warmup 1
run bs python bench.py --de slow --no-cpu-baseline --no-transfers --no-pearson --steps 10 --warmup 3
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rank_mfma.py tests/test_gpu_de.py tests/test_gpu_streams.py tests/test_gpu_parity_b.py > gpurun_out/qa/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/qa/tests.log; exit 1; }
tail -1 gpurun_out/qa/tests.log
