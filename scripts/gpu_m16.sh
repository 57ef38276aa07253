# matrix-core rank kernel: rank parity, then bench lines at D SLOW, D (default and every gene on the matrix cores), C (and the 16-wide kernel for the slot genes), B
set -u
mkdir -p gpurun_out/m16
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rank_mfma.py tests/test_gpu_de.py > gpurun_out/m16/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/m16/tests.log; exit 1; }
tail -2 gpurun_out/m16/tests.log
run() { local n=$1; shift; timeout -k 10 300 "$@" > gpurun_out/m16/$n.json 2> gpurun_out/m16/$n.err || { echo "$n failed"; tail -5 gpurun_out/m16/$n.err; exit 1; }; python3 -c "
import json,sys
for l in open('gpurun_out/m16/$n.json'):
    if l.startswith('{'):
        d=json.loads(l); st=d.get('stage_ms') or {}; print('$n', round(d['ms_per_step'],2), 'rank', round(st.get('gene_rank',0),2))
"; }
D="python bench.py --config D --no-cpu-baseline --no-transfers --no-pearson --steps 3 --warmup 1"
C="python bench.py --config C --no-cpu-baseline --no-transfers --no-pearson --steps 3 --warmup 1"
run dslow python bench.py --config D --de slow --no-cpu-baseline --no-transfers --no-pearson --steps 2 --warmup 1
run d $D
SCC_RANK_MFMA=2 run d_all $D
run c $C
SCC_RANK_MFMA16=1 run c_m16 $C
run b python bench.py --no-cpu-baseline --no-transfers --no-pearson --steps 10 --warmup 3
