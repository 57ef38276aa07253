# final check on the committed tree: smoke, the whole GPU suite, the default bench line
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/z_smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/z_smoke.log; exit 1; }
tail -2 gpurun_out/z_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/z_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/z_tests.log; exit 1; }
tail -1 gpurun_out/z_tests.log
timeout -k 10 300 python bench.py > gpurun_out/z_bench.json 2> gpurun_out/z_bench.err || { echo "bench rc=$?"; exit 1; }
python -c "
import json
d=json.loads(open('gpurun_out/z_bench.json').read().strip().splitlines()[-1])
print(d['metric'], d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['cpu_baseline']['value'])"
echo ALLDONE
