set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/tdist.log 2>&1
tail -2 gpurun_out/tdist.log
for m in 0 1 2 2 1; do
 SCC_EIG_PIN=$m timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/pin$m.log 2>&1
 python3 -c "import json;d=json.loads([l for l in open('gpurun_out/pin$m.log') if l.startswith('{')][0]);s=d['stage_ms'];print('pin$m',round(d['ms_per_step'],3),s['eig_vec'],s['eigen'])"
done
