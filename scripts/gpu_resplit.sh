mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_de.py -x -q --timeout 300 > gpurun_out/t_de.log 2>&1; rc=$?
tail -5 gpurun_out/t_de.log; [ $rc -ne 0 ] && exit $rc
bash scripts/stamps.sh C && bash scripts/stamps.sh D
