# distance store-kernel sweep (SCC_DIST_KERNEL x SCC_DIST_COLS x SCC_DIST_NT) at configs B and D
set -e
B="python bench.py --no-cpu-baseline --no-pearson --no-transfers"
SCC_DIST_NT=1 timeout -k 10 120 $B > gpurun_out/ds_B_1_64_nt.log 2>&1
timeout -k 10 120 $B > gpurun_out/ds_B_1_64.log 2>&1
for v in "1 64" "1 256"; do set -- $v
  SCC_DIST_KERNEL=$1 SCC_DIST_COLS=$2 timeout -k 10 300 $B --config D --steps 3 --warmup 1 > gpurun_out/ds_D_$1_$2.log 2>&1
done
SCC_DIST_NT=1 SCC_DIST_COLS=64 timeout -k 10 300 $B --config D --steps 3 --warmup 1 > gpurun_out/ds_D_1_64_nt.log 2>&1
