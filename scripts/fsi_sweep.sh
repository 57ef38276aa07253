set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
B="python bench.py --no-cpu-baseline --no-transfers --no-pearson --steps 10 --warmup 3"
for v in "SCC_EIG_FSI_PASSES=1" "SCC_EIG_FSI_SEG=4" "SCC_EIG_FSI_SEG=4 SCC_EIG_FSI_PASSES=1" "SCC_EIG_FSI_SEG=6 SCC_EIG_FSI_PASSES=1"; do
  n=$(echo $v | tr ' =' '__')
  echo "== $v"
  env $v SCC_EIG_SI_LOG=1 timeout -k 10 300 $B > gpurun_out/sw_$n.log 2>&1 || { echo "rc=$?"; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"eigen": [0-9.]*' gpurun_out/sw_$n.log | head -2 | tr '\n' ' '
  grep "scc fsi" gpurun_out/sw_$n.log | tail -1
done
