#!/bin/bash
# Kernel-time profiles of bench.py under SCC_* experiment settings, one
# rocprofv3 process per setting: prof_variants.sh "SCC_X=1" "SCC_X=2" ...
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/var
export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i+1))
  env_kv=$v
  export ${env_kv}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/var/v$i -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/var/v$i.log 2>&1
  rc=$?; echo "variant $i ($v) rc=$rc"
  unset ${env_kv%%=*}
  [ $rc -ne 0 ] && exit $rc
done
exit 0
