# knob sweep: scatter staging cap and tridiagonalisation workgroups at config B, subspace iterations at D and C
set -u
mkdir -p gpurun_out/sweep
export TMPDIR=/tmp
run() {  # run <tag> <config> [ENV=VAL ...]
  local tag=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-pearson --no-transfers --steps 6 --warmup 2 \
    > gpurun_out/sweep/$tag.json 2> gpurun_out/sweep/$tag.err || { echo "$tag rc=$?"; return 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/sweep/$tag.json').read().strip().splitlines()[-1])
s=d['stage_ms']; print('$tag', round(d['ms_per_step'],3), 'ingest', round(s['ingest'],3), 'eigen', round(s['eigen'],3), 'rank', round(s['gene_rank'],3))"
  grep -a "scc si" gpurun_out/sweep/$tag.err | sort | uniq -c | head -3
}
run b_base B
run b_sc2048 B SCC_SC_CAP=2048
run b_sc8192 B SCC_SC_CAP=8192
run b_nwg16 B SCC_EIG_NWG=16
run b_nwg24 B SCC_EIG_NWG=24
run b_nwg28 B SCC_EIG_NWG=28
run d_it20 D SCC_EIG_SI_IT=20 SCC_EIG_SI_LOG=1
run d_it16 D SCC_EIG_SI_IT=16 SCC_EIG_SI_LOG=1
run c_it20 C SCC_EIG_SI_IT=20 SCC_EIG_SI_LOG=1
run c_it16 C SCC_EIG_SI_IT=16 SCC_EIG_SI_LOG=1
echo ALLDONE
