#!/bin/bash
# distance stage at config D with 64 vs 256 columns per tile
cd "${GRAFT_REPO_ROOT:-.}"
for c in 64 256; do
  SCC_DIST_COLS=$c timeout -k 10 300 python bench.py --config D --no-cpu-baseline --no-transfers --no-pearson --steps 2 --warmup 1 > gpurun_out/dcols_$c.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/dcols_$c.json').read().strip().splitlines()[-1]); print('cols $c', d['ms_per_step'], d['stage_ms']['dist'])"
done
SCC_DIST_COLS=256 timeout -k 10 300 python scripts/dist_tile_sweep.py B 0 || exit 1
