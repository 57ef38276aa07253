# one bench line per configuration (HBM-resident step, stage times), with the
# rank stage's work lists (SCC_RANK_LOG=1 on the warm-up runs' stderr)
set -u
mkdir -p gpurun_out/cfg
export TMPDIR=/tmp
run() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/cfg/$n.json 2> gpurun_out/cfg/$n.err; local rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/cfg/$n.err; exit $rc; }; python3 - "$n" <<'PY'
import json, sys
n = sys.argv[1]
for line in open(f"gpurun_out/cfg/{n}.json"):
    if line.startswith("{"):
        d = json.loads(line)
        st = d.get("stage_ms") or d.get("stage_ms_per_step")
        print(n, "ms/step %.2f" % d["ms_per_step"], {k: round(v, 2) for k, v in st.items() if v > 0.05}, d.get("dataset_ms", {}).get("ms"))
PY
grep "scc rank" gpurun_out/cfg/$n.err | tail -1; }
SCC_RANK_LOG=1 run B 300 python bench.py --no-cpu-baseline --no-transfers --no-pearson --steps 10 --warmup 3
SCC_RANK_LOG=1 run C 400 python bench.py --config C --no-cpu-baseline --no-transfers --no-pearson --steps 3 --warmup 2
SCC_RANK_LOG=1 run D 400 python bench.py --config D --no-cpu-baseline --no-transfers --no-pearson --steps 3 --warmup 2
SCC_RANK_LOG=1 run E 400 python bench.py --config E --no-cpu-baseline --steps 3 --warmup 1
SCC_RANK_LOG=1 run Dslow 400 python bench.py --config D --de slow --no-cpu-baseline --no-transfers --no-pearson --steps 2 --warmup 1
SCC_RANK_LOG=1 run Bslow 300 python bench.py --de slow --no-cpu-baseline --no-transfers --no-pearson --steps 10 --warmup 3
