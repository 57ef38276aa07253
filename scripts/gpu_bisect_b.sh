# config-B rank kernels at earlier commits (worktrees under .bisect/, each with its own build)
set -u
export TMPDIR=/tmp
root=$(pwd)
mkdir -p gpurun_out/bis
for c in ${BIS:-5ac3d2e 49456db 90e6259 5871ff4 3e98c3d HEAD}; do
  d=.bisect/$c; [ $c = HEAD ] && d=.
  (cd $d && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $root/gpurun_out/bis/$c -o run -- python3 bench.py --no-cpu-baseline --no-transfers --no-pearson --steps 10 --warmup 3 > $root/gpurun_out/bis/$c.json 2> $root/gpurun_out/bis/$c.err) || { echo "$c failed"; tail -3 gpurun_out/bis/$c.err; exit 1; }
  python3 - "$c" <<'PY'
import csv, json, sys
c = sys.argv[1]
rows = {r["Name"].replace("void ", "").split("(")[0]: float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(f"gpurun_out/bis/{c}/run_kernel_stats.csv"))}
pick = {k: round(v, 1) for k, v in rows.items() if k.startswith(("k_rank_split", "k_rank_cross", "k_rank_mfma16", "k_rank_item<512", "k_rank_classify", "k_gene_stats", "k_ing_scatter"))}
st = {}
for l in open(f"gpurun_out/bis/{c}.json"):
    if l.startswith("{"):
        d = json.loads(l); st = d.get("stage_ms") or {}
print(c, "rank", round(st.get("gene_rank", 0), 3), pick)
PY
done
