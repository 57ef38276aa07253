#!/usr/bin/env python3
"""bench.py — headline benchmark of the scConsensus MI355X engine.

Metric (BASELINE.json): end-to-end DE + distance seconds and cell-pairs/sec at
the 26k-cell PBMC shape (config B: 26,000 cells x 10,000 genes, 12 consensus
clusters, 66 pairs), 1/2/4/8 GPUs.

One step = one pass of the hot path over one synthetic job resident in HBM:
  scc_de_run(FAST)   reclusterDEConsensusFast's pair loop, all 66 pairs x all
                     genes (stats, Wilcoxon, BH, filters, top-N, union)
  scc_distance       PCA(15) + packed Euclidean dist (N(N-1)/2 fp64, kept in HBM)
value = cell-pairs / second = jobs * N(N-1)/2 / step time.

Multi-GPU: one process per GPU (torchrun); by default every rank runs its own
job (seed offset by rank) with no data-path collective ("scaling": "weak").
--mode shard runs ONE job over all ranks ("scaling": "strong"): DE on gene
row-blocks combined by one RCCL all-reduce (scc_de_run_shard / scc_de_finish),
then each rank's column slice of the packed distance (scc_distance_cols).  The
step time is the max over ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0    # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PEAK_FP64_TFS = 78.6     # MI355X FP64 matrix (spec)
PEAK_FP32_TFS = 157.3    # MI355X FP32 matrix (v_mfma_f32_32x32x2_f32; MI355X_MICROARCH.md)


def _args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="B")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pearson", action="store_true", help="skip the side measurement of the Pearson kernel")
    ap.add_argument("--cpu-sample-genes", type=int, default=300)
    ap.add_argument("--mode", choices=["jobs", "shard"], default="jobs",
                    help="jobs: one job per rank (weak scaling); shard: ONE job over all ranks (strong scaling: "
                         "DE gene row-blocks + one all-reduce, distance column slices)")
    return ap.parse_args()


DEVICE_GEN = ("C", "D", "E")


def cpu_baseline(d, code, K, union, sample_genes, seed=0):
    """The oracle (C restatement of the R algorithm, 1 thread) on a bounded
    sample of the same workload, scaled linearly: DE on a seeded gene sample
    (all 66 pairs), exact PCA on the union, `dist` on a row sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from scipy.spatial.distance import cdist
    rng = np.random.default_rng(seed)
    if not hasattr(d, "scipy_csc"):
        d = d.to_host()
    genes = np.sort(rng.choice(d.G, min(sample_genes, d.G), replace=False))
    csr = d.scipy_csc().tocsr()
    Xs = np.asarray(csr[genes].todense())
    t0 = time.perf_counter()
    O.de_fast(Xs, code, K)
    t_de = (time.perf_counter() - t0) * d.G / len(genes)
    Xu = np.asarray(csr[union].todense())
    t0 = time.perf_counter()
    S = O.pca_scores(Xu, np.arange(len(union)))
    t_pca = time.perf_counter() - t0
    rows = rng.choice(d.N, 256, replace=False)
    t0 = time.perf_counter()
    cdist(S[rows], S, "euclidean")
    t_dist = (time.perf_counter() - t0) * (d.N / 2) / len(rows)
    t = t_de + t_pca + t_dist
    return {"value": d.N * (d.N - 1) / 2 / t, "unit": "cell-pairs/s", "cores": 1, "kind": "port",
            "sample": f"oracle DE on {len(genes)}/{d.G} genes x all {K*(K-1)//2} pairs scaled x{d.G/len(genes):.1f}; "
                      f"exact SVD PCA on |U|={len(union)}; dist on 256/{d.N} rows scaled; "
                      f"est. end-to-end {t:.1f} s (DE {t_de:.1f}, PCA {t_pca:.1f}, dist {t_dist:.1f})",
            "end_to_end_s": t}


def de_only(a, eng, ds, d, code, K, dist, world):
    """Config E (BASELINE: "1M-cell sparse CSR input, 100 clusters (4950
    pairs), DE-only"): the FAST DE over all pairs, K > 64 through the grouped
    orchestration (scconsensus_amd/grouped.py), rows fetched to the host."""
    from scconsensus_amd import grouped

    def step():
        return grouped.de_fast_grouped(eng, ds, code, K)

    for _ in range(a.warmup):
        r = step()
    eng.synchronize()
    eng.reset_timers()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        r = step()
    eng.synchronize()
    dist.barrier()
    dt = dist.max_over_ranks(time.perf_counter() - t0)
    s_step = dt / a.steps
    fams = ["ingest", "gene_stats", "pair_filter", "gene_rank", "pair_test", "pair_select"]
    stage_ms = {}
    for f in fams:
        t, n = eng.kernel_time(f)
        stage_ms[f] = round(t / max(a.steps, 1), 3)  # per step (several engine runs per step)
    P = K * (K - 1) // 2
    out = {"metric": "DE-only seconds per reclusterDEConsensusFast DE at config E", "value": s_step, "unit": "s",
           "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "ms_per_step": s_step * 1e3,
           "higher_is_better": False, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
           "data": "synthetic (SURVEY §8d generator on the GPU, gene-major CSR)",
           "config": {"workload": f"config E: FAST DE (all {P} pairs, Wilcoxon), {d.N} cells x {d.G} genes CSR, K={K}",
                      "cells": d.N, "genes": d.G, "clusters": K, "pairs": P, "nnz": d.nnz,
                      "union": len(r.union), "rows": int(len(r.rows.gene)), "engine_runs_per_step": max(1, -(-K // grouped.GROUP) * (-(-K // grouped.GROUP) - 1) // 2),
                      "parallelism": f"jobs{world}"},
           "stage_ms_per_step": stage_ms}
    if dist.rank == 0:
        print(json.dumps(out), flush=True)
    dist.close()


def main():
    a = _args()
    if a.mode == "shard":
        import torch  # noqa: F401  (torch's HIP runtime first: the shard buffers are torch tensors)
    from scconsensus_amd import parallel
    # RCCL ("nccl") when launched by torchrun with N > 1.  SCC_SHARE_GPU=1 with
    # SCC_DIST_BACKEND=gloo rehearses several ranks on one GPU (tests only).
    dist = parallel.init(os.environ.get("SCC_DIST_BACKEND") or None)
    rank, world, local = dist.rank, dist.world, dist.local_rank
    from scconsensus_amd import _native as nat
    from scconsensus_amd import api, synth
    from scconsensus_amd.synth import CONFIGS

    cfg = CONFIGS[a.config]
    shard = a.mode == "shard"
    seed = cfg["seed"] if shard else parallel.job_seed(cfg["seed"], rank)
    gpu = 0 if os.environ.get("SCC_SHARE_GPU") else local
    if a.config in DEVICE_GEN:  # C/D/E: generated in HBM (host generation takes minutes)
        import torch
        d = synth.generate_device(a.config, f"cuda:{gpu}", seed=seed, layout="csr" if a.config == "E" else "csc")
        torch.cuda.synchronize()
    else:
        d = synth.generate(a.config, seed=seed)
    names, code = api.select_clusters(d.labels, 10)
    K = len(names)
    P = K * (K - 1) // 2
    eng = nat.Engine(gpu, profile=True)
    if a.config == "E":
        ds = eng.dataset_csr_device(d.indptr.data_ptr(), d.indices.data_ptr(), d.data.data_ptr(), d.G, d.N, d.nnz)
        return de_only(a, eng, ds, d, code, K, dist, world)
    if a.config in DEVICE_GEN:
        ds = eng.dataset_csc_device(d.indptr.data_ptr(), d.indices.data_ptr(), d.data.data_ptr(), d.G, d.N, d.nnz)
    else:
        ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)  # H2D before timing
    npairs_cells = d.N * (d.N - 1) / 2

    if shard:
        import torch
        from scconsensus_amd import sharded
        tdev = torch.device(f"cuda:{gpu}")

    def step():
        if shard:  # one job: gene row-blocks + one RCCL all-reduce, then this rank's distance columns
            r = sharded.de_sharded(eng, ds, code, K, dist, tdev, fetch="union")
            sharded.distance_sharded(eng, ds, r.union, dist, device_out_ptr=0)
            return r
        r = eng.de_run(ds, code, K, nat.SCC_DE_FAST, fetch="union")
        eng.distance(ds, r.union, nat.SCC_DIST_PCA_EUCLID, device_out_ptr=0)
        return r

    barrier = dist.barrier

    for _ in range(a.warmup):
        r = step()
    eng.synchronize()
    eng.reset_timers()
    barrier()
    eng.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        r = step()
    eng.synchronize()
    barrier()
    t1 = time.perf_counter()
    dt = dist.max_over_ranks(t1 - t0)
    ms = dt / a.steps * 1e3
    fams = ["ingest", "gene_stats", "pair_filter", "gene_rank", "pair_test", "pair_select", "gather", "center", "gram",
            "eigen", "eig_tridiag", "eig_vec", "eig_fin", "scores", "dist"]
    times = {f: eng.kernel_time(f) for f in fams}
    stage_ms = {f: (t[0] / max(t[1], 1)) for f, t in times.items()}
    # algorithmic work per launch of each timed kernel (family): what roofline.achieved divides
    nu = len(r.union)
    nnz = d.nnz
    ncc = (d.N + 31) // 32
    alg = {
        # packed fp64 R `dist` output + the N x 16 scores read
        "dist": ("hbm", 8.0 * npairs_cells + 16 * 8.0 * d.N, "k_dist_euclid"),
        # CSC read twice (12 B/nnz + 8 B/cell), keys written once (8 B/nnz), chunk counts (4 B, 3 passes)
        "ingest": ("hbm", 2 * (12.0 * nnz + 8.0 * (d.N + 1)) + 8.0 * nnz + 3 * 4.0 * ncc * d.G, "k_ing_scatter"),
        "gene_stats": ("hbm", 8.0 * nnz + 32.0 * K * d.G, "k_gene_stats"),
        # keys read once; per (pair, gene) accumulators written (S, E, X)
        "gene_rank": ("hbm", 8.0 * nnz + 24.0 * P * d.G, "k_rank_item"),
        # Householder tridiagonalisation 4/3 n^3 fp64 flops (one hand-off per column: latency-bound)
        "eig_tridiag": ("mfma", 4.0 / 3.0 * nu ** 3, "k_tridiag"),
        "gram": ("mfma", 2.0 * d.N * nu * nu / 2, "k_gram_f64"),
    }
    dom = max(alg, key=lambda f: stage_ms.get(f, 0.0))
    traffic = None
    tpath = os.path.join(ROOT, "profiles", f"pmc_traffic_{a.config}.json")
    if os.path.exists(tpath):
        tk = json.load(open(tpath))["kernels"]
        hits = [v["traffic_bytes_per_launch"] for k, v in tk.items() if k.startswith(alg[dom][2])]
        traffic = sum(hits) if hits else None

    def roof(f):
        bound, work, kname = alg[f]
        t_s = stage_ms[f] / 1e3
        if bound == "hbm":
            ach = work / t_s / 1e9
            return {"bound": "hbm", "achieved": ach, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": ach / PEAK_HBM_GBS,
                    "kernel": kname, "bytes_per_launch": work, "avg_launch_ms": stage_ms[f]}
        ach = work / t_s / 1e12
        if bound == "mfma32":
            return {"bound": "mfma", "dtype": "f32", "achieved": ach, "peak": PEAK_FP32_TFS, "unit": "TFLOP/s",
                    "frac": ach / PEAK_FP32_TFS, "kernel": kname, "flops_per_launch": work,
                    "avg_launch_ms": stage_ms[f], "output_bytes_per_launch": 8.0 * npairs_cells}
        return {"bound": "mfma", "achieved": ach, "peak": PEAK_FP64_TFS, "unit": "TFLOP/s",
                "frac": ach / PEAK_FP64_TFS, "kernel": kname, "flops_per_launch": work, "avg_launch_ms": stage_ms[f]}

    # north_star's MFMA kernel: the Pearson 1 - cor distance (Fast:403) on the
    # same union, measured beside the step (not part of the reference's path)
    if not a.no_pearson:
        eng.distance(ds, r.union, nat.SCC_DIST_PEARSON, device_out_ptr=0)  # warm-up (first launch, buffers)
        eng.synchronize()
        eng.reset_timers()
        for _ in range(5):
            eng.distance(ds, r.union, nat.SCC_DIST_PEARSON, device_out_ptr=0)
        eng.synchronize()
        for f in ("zscore", "pearson"):
            t = eng.kernel_time(f)
            stage_ms[f] = t[0] / max(t[1], 1)
        alg["pearson"] = ("mfma32", float(d.N) * (d.N - 1) * nu, "k_pearson_mfma")

    roof_dom = roof(dom)
    roof_dom["traffic"] = traffic
    roof_dom["traffic_source"] = (f"profiles/pmc_traffic_{a.config}.json (scripts/pmc_traffic.sh)"
                                  if traffic is not None else None)
    if dom == "eig_tridiag":
        roof_dom["note"] = ("fp64 vector work on a one-stage Householder reduction: n-1 dependent "
                            "cross-workgroup hand-offs, latency-bound (no MFMA shape)")
    kernels = {f: roof(f) for f in alg if f in stage_ms and stage_ms[f] > 0}
    value = (1 if shard else world) * npairs_cells / (ms / 1e3)
    out = {
        "metric": "end-to-end DE+distance cell-pairs/sec at 26k PBMC shape",
        "value": value,
        "unit": "cell-pairs/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": ms,
        "end_to_end_s": ms / 1e3,
        "higher_is_better": True,
        "scaling": "strong" if shard else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (SURVEY §8d NB log1p generator, seed per rank)",
        "config": {"workload": f"config {a.config}: reclusterDEConsensusFast DE (all {P} pairs) + PCA15 "
                               f"Euclidean dist, {d.N} cells x {d.G} genes, K={K}",
                   "cells": d.N, "genes": d.G, "clusters": K, "pairs": P, "nnz": nnz, "union": nu,
                   "parallelism": f"shard{world}" if shard else f"jobs{world}"},
        "stage_ms": {k: round(v, 4) for k, v in stage_ms.items()},
        "roofline": roof_dom,
        "kernels": kernels,
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        ng = a.cpu_sample_genes if a.config in ("A", "B") else max(16, int(300 * 66 * 26000 / (P * d.N)))
        out["cpu_baseline"] = cpu_baseline(d, code, K, r.union, ng)
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.close()


if __name__ == "__main__":
    main()
