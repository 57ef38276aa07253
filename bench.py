#!/usr/bin/env python3
"""bench.py — headline benchmark of the scConsensus MI355X engine.

Metric (BASELINE.json): end-to-end DE + distance seconds and cell-pairs/sec at
the 26k-cell PBMC shape (config B: 26,000 cells x 10,000 genes, 12 consensus
clusters, 66 pairs), 1/2/4/8 GPUs.

One step = one pass of the hot path over one synthetic job resident in HBM:
  DE       reclusterDEConsensusFast's pair loop, all 66 pairs x all genes
           (stats, Wilcoxon, BH, filters, top-N, union; Fast:57-392)
  distance PCA(15) + packed Euclidean dist (N(N-1)/2 fp64, kept in HBM; Fast:398-400)
value = cell-pairs / second = N(N-1)/2 / step time (HBM-resident; the
transfer-inclusive times are reported beside it in "end_to_end_ms").

Multi-GPU (`--gpus N`): one process per GPU.  Without torchrun's WORLD_SIZE in
the environment, bench.py launches its own N ranks (torch.distributed.run on
127.0.0.1) before touching the GPU.  Default `--mode shard`: ONE job over all
ranks ("scaling": "strong"): gene row-blocks balanced by stored
values + one all-gather of compact tested-cell records, the PCA over cell
blocks (all-gather of column sums, all-reduce of the |U|^2 Gram and of the
disjoint score rows), then each rank's equal-entry column slice of the packed
distance.  `--mode jobs` (opt-in, "scaling": "weak"): every rank runs its own
job (seed offset by rank) with no data-path collective.  The step time is the
max over ranks.

`--route devices` measures the route R's `nCores` takes instead
(Fast:33,61-65 -> scc_opts.devices): ONE process, one engine context over a
device list (`--gpus N`: devices 0..N-1; SCC_BENCH_DEVICES="0,0" rehearses a
two-entry list on one GPU), the DE's gene blocks and the distance's column
slices spread over the list inside libscc (peer copies, no RCCL).  Under a
multi-rank launch (the driver's `--gpus N` runs) rank 0 also times this route
over all N GPUs after the rank route and reports it as "route_devices".
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0    # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PEAK_FP64_TFS = 78.6     # MI355X FP64 matrix (spec)
PEAK_FP32_TFS = 157.3    # MI355X FP32 matrix (v_mfma_f32_32x32x2_f32; MI355X_MICROARCH.md)


def _args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="B")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pearson", action="store_true", help="skip the side measurement of the Pearson kernel")
    ap.add_argument("--no-transfers", action="store_true", help="skip the D2H / H2D side measurements")
    ap.add_argument("--cpu-sample-genes", type=int, default=1500)
    ap.add_argument("--no-stage-events", action="store_true",
                    help="no per-stage HIP events in the engine (diagnostic: their cost on the step)")
    ap.add_argument("--split-calls", action="store_true",
                    help="scc_de_run then scc_distance (two C calls) instead of the fused scc_de_distance")
    ap.add_argument("--mode", choices=["shard", "jobs"], default="shard",
                    help="shard: ONE job over all ranks (strong scaling); jobs: one job per rank (weak scaling)")
    ap.add_argument("--de", choices=["fast", "slow"], default="fast",
                    help="reclusterDEConsensusFast (default) or reclusterDEConsensus (SLOW: every gene for every pair)")
    ap.add_argument("--route", choices=["ranks", "devices"], default="ranks",
                    help="ranks: one process per GPU (torch.distributed / RCCL); devices: one process over a device "
                         "list inside libscc (the R drop-in's nCores route)")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU only: the launcher / rank / timing path with a placeholder step (tests)")
    return ap.parse_args(argv)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(a) -> int:
    """Start N rank processes (torch.distributed.run, 127.0.0.1) running this
    script with the same arguments; nothing here has touched the GPU."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


DEVICE_GEN = ("C", "D", "E")


def cpu_baseline(d, code, K, union, sample_genes, seed=0):
    """The oracle (this repo's C restatement of the R algorithm, test
    infrastructure) timed on the host beside the GPU:
    * all cores: the FULL config-B DE (every gene, all pairs; genes split over
      threads -- ctypes releases the GIL) + the exact PCA + the full `dist`
      (row blocks over threads);
    * 1 thread: a seeded gene sample, scaled linearly ("extrapolated")."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import concurrent.futures as cf

    import oracle as O
    from scipy.spatial.distance import cdist
    rng = np.random.default_rng(seed)
    if not hasattr(d, "scipy_csc"):
        d = d.to_host()
    csr = d.scipy_csc().tocsr()
    threads = max(1, min(int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1), 16,
                         os.cpu_count() or 1))
    # ---- 1 thread, gene sample
    genes = np.sort(rng.choice(d.G, min(sample_genes, d.G), replace=False))
    Xs = np.asarray(csr[genes].todense())
    t0 = time.perf_counter()
    O.de_fast(Xs, code, K)
    t_de1 = (time.perf_counter() - t0) * d.G / len(genes)
    del Xs
    Xu = np.asarray(csr[union].todense())
    t0 = time.perf_counter()
    S = O.pca_scores(Xu, np.arange(len(union)))
    t_pca = time.perf_counter() - t0
    rows = rng.choice(d.N, 256, replace=False)
    t0 = time.perf_counter()
    cdist(S[rows], S, "euclidean")
    t_dist1 = (time.perf_counter() - t0) * (d.N / 2) / len(rows)
    t1 = t_de1 + t_pca + t_dist1
    # ---- all cores, full workload (config A/B sizes)
    full = d.G * d.N <= 400_000_000
    out = {"unit": "cell-pairs/s", "kind": "port"}
    if full:
        blocks = np.array_split(np.arange(d.G), threads * 8)

        def de_block(gs):
            O.de_fast(np.asarray(csr[gs].todense()), code, K)

        t0 = time.perf_counter()
        with cf.ThreadPoolExecutor(threads) as ex:
            list(ex.map(de_block, blocks))
        t_de = time.perf_counter() - t0
        t0 = time.perf_counter()
        O.pca_scores(Xu, np.arange(len(union)))
        t_pcaT = time.perf_counter() - t0
        rb = np.array_split(np.arange(d.N), threads * 4)
        t0 = time.perf_counter()
        with cf.ThreadPoolExecutor(threads) as ex:  # each block: its rows x the earlier columns
            list(ex.map(lambda r: cdist(S[r], S[: r[-1] + 1], "euclidean") if len(r) else None, rb))
        t_dist = time.perf_counter() - t0
        t = t_de + t_pcaT + t_dist
        out.update({"value": d.N * (d.N - 1) / 2 / t, "cores": threads, "end_to_end_s": t,
                    "sample": f"FULL workload on {threads} threads (not extrapolated): oracle DE over all {d.G} genes "
                              f"x {K*(K-1)//2} pairs in {len(blocks)} gene blocks, exact SVD PCA on |U|={len(union)}, "
                              f"full dist in {len(rb)} row blocks; DE {t_de:.2f} s, PCA {t_pcaT:.2f} s, "
                              f"dist {t_dist:.2f} s"})
    out["single_thread"] = {
        "value": d.N * (d.N - 1) / 2 / t1, "cores": 1, "end_to_end_s": t1, "extrapolated": True,
        "sample": f"oracle DE on {len(genes)}/{d.G} genes x all {K*(K-1)//2} pairs scaled x{d.G/len(genes):.1f}; "
                  f"exact SVD PCA on |U|={len(union)}; dist on 256/{d.N} rows scaled; est. end-to-end {t1:.1f} s "
                  f"(DE {t_de1:.1f}, PCA {t_pca:.1f}, dist {t_dist1:.1f})"}
    if not full:
        out.update({"value": out["single_thread"]["value"], "cores": 1, "end_to_end_s": t1, "extrapolated": True,
                    "sample": out["single_thread"]["sample"]})
    return out


def cold_call(d, code, K, gpu, de_mode):
    """The R drop-in's one-shot call, timed as one number, in the glue's order
    (integration/R/scConsensusAMD.R reclusterDEConsensusFast -> scc_r.c;
    Fast:22-33,398-400): the dataset created from host CSC arrays (H2D), the
    first -- validating -- scc_de_run returning the union and nodg to the
    host, then scc_distance into a fresh pageable host vector (R's
    allocVector).  "first": a new engine context (its workspace allocations,
    streams and tables; HIP itself is already initialised in this process);
    "repeat": the next call on that context with a fresh dataset (the second
    reclusterDEConsensusFast of an R session)."""
    from scconsensus_amd import _native as nat
    out = {}
    t0 = time.perf_counter()
    eng = nat.Engine(gpu)
    out["context_create"] = (time.perf_counter() - t0) * 1e3
    try:
        for tag in ("first", "repeat"):
            t0 = time.perf_counter()
            ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
            t1 = time.perf_counter()
            r = eng.de_run(ds, code, K, de_mode, fetch="nodg")
            t2 = time.perf_counter()
            host = np.empty(d.N * (d.N - 1) // 2, np.float64)
            eng.distance(ds, r.union, nat.SCC_DIST_PCA_EUCLID, out=host)
            t3 = time.perf_counter()
            ds.close()
            out[tag] = {"total": (t3 - t0) * 1e3, "dataset_h2d": (t1 - t0) * 1e3, "de_to_host": (t2 - t1) * 1e3,
                        "distance_to_pageable_host": (t3 - t2) * 1e3}
            del host
    finally:
        eng.close()
    out["first_including_context"] = out["context_create"] + out["first"]["total"]
    out["note"] = ("ms; each leg ends with its result on the host (the glue's .Call boundaries); "
                   "value stays the warmed HBM-resident step")
    return out


def de_only(a, eng, ds, d, code, K, dist, world, dataset_ms=None):
    """Config E (BASELINE: "1M-cell sparse CSR input, 100 clusters (4950
    pairs), DE-only"): the FAST DE over all pairs, rows fetched to the host."""
    from scconsensus_amd import _native as nat

    def step():  # ONE scc_de_run (any K: group-pair runs past 128 clusters happen inside libscc)
        return eng.de_run(ds, code, K, nat.SCC_DE_FAST, fetch="rows")

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
        stage_ms[f] = round(t / max(a.steps, 1), 3)  # per step (one engine run, one launch of each stage)
    P = K * (K - 1) // 2
    nnz, G, N = d.nnz, d.G, d.N
    ncc = (N + 31) // 32
    # SURVEY §8(d)'s algorithmic bytes per launch (the same accounting as the
    # DE + distance line): B_DE = X read once (CSC: 12 B per stored value +
    # 8 B per cell) + 4 N (codes) + 24 K G (cnt, S_expm1, S_x) + 16 P G (2U + p)
    alg = {
        "ingest": (12.0 * nnz + 8.0 * (N + 1) + 8.0 * nnz + 3 * 4.0 * ncc * G,
                   "ingest stage (k_ing_hist, k_ing_colsum/segscan/colapply, scans, k_ing_scatter)"),
        "gene_stats": (8.0 * nnz + 32.0 * K * G, "k_gene_stats"),
        "gene_rank": (8.0 * nnz + 24.0 * P * G,
                      "rank stage (k_rank_classify/split/resplit/waves/cross; k_rank_item on a second stream)"),
    }
    kernels = {}
    for f, (work, kname) in alg.items():
        if stage_ms.get(f, 0.0) > 0.0:
            ach = work / (stage_ms[f] / 1e3) / 1e9
            kernels[f] = {"bound": "hbm", "achieved": ach, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                          "frac": ach / PEAK_HBM_GBS, "kernel": kname, "bytes_per_launch": work,
                          "avg_launch_ms": stage_ms[f]}
    b_de = 12.0 * nnz + 8.0 * (N + 1) + 4.0 * N + 24.0 * K * G + 16.0 * P * G
    ach = b_de / s_step / 1e9
    kernels["de_total"] = {"bound": "hbm", "achieved": ach, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                           "frac": ach / PEAK_HBM_GBS, "kernel": "the whole DE step (B_DE over the step time)",
                           "bytes_per_launch": b_de, "avg_launch_ms": s_step * 1e3}
    dom = max(alg, key=lambda f: stage_ms.get(f, 0.0))
    roof = dict(kernels.get(dom, {"bound": "hbm", "achieved": None, "kernel": alg[dom][1]}))
    roof["traffic"] = None
    tpath = os.path.join(ROOT, "profiles", "pmc_traffic_E.json")
    if os.path.exists(tpath):
        tk = json.load(open(tpath))["kernels"]
        pref = {"gene_rank": "k_rank", "ingest": "k_ing", "gene_stats": "k_gene_stats"}[dom]
        hits = [v["traffic_bytes_per_launch"] for k, v in tk.items() if k.startswith(pref)]
        roof["traffic"] = sum(hits) if hits else None
        roof["traffic_source"] = "profiles/pmc_traffic_E.json (scripts/pmc_traffic.sh E)"
    roof["note"] = "avg_launch_ms is the whole stage (its kernels back to back), not one kernel"
    out = {"metric": "DE-only seconds per reclusterDEConsensusFast DE at config E", "value": s_step, "unit": "s",
           "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "ms_per_step": s_step * 1e3,
           "higher_is_better": False, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
           "scaling_note": "N > 1: one independent config-E job per rank (no data-path collective)",
           "data": "synthetic (SURVEY §8d generator on the GPU, gene-major CSR)",
           "config": {"workload": f"config E: FAST DE (all {P} pairs, Wilcoxon), {d.N} cells x {d.G} genes CSR, K={K}",
                      "cells": d.N, "genes": d.G, "clusters": K, "pairs": P, "nnz": d.nnz,
                      "union": len(r.union), "rows": int(len(r.rows.gene)),
                      "engine_runs_per_step": 1 if K <= 128 else (-(-K // 64)) * (-(-K // 64) - 1) // 2,
                      "parallelism": f"jobs{world}" if world > 1 else "single"},
           "stage_ms_per_step": stage_ms, "roofline": roof, "kernels": kernels}
    if dataset_ms:
        # the CSR -> CSC build: minimum traffic = the CSR read once (12 B per
        # stored value + 8 B per gene) + the CSC written once (12 B per stored
        # value + 8 B per cell)
        t_b = sum(dataset_ms[1:]) / max(1, len(dataset_ms) - 1)
        mn = 12.0 * nnz + 8.0 * (G + 1) + 12.0 * nnz + 8.0 * (N + 1)
        dsb = {"first_ms": dataset_ms[0], "ms": t_b, "runs_ms": dataset_ms,
               "min_bytes": mn, "achieved_gbs": mn / (t_b / 1e3) / 1e9,
               "frac": mn / (t_b / 1e3) / 1e9 / PEAK_HBM_GBS,
               "note": "scc_dataset_create_csr_device wall time (synchronised), CSR -> resident CSC; not in value"}
        if os.path.exists(tpath):
            tk = json.load(open(tpath))["kernels"]
            hits = {k: v["traffic_bytes_per_launch"] for k, v in tk.items() if k.startswith("k_ct_")}
            if hits:
                dsb["traffic"] = sum(hits.values())
                dsb["traffic_kernels"] = hits
                dsb["traffic_vs_min"] = sum(hits.values()) / mn
        out["dataset_ms"] = dsb
        out["de_plus_dataset_ms"] = s_step * 1e3 + t_b
    if dist.rank == 0:
        print(json.dumps(out), flush=True)
    dist.close()


def dry_run(a, dist):
    """CPU rehearsal of the launcher / rank / timing path (tests)."""
    def step():
        time.sleep(0.002 * (1 + dist.rank))

    for _ in range(a.warmup):
        step()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    dist.barrier()
    dt = dist.max_over_ranks(time.perf_counter() - t0)
    shard = a.mode == "shard"
    out = {"metric": "dry run", "value": 0.0, "n_gpus": dist.world, "steps": a.steps, "warmup": a.warmup,
           "ms_per_step": dt / a.steps * 1e3, "scaling": "strong" if shard else "weak", "dry_run": True,
           "config": {"parallelism": f"{'shard' if shard else 'jobs'}{dist.world}"}}
    if dist.rank == 0:
        print(json.dumps(out), flush=True)
    dist.close()


def _device_list(a):
    env = os.environ.get("SCC_BENCH_DEVICES")
    if env:
        return [int(x) for x in env.split(",") if x.strip() != ""]
    return list(range(a.gpus))


def devices_route(a, d, code, K, devices, steps, warmup):
    """One process, one context over `devices` (scc_opts.devices): the fused
    DE + distance step with the distance kept in HBM, timed like the main
    line (synchronize on both sides)."""
    from scconsensus_amd import _native as nat
    eng = nat.Engine(devices[0], devices=devices if len(devices) > 1 else None)
    try:
        if hasattr(d.indptr, "data_ptr"):
            ds = eng.dataset_csc_device(d.indptr.data_ptr(), d.indices.data_ptr(), d.data.data_ptr(), d.G, d.N, d.nnz)
        else:
            ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)

        mode = nat.SCC_DE_SLOW if getattr(a, "de", "fast") == "slow" else nat.SCC_DE_FAST

        def step():
            return eng.de_distance(ds, code, K, mode, nat.SCC_DIST_PCA_EUCLID, device_out_ptr=0)[0]

        for _ in range(max(1, warmup)):
            r = step()
        eng.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            r = step()
        eng.synchronize()
        ms = (time.perf_counter() - t0) / steps * 1e3
        ds.close()
    finally:
        eng.close()
    n_dev = len(set(devices))
    return {"route": "devices", "devices": devices, "n_gpus": n_dev, "ms_per_step": ms,
            "value": d.N * (d.N - 1) / 2 / (ms / 1e3), "unit": "cell-pairs/s", "union": len(r.union),
            "parallelism": f"devices{len(devices)}" + (f" on {n_dev} GPU(s)" if n_dev != len(devices) else "")}


def main():
    a = _args()
    if a.route == "devices" and "WORLD_SIZE" not in os.environ:
        a.mode = "shard"
    elif a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a))
    shard = a.mode == "shard"
    if shard and not a.dry_run:
        import torch  # noqa: F401  (torch's HIP runtime first: the shard buffers are torch tensors)
    from scconsensus_amd import parallel
    # RCCL ("nccl") when launched with N > 1 GPUs.  SCC_SHARE_GPU=1 with
    # SCC_DIST_BACKEND=gloo rehearses several ranks on one GPU (tests only).
    dist = parallel.init(os.environ.get("SCC_DIST_BACKEND") or ("gloo" if a.dry_run else None))
    rank, world, local = dist.rank, dist.world, dist.local_rank
    route_devices = a.route == "devices" and world == 1
    if world != a.gpus and not route_devices:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}")
    devices = _device_list(a) if route_devices else [0]
    if a.dry_run:
        return dry_run(a, dist)
    from scconsensus_amd import _native as nat
    from scconsensus_amd import api, synth
    from scconsensus_amd.synth import CONFIGS

    cfg = CONFIGS[a.config]
    seed = cfg["seed"] if shard else parallel.job_seed(cfg["seed"], rank)
    gpu = 0 if os.environ.get("SCC_SHARE_GPU") else local
    h2d_ms = None
    if a.config in DEVICE_GEN:  # C/D/E: generated in HBM (host generation takes minutes)
        import torch
        d = synth.generate_device(a.config, f"cuda:{gpu}", seed=seed, layout="csr" if a.config == "E" else "csc")
        torch.cuda.synchronize()
    else:
        d = synth.generate(a.config, seed=seed)
    names, code = api.select_clusters(d.labels, 10)
    K = len(names)
    P = K * (K - 1) // 2
    eng = nat.Engine(gpu, profile=not a.no_stage_events,
                     devices=devices if route_devices and len(devices) > 1 else None)
    if a.config == "E":
        # the gene-major CSR is transposed into the resident CSC when the
        # dataset is created (k_ct_bounds / k_ct_tiles / k_ct_pass1 / k_ct_pass2): an R call on a
        # dgRMatrix pays it once per call, so it is timed and reported beside
        # the DE (first build: allocations; then the mean of repeated builds)
        build = []
        for i in range(3):
            eng.synchronize()
            t0 = time.perf_counter()
            ds = eng.dataset_csr_device(d.indptr.data_ptr(), d.indices.data_ptr(), d.data.data_ptr(), d.G, d.N,
                                        d.nnz)
            eng.synchronize()
            build.append((time.perf_counter() - t0) * 1e3)
            if i < 2:
                ds.close()
        return de_only(a, eng, ds, d, code, K, dist, world, dataset_ms=build)
    if a.config in DEVICE_GEN:
        ds = eng.dataset_csc_device(d.indptr.data_ptr(), d.indices.data_ptr(), d.data.data_ptr(), d.G, d.N, d.nnz)
    else:
        ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)  # warm-up upload (allocations, first touch)
        ds.close()
        t0 = time.perf_counter()
        ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)  # input H2D: before the timed region
        h2d_ms = (time.perf_counter() - t0) * 1e3
    npairs_cells = d.N * (d.N - 1) / 2
    multi = shard and world > 1
    if multi:
        import torch
        from scconsensus_amd import sharded
        tdev = torch.device(f"cuda:{gpu}")
        if a.config in DEVICE_GEN:
            gene_w = torch.bincount(d.indices.to(torch.int64), minlength=d.G).cpu().numpy()
        else:
            gene_w = np.bincount(d.indices, minlength=d.G)

    de_mode = nat.SCC_DE_SLOW if a.de == "slow" else nat.SCC_DE_FAST

    def step(dist_out=0):
        """dist_out 0: the distance stays in HBM; a host array: streamed into it."""
        if multi:  # one job: gene row-blocks + record all-gather, PCA over cell blocks, this rank's columns
            r = sharded.de_sharded(eng, ds, code, K, dist, tdev, fetch="union", weights=gene_w, mode=de_mode)
            if dist_out is None or isinstance(dist_out, int):
                sharded.distance_sharded(eng, ds, r.union, dist, tdev, device_out_ptr=0)
            else:
                scores = sharded.pca_sharded(eng, ds, r.union, dist, tdev)
                lo, hi = sharded.column_shard(ds.N, dist.rank, dist.world)
                eng.distance_scores(scores.data_ptr(), ds.N, lo, hi, out=dist_out[: hi * (2 * ds.N - hi - 1) // 2
                                                                                 - lo * (2 * ds.N - lo - 1) // 2])
            return r
        if a.split_calls:  # scc_de_run, then scc_distance on the returned union
            r = eng.de_run(ds, code, K, de_mode, fetch="union")
            if isinstance(dist_out, int):
                eng.distance(ds, r.union, nat.SCC_DIST_PCA_EUCLID, device_out_ptr=0)
            else:
                eng.distance(ds, r.union, nat.SCC_DIST_PCA_EUCLID, out=dist_out)
            return r
        # scc_de_distance: the same two stages in one C call
        if isinstance(dist_out, int):
            r, _ = eng.de_distance(ds, code, K, de_mode, nat.SCC_DIST_PCA_EUCLID, device_out_ptr=0)
        else:
            r, _ = eng.de_distance(ds, code, K, de_mode, nat.SCC_DIST_PCA_EUCLID, out=dist_out)
        return r

    def timed(nsteps, **kw):
        eng.synchronize()
        dist.barrier()
        eng.synchronize()
        t0 = time.perf_counter()
        for _ in range(nsteps):
            r = step(**kw)
        eng.synchronize()
        dist.barrier()
        return r, dist.max_over_ranks(time.perf_counter() - t0) / nsteps * 1e3

    # Warm-up: the first step allocates; the others time every stage (HIP
    # events around each stage: the per-stage table).  An event between two
    # kernels leaves the GPU idle ~12 us (0.14 ms per config-B step with every
    # stage timed), so the timed region then brackets only the dominant stage.
    fams = ["ingest", "gene_stats", "pair_filter", "gene_rank", "pair_test", "pair_select", "gather", "center", "gram",
            "eigen", "eig_tridiag", "eig_vec", "eig_fin", "scores", "dist"]
    os.environ.pop("SCC_PROFILE_STAGES", None)
    r = step()
    eng.synchronize()
    eng.reset_timers()
    nprof = max(1, a.warmup - 1)
    for _ in range(nprof):
        r = step()
    eng.synchronize()
    times = {f: eng.kernel_time(f) for f in fams}
    stage_ms = {f: (t[0] / max(t[1], 1)) for f, t in times.items()}
    # algorithmic work per launch of each timed kernel (family): what roofline.achieved divides
    nu = len(r.union)
    nnz = d.nnz
    ncc = (d.N + 31) // 32
    # a rank's (or, on the device-list route, a device's) share of the packed
    # output: equal-entry column slices, one launch per slice
    ndev_route = len(devices) if route_devices else 1
    frac_entries = 1.0 / world if multi else 1.0 / ndev_route
    nshare = world if multi else ndev_route  # gene blocks / Gram shards per launch
    alg = {
        # packed fp64 R `dist` output + the N x 16 scores read
        "dist": ("hbm", 8.0 * npairs_cells * frac_entries + 16 * 8.0 * d.N, "k_dist_aligned"),
        # the minimum: CSC read once (12 B/nnz + 8 B/cell), keys written once (8 B/nnz), chunk counts (4 B,
        # 3 passes); the kernels read the CSC twice (count, then scatter), which this does not credit
        "ingest": ("hbm", (12.0 * nnz + 8.0 * (d.N + 1)) + 8.0 * nnz / nshare + 3 * 4.0 * ncc * d.G / nshare,
                   "ingest stage (k_ing_hist, k_ing_colsum/segscan/colapply, scans, k_ing_scatter)"),
        "gene_stats": ("hbm", (8.0 * nnz + 32.0 * K * d.G) / nshare, "k_gene_stats"),
        # keys read once; per (pair, gene) accumulators written (S, E, X)
        "gene_rank": ("hbm", (8.0 * nnz + 24.0 * P * d.G) / nshare,
                      "rank stage (k_rank_classify/split/resplit/waves/cross; k_rank_item on a second stream)"),
        # Householder tridiagonalisation 4/3 n^3 fp64 flops (one hand-off per column: latency-bound)
        "eig_tridiag": ("mfma", 4.0 / 3.0 * nu ** 3, "k_tridiag"),
        "gram": ("mfma", 2.0 * d.N * nu * nu / 2 / (world if multi else 1), "k_gram_f64"),  # one device on the list route
    }
    if 128 <= nu <= 1024 and stage_ms.get("eig_vec", 0.0) < 0.02:
        # the filtered subspace iteration in one persistent launch answered
        # (scc_subspace.hip k_fsi_engine): 5 segments of 8 products + the
        # Rayleigh-Ritz product of C (n x n) by the 64-column block, 13 Grams
        # of the block; no k_tridiag at size n
        alg["eig_tridiag"] = ("mfma", 41 * 2.0 * nu * nu * 64 + 13 * 2.0 * nu * 64 * 64,
                              "eigen stage: filtered subspace iteration in one persistent launch (k_fsi_engine: "
                              "41 block products, 12 CholQR passes, Rayleigh-Ritz and the guard)")
    elif nu >= 400 and stage_ms.get("eig_vec", 0.0) < 0.02:
        # (eig_vec is the gap between two events recorded back to back when the
        # subspace iteration answered: a few microseconds, never the 0.3+ ms of
        # the direct solver's vectors)
        # the subspace iteration answered (scc_subspace.hip, |U| >= 400): 31 products of
        # C (n x n) by the 64-column block + the n = 64 Rayleigh-Ritz; no k_tridiag at size n
        alg["eig_tridiag"] = ("mfma", 31 * 2.0 * nu * nu * 64,
                              "eigen stage: block subspace iteration (k_si_mul/gram/cholinv/apply, "
                              "Rayleigh-Ritz through the direct solver at n = 64)")
    dom = max(alg, key=lambda f: stage_ms.get(f, 0.0))
    # the timed region: HIP events around the dominant stage only
    os.environ["SCC_PROFILE_STAGES"] = dom
    eng.reset_timers()
    r, ms = timed(a.steps)
    t_dom = eng.kernel_time(dom)
    stage_ms_warmup_dom = stage_ms[dom]
    stage_ms[dom] = t_dom[0] / max(t_dom[1], 1)
    os.environ["SCC_PROFILE_STAGES"] = "-"  # the side measurements below: no stage events
    traffic = None
    # counters of THIS DE mode only (a SLOW line never borrows FAST's kernels' traffic)
    ttag = a.config + ("_slow" if a.de == "slow" else "")
    tpath = os.path.join(ROOT, "profiles", f"pmc_traffic_{ttag}.json")
    if os.path.exists(tpath) and not multi:
        tk = json.load(open(tpath))["kernels"]
        kpre = {"dist": "k_dist", "ingest": "k_ing", "gene_stats": "k_gene_stats", "gene_rank": "k_rank",
                "gram": "k_gram", "eig_tridiag": "k_fsi_engine" if "k_fsi_engine" in alg[dom][2] else "k_tridiag"}
        hits = [v["traffic_bytes_per_launch"] for k, v in tk.items() if k.startswith(kpre.get(dom, alg[dom][2]))]
        traffic = sum(hits) if hits else None

    def roof(f):
        bound, work, kname = alg[f]
        t_s = stage_ms[f] / 1e3
        if t_s <= 0.0:  # --no-stage-events: no per-kernel times
            return {"bound": bound, "achieved": None, "kernel": kname}
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

    # transfers beside the HBM-resident step: the packed dist streamed to host
    # memory (pageable: the pinned staging ring; pinned: direct DMA), and the
    # input's H2D upload (host-generated configs)
    e2e = {"hbm_resident": ms, "value_uses": "hbm_resident"}
    if not a.no_transfers:
        import torch
        nloc = npairs_cells if not multi else (lambda lo, hi: hi * (2 * d.N - hi - 1) // 2 - lo * (2 * d.N - lo - 1) // 2)(
            *sharded.column_shard(d.N, rank, world))
        host = np.empty(int(nloc), np.float64)
        host[::4096] = 0.0  # first touch outside the timed steps
        step(dist_out=host)
        _, e2e["with_dist_d2h_pageable"] = timed(max(1, min(a.steps, 3)), dist_out=host)
        del host
        pin = torch.empty(int(nloc), dtype=torch.float64, pin_memory=True).numpy()
        step(dist_out=pin)
        _, e2e["with_dist_d2h_pinned"] = timed(max(1, min(a.steps, 3)), dist_out=pin)
        del pin
        e2e["dist_gb"] = 8.0 * nloc / 1e9
        e2e["d2h_gbs_pinned"] = 8.0 * nloc / 1e9 / max(1e-9, (e2e["with_dist_d2h_pinned"] - ms) / 1e3)
        if h2d_ms is not None:
            e2e["input_h2d"] = h2d_ms
            e2e["with_input_h2d_and_dist_d2h_pinned"] = h2d_ms + e2e["with_dist_d2h_pinned"]

    # north_star's MFMA kernel: the Pearson 1 - cor distance (Fast:403) on the
    # same union, measured beside the step (not part of the reference's path)
    if not a.no_pearson and not multi:
        os.environ["SCC_PROFILE_STAGES"] = "zscore,pearson"
        # warm-up: the first launch allocates; the GPU sat idle through the
        # PCIe-bound transfer measurements before this, so a few more launches
        # bring the clocks back before the timed ones (1 warm-up launch gave
        # 0.57-0.63 of peak run to run on the same binary; 6 gave 0.61-0.66):
        # launches for at least a quarter of a second, then 20 timed
        t_w = time.perf_counter()
        for i in range(1000):
            eng.distance(ds, r.union, nat.SCC_DIST_PEARSON, device_out_ptr=0)
            if i >= 5 and i % 4 == 3:
                eng.synchronize()
                if time.perf_counter() - t_w > 0.25:
                    break
        eng.synchronize()
        eng.reset_timers()
        for _ in range(20):
            eng.distance(ds, r.union, nat.SCC_DIST_PEARSON, device_out_ptr=0)
        eng.synchronize()
        for f in ("zscore", "pearson"):
            t = eng.kernel_time(f)
            stage_ms[f] = t[0] / max(t[1], 1)
        alg["pearson"] = ("mfma32", float(d.N) * (d.N - 1) * nu, "k_pearson_mfma")

    cold = None
    if not a.no_transfers and world == 1 and not route_devices and a.config not in DEVICE_GEN:
        cold = cold_call(d, code, K, gpu, de_mode)

    roof_dom = roof(dom)
    roof_dom["traffic"] = traffic
    roof_dom["traffic_source"] = (f"profiles/pmc_traffic_{ttag}.json (scripts/pmc_traffic.sh {a.config} {a.de})"
                                  if traffic is not None else None)
    if alg[dom][2].endswith("stage") or " stage" in alg[dom][2]:
        roof_dom["note"] = "avg_launch_ms is the whole stage (its kernels back to back), not one kernel"
    elif dom == "eig_tridiag":
        roof_dom["note"] = ("fp64 vector work on a one-stage Householder reduction: n-1 dependent "
                            "cross-workgroup hand-offs, latency-bound (no MFMA shape)")
    kernels = {f: roof(f) for f in alg if f in stage_ms and stage_ms[f] > 0}
    jobs = world if not shard else 1
    value = jobs * npairs_cells / (ms / 1e3)
    side_devices = None
    if world > 1 and shard and a.config in ("A", "B", "C", "D"):
        # the R drop-in's route over the same N GPUs: rank 0 alone drives a
        # device list [0 .. N-1] (the other ranks wait at the barrier)
        dist.barrier()
        if rank == 0:
            try:
                side_devices = devices_route(a, d, code, K, list(range(world)), max(1, min(a.steps, 10)), a.warmup)
            except Exception as ex:  # reported, never silently dropped
                side_devices = {"route": "devices", "error": repr(ex)}
        dist.barrier()
    out = {
        "metric": f"end-to-end DE+distance cell-pairs/sec at config {a.config}"
                  + (" (26k PBMC shape)" if a.config == "B" else "") + (" [SLOW DE]" if a.de == "slow" else ""),
        "value": value,
        "unit": "cell-pairs/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": ms,
        "end_to_end_s": ms / 1e3,
        "end_to_end_ms": e2e,
        "higher_is_better": True,
        "scaling": "strong" if shard else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (SURVEY §8d NB log1p generator" + (", seed per rank)" if not shard else ")"),
        "config": {"workload": f"config {a.config}: reclusterDEConsensus{'' if a.de == 'slow' else 'Fast'} DE "
                               f"(all {P} pairs) + PCA15 "
                               f"Euclidean dist, {d.N} cells x {d.G} genes, K={K}",
                   "cells": d.N, "genes": d.G, "clusters": K, "pairs": P, "nnz": nnz, "union": nu,
                   "parallelism": (f"devices{len(devices)}" if route_devices and len(devices) > 1
                                   else (f"shard{world}" if shard else f"jobs{world}"))},
        "route": "devices" if route_devices else "ranks",
        "stage_ms": {k: round(v, 4) for k, v in stage_ms.items()},
        "stage_ms_source": (f"{dom}: HIP events over the timed region (the only stage timed there); the others: "
                            f"{nprof} warm-up step(s) with every stage timed (each event adds ~12 us of GPU idle, "
                            f"so those steps are not the timed ones); {dom} in those steps: "
                            f"{stage_ms_warmup_dom:.4f} ms"),
        "roofline": roof_dom,
        "kernels": kernels,
    }
    if route_devices:
        out["devices"] = devices
        out["n_gpus"] = len(set(devices))
    if side_devices is not None:
        out["route_devices"] = side_devices
    if cold is not None:
        out["cold_call_ms"] = cold
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        ng = a.cpu_sample_genes if a.config in ("A", "B") else max(16, int(300 * 66 * 26000 / (P * d.N)))
        out["cpu_baseline"] = cpu_baseline(d, code, K, r.union, ng)
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.close()


if __name__ == "__main__":
    main()
