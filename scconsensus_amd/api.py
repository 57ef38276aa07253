"""Host-side mirror of the reference R API (same names, argument meaning and
error behaviour), running the data-parallel core on the MI355X engine.

Reference signatures:
  reclusterDEConsensusFast(dataMatrix, consensusClusterLabels, method = "wilcox",
      qValThrs = 0.1, logFCThrs = 0.5, deepSplitValues = 1:4, minClusterSize = 10,
      minPerCent = 20, filename = "de_gene_object.rds", plotName = "DE_Heatmap",
      NumbertopDEGenes = 30, nCores = 1)              R/reclusterDEConsensusFast.R:22-33
  reclusterDEConsensus(dataMatrix, consensusClusterLabels, method = "Wilcoxon",
      meanScalingFactor = 5, qValThrs, fcThrs, deepSplitValues = 1:4,
      minClusterSize = 10, filename = "de_gene_object.rds", plotName = "DE_Heatmap")
                                                       R/reclusterDEConsensus.R:20-29

What runs where: cluster selection (A0), printing and the
saved object stay on the host like in R; the pairwise DE, BH/filters/union and
the distance matrix run in libscc on the GPU; hclust(ward.D2), cutreeDynamic
(hybrid, pamStage = FALSE) and labels2colors run on the host as the reference
keeps them there (libscc's host functions scc_hclust_ward_d2 /
scc_cutree_hybrid).  The ComplexHeatmap plot is not part of
this engine; ``plotName`` is ignored.
"""
from __future__ import annotations

import numpy as np

from . import _native as nat

_ENGINES: dict = {}


def _engine(device: int = 0) -> nat.Engine:
    if device not in _ENGINES:
        _ENGINES[device] = nat.Engine(device)
    return _ENGINES[device]


def select_clusters(labels, min_cluster_size: int, cluster_order=None):
    """A0 (Fast:40-53, slow:39-54): table(labels); keep count > minClusterSize;
    drop names containing "grey".  Returns (names, code[N]) with code = -1 for
    cells not compared.  R orders table() names by the locale's collation;
    the default here is code-point order (R's C locale) — pass
    ``cluster_order`` to reproduce another collation."""
    raw = np.asarray(labels, dtype=object)
    # R's table() drops NA and `labels == x` never matches NA (Fast:40-44): a
    # missing label (None / NaN / pandas NA) is no cluster, its cell coded -1
    missing = np.fromiter((_is_missing(v) for v in raw), bool, len(raw))
    labels = raw.astype(str)
    names, counts = np.unique(labels[~missing], return_counts=True)
    if cluster_order is not None:
        pos = {n: i for i, n in enumerate(cluster_order)}
        idx = sorted(range(len(names)), key=lambda i: pos.get(names[i], len(pos) + i))
        names, counts = names[idx], counts[idx]
    keep = [str(n) for n, c in zip(names, counts) if c > min_cluster_size and "grey" not in str(n)]
    lut = {n: i for i, n in enumerate(keep)}
    code = np.fromiter((lut.get(s, -1) for s in labels), np.int32, len(labels))
    code[missing] = -1
    return keep, code


def _is_missing(v) -> bool:
    if v is None:
        return True
    if isinstance(v, (float, np.floating)):
        return bool(np.isnan(v))
    try:
        import pandas as pd
        return v is pd.NA or v is pd.NaT
    except ImportError:  # pragma: no cover
        return False


def _as_matrix(dataMatrix):
    """Accept scipy.sparse (genes x cells), numpy dense (genes x cells) or a
    synth.Dataset; return ('csc' | 'csr', indptr, idx, vals, G, N) or ('dense', X)."""
    try:
        import scipy.sparse as sp
        if sp.issparse(dataMatrix) and dataMatrix.format == "csr":  # gene-major: transposed on the device
            m = dataMatrix.copy() if not dataMatrix.has_sorted_indices else dataMatrix
            m.sort_indices()
            return "csr", m.indptr.astype(np.int64), m.indices.astype(np.int32), m.data.astype(np.float64), \
                m.shape[0], m.shape[1]
        if sp.issparse(dataMatrix):
            m = dataMatrix.tocsc()
            m.sort_indices()
            return "csc", m.indptr.astype(np.int64), m.indices.astype(np.int32), m.data.astype(np.float64), \
                m.shape[0], m.shape[1]
    except ImportError:  # pragma: no cover
        pass
    if hasattr(dataMatrix, "indptr") and hasattr(dataMatrix, "labels"):
        d = dataMatrix
        return "csc", d.indptr, d.indices, d.data, d.G, d.N
    X = np.asarray(dataMatrix, np.float64)
    return "dense", X


def _upload(eng, m):
    if m[0] == "csc":
        _, indptr, rows, vals, G, N = m
        return eng.dataset_csc(indptr, rows, vals, G, N)
    if m[0] == "csr":
        _, indptr, cols, vals, G, N = m
        return eng.dataset_csr(indptr, cols, vals, G, N)
    return eng.dataset_dense(m[1])


# WGCNA standardColors(): the 34 base colours (labels2colors' palette for
# labels 1..34).  WGCNA extends the list with the rest of R's colors() in a
# fixed pseudo-random order; R is absent here, so labels above 34 use the
# first entries of that extension as recalled (unpinned) and then "colorK".
STANDARD_COLORS = [
    "turquoise", "blue", "brown", "yellow", "green", "red", "black", "pink", "magenta", "purple", "greenyellow",
    "tan", "salmon", "cyan", "midnightblue", "lightcyan", "grey60", "lightgreen", "lightyellow", "royalblue",
    "darkred", "darkgreen", "darkturquoise", "darkgrey", "orange", "darkorange", "white", "skyblue", "saddlebrown",
    "steelblue", "paleturquoise", "violet", "darkolivegreen", "darkmagenta",
    "sienna3", "yellowgreen", "skyblue3", "plum1", "orangered4", "mediumpurple3", "lightsteelblue1", "lightcyan1",
    "ivory", "floralwhite", "darkorange2", "brown4", "bisque4", "darkslateblue", "plum2", "thistle2", "thistle1",
    "salmon4", "palevioletred3", "navajowhite2", "maroon", "lightpink4", "lavenderblush3", "honeydew1",
    "darkseagreen4", "coral1", "antiquewhite4", "coral2", "mediumorchid", "skyblue2", "yellow4", "skyblue1", "plum",
    "orangered3", "mediumpurple2", "lightsteelblue", "lightcoral", "indianred4", "firebrick4", "darkolivegreen4",
    "brown2", "blue2", "darkviolet", "plum3", "thistle3", "thistle",
]


def labels2colors(labels):
    """WGCNA::labels2colors(labels) for numeric labels (Fast:428): 0 -> "grey",
    k -> standardColors()[k]."""
    lab = np.asarray(labels)
    return [("grey" if v == 0 else STANDARD_COLORS[v - 1] if v <= len(STANDARD_COLORS) else f"color{v}")
            for v in lab.tolist()]


def _hclust_ward_d2(dist_packed, N):
    """fastcluster::hclust(d, "ward.D2") (Fast:406-411) -> R hclust fields."""
    merge, height, order = nat.hclust_ward_d2(dist_packed, N)
    return {"merge": merge, "height": height, "order": order, "method": "ward.D2", "dist.method": "euclidean"}


def _dynamic_colors(tree, dist_packed, deepSplitValues, minClusterSize, eng=None, info=None):
    """Fast:418-431: cutreeDynamic(dendro, distM = as.matrix(d), deepSplit = dsv,
    pamStage = FALSE, minClusterSize) -> labels2colors, named "deepsplit: dsv".
    With ``eng`` (FAST, which computes the silhouette for every deepSplit):
    R's stop when a deepSplit yields < 2 groups; with a list ``info`` too, the
    reference's deepSplitInfo rows
    (Fast:433: DeepSplit, NumbersOfClusters, SI = mean of
    summary(cluster::silhouette(groups, as.matrix(d)))$clus.avg.widths), the
    silhouette computed by the engine on its HBM-resident copy of d."""
    out = {}
    N = len(tree["order"])
    for dsv in deepSplitValues:
        lab, _ = nat.cutree_hybrid(tree["merge"], tree["height"], dist_packed, int(dsv), int(minClusterSize))
        out[f"deepsplit: {dsv}"] = labels2colors(lab)
        if eng is not None:
            lab = np.asarray(lab, np.int32)
            k = len(np.unique(lab))
            if not 2 <= k < N:
                # silhouette() returns NA and summary(NA)$clus.avg.widths stops (Fast:433)
                raise RuntimeError("$ operator is invalid for atomic vectors (silhouette of "
                                   f"{k} group(s) at deepSplit {dsv}, Fast:433)")
            if info is not None:  # the SI the reference computes and discards
                info.append({"DeepSplit": dsv, "NumbersOfClusters": k,
                             "SI": float(np.mean(eng.silhouette(N, lab)[1]))})
    return out


def _save(obj, filename):
    if not filename:
        return
    import pickle
    with open(filename if filename.endswith(".pkl") else filename + ".pkl", "wb") as f:
        pickle.dump(obj, f)


def reclusterDEConsensusFast(dataMatrix, consensusClusterLabels, method="wilcox", qValThrs=0.1, logFCThrs=0.5,
                             deepSplitValues=(1, 2, 3, 4), minClusterSize=10, minPerCent=20,
                             filename="de_gene_object.rds", plotName="DE_Heatmap", NumbertopDEGenes=30, nCores=1,
                             *, gene_names=None, cluster_order=None, device=0, save=False, return_details=False):
    if method not in ("wilcox", "t"):
        # Fast:306-333: "bimod"/"roc" need Seurat helpers the reference never loads
        raise NotImplementedError(f"Unknown test: {method} (this engine implements test.use = 'wilcox' and 't')")
    eng = _engine(device)
    m = _as_matrix(dataMatrix)
    N = m[-1] if m[0] in ("csc", "csr") else m[1].shape[1]
    G = m[-2] if m[0] in ("csc", "csr") else m[1].shape[0]
    names, code = select_clusters(consensusClusterLabels, minClusterSize, cluster_order)
    if len(names) < 2:
        raise ValueError("need at least two clusters with > minClusterSize cells")
    ds = _upload(eng, m)
    # any K: more than 128 clusters run as group-pair runs inside libscc (scc_de_run)
    res = eng.de_run(ds, code, len(names), nat.SCC_DE_FAST, q_val_thrs=qValThrs, log_fc_thrs=logFCThrs,
                     min_per_cent=float(minPerCent), top_n=NumbertopDEGenes,
                     fetch="rows" if return_details else "union", test=method)
    if res.status == nat.SCC_ERR_RSTOP:
        raise RuntimeError(res.message)
    uni = res.union
    gnames = np.asarray(gene_names if gene_names is not None else [f"gene{g}" for g in range(G)], dtype=object)
    print(f" chr [1:{len(uni)}] " + " ".join(f'"{g}"' for g in gnames[uni[:5]]) + (" ..." if len(uni) > 5 else ""))
    if len(uni) == 0:
        raise RuntimeError("no DE genes (R fails on an empty deGenes data frame, Fast:386)")
    d = eng.distance(ds, uni, nat.SCC_DIST_PCA_EUCLID)
    tree = _hclust_ward_d2(d, N)
    info = [] if return_details else None  # deepSplitInfo: computed by the reference, never returned (Fast:433)
    ret = {"deGeneUnion": list(gnames[uni]), "cellTree": tree,
           "dynamicColors": _dynamic_colors(tree, d, deepSplitValues, minClusterSize, eng, info)}
    if save:
        _save(ret, filename)
    if return_details:
        ret["_details"] = {"clusters": names, "code": code, "de": res, "dist": d, "union_idx": uni,
                           "deepSplitInfo": info}
    ds.close()
    return ret


def reclusterDEConsensus(dataMatrix, consensusClusterLabels, method="Wilcoxon", meanScalingFactor=5, qValThrs=None,
                         fcThrs=None, deepSplitValues=(1, 2, 3, 4), minClusterSize=10, filename="de_gene_object.rds",
                         plotName="DE_Heatmap", *, gene_names=None, cluster_order=None, device=0, save=False,
                         return_details=False):
    if qValThrs is None or fcThrs is None:
        raise TypeError('argument "qValThrs"/"fcThrs" is missing, with no default')
    if method == "edgeR":
        raise NotImplementedError("edgeR branch stays on the host in the reference design (SURVEY D3)")
    if method != "Wilcoxon":
        print("Incorrect method chosen.")  # slow:158-161
        return None
    eng = _engine(device)
    m = _as_matrix(dataMatrix)
    N = m[-1] if m[0] in ("csc", "csr") else m[1].shape[1]
    G = m[-2] if m[0] in ("csc", "csr") else m[1].shape[0]
    names, code = select_clusters(consensusClusterLabels, minClusterSize, cluster_order)
    if len(names) < 2:
        raise ValueError("need at least two clusters with > minClusterSize cells")
    ds = _upload(eng, m)
    res = eng.de_run(ds, code, len(names), nat.SCC_DE_SLOW, q_val_thrs=qValThrs, fc_thrs=fcThrs,
                     mean_scaling_factor=float(meanScalingFactor), fetch="all")
    if res.status == nat.SCC_ERR_RSTOP:
        raise RuntimeError(res.message)
    gnames = np.asarray(gene_names if gene_names is not None else [f"gene{g}" for g in range(G)], dtype=object)
    K = len(names)
    p = 0
    qlist, lflist, delist = {}, {}, {}
    for i in range(K - 1):
        for j in range(i + 1, K):
            n_de = int((res.de[p] == 1).sum())
            print(f"{names[i]}, {names[j]} DE genes: {n_de}")  # slow:172-178
            qlist[(names[i], names[j])] = res.q[p]
            lflist[(names[i], names[j])] = res.logfc[p]
            delist[(names[i], names[j])] = list(gnames[res.de[p] == 1])
            p += 1
    uni = res.union
    if len(uni) == 0:
        raise RuntimeError("empty DE gene union")
    d = eng.distance(ds, uni, nat.SCC_DIST_PCA_EUCLID)
    tree = _hclust_ward_d2(d, N)
    ret = {"deGeneUnion": list(gnames[uni]), "cellTree": tree,
           "dynamicColors": _dynamic_colors(tree, d, deepSplitValues, minClusterSize)}
    if save:
        _save({"qValueList": qlist, "logFCList": lflist, "deGeneList": delist}, "de_lists")
        _save(ret, filename)
    if return_details:
        ret["_details"] = {"clusters": names, "code": code, "de": res, "dist": d, "union_idx": uni}
    ds.close()
    return ret
