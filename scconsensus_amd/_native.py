"""ctypes binding of ``lib/libscc.so`` — the C ABI declared in ``include/scc.h``.

There is no fallback: if the HIP library is missing this module raises, and if
no MI355X is visible ``Engine()`` raises ``SccError(SCC_ERR_HIP)``.
"""
from __future__ import annotations

import atexit
import ctypes
import os
import weakref
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libscc.so")

SCC_OK = 0
SCC_ERR_INVALID = 1
SCC_ERR_HIP = 2
SCC_ERR_OOM = 3
SCC_ERR_NONFINITE = 4
SCC_ERR_RSTOP = 5
SCC_ERR_UNSUPPORTED = 6
SCC_DE_FAST = 0
SCC_DE_SLOW = 1
SCC_TEST_WILCOX = 0
SCC_TEST_T = 1
SCC_DIST_PCA_EUCLID = 0
SCC_DIST_PEARSON = 1
SCC_PTR_HOST = 0
SCC_PTR_DEVICE = 1

# every symbol include/scc.h declares (tests check the library exports them all)
EXPORTS = [
    "scc_ctx_create", "scc_device_count", "scc_ctx_destroy", "scc_ctx_last_error", "scc_ctx_synchronize", "scc_ctx_set_stream",
    "scc_ctx_kernel_time",
    "scc_ctx_reset_timers", "scc_dataset_create_csc", "scc_dataset_create_csr", "scc_dataset_create_dense", "scc_dataset_destroy",
    "scc_dataset_read_csc",
    "scc_de_run", "scc_de_shard_bytes", "scc_de_run_shard", "scc_de_finish", "scc_de_run_shard_records",
    "scc_de_finish_records", "scc_de_finish_records_pairs", "scc_de_union_first_occ", "scc_de_result_counts", "scc_de_result_union", "scc_de_result_rows",
    "scc_de_result_pair_vectors", "scc_de_result_log_threshold", "scc_de_result_nodg", "scc_de_result_destroy",
    "scc_distance", "scc_de_distance", "scc_distance_cols", "scc_pca_shard_colsum", "scc_pca_shard_gram", "scc_pca_shard_scores", "scc_pca_shard_eigen", "scc_pca_shard_project",
    "scc_distance_scores", "scc_silhouette", "scc_last_pca_scores",
    "scc_hclust_ward_d2", "scc_cutree_hybrid",
    "scc_diag_eigen_topk", "scc_diag_small_syev", "scc_diag_cholinv", "scc_diag_eig_last_path",
    "scc_diag_small_syev_stamps",
]


class SccError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"scc error {code}: {msg}")
        self.code = code


class Opts(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("profile", ctypes.c_int32), ("n_devices", ctypes.c_int32),
                ("reserved", ctypes.c_int32 * 5), ("devices", ctypes.POINTER(ctypes.c_int32))]


class DeParams(ctypes.Structure):
    _fields_ = [("mode", ctypes.c_int32), ("top_n", ctypes.c_int32), ("q_val_thrs", ctypes.c_double),
                ("log_fc_thrs", ctypes.c_double), ("min_per_cent", ctypes.c_double), ("fc_thrs", ctypes.c_double),
                ("mean_scaling_factor", ctypes.c_double), ("test_all", ctypes.c_int32),
                ("test", ctypes.c_int32)]


_lib = None
_live_datasets: "weakref.WeakSet" = weakref.WeakSet()
_live_engines: "weakref.WeakSet" = weakref.WeakSet()
_shutdown = False


@atexit.register
def _teardown():
    # release device objects in dependency order while the HIP runtime is
    # still alive (interpreter-exit __del__ order is arbitrary)
    global _shutdown
    for d in list(_live_datasets):
        d.close()
    for e in list(_live_engines):
        e.close()
    _shutdown = True


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: run `python -m scconsensus_amd.build` (hipcc, gfx950)")
    L = ctypes.CDLL(LIB_PATH)
    vp = ctypes.c_void_p
    P = ctypes.POINTER
    i32, i64, dbl, u8 = ctypes.c_int32, ctypes.c_int64, ctypes.c_double, ctypes.c_uint8
    sig = {
        "scc_ctx_create": (ctypes.c_int, [P(Opts), P(vp)]),
        "scc_device_count": (ctypes.c_int, [P(i32)]),
        "scc_ctx_destroy": (None, [vp]),
        "scc_ctx_last_error": (ctypes.c_char_p, [vp]),
        "scc_ctx_synchronize": (ctypes.c_int, [vp]),
        "scc_ctx_set_stream": (ctypes.c_int, [vp, vp, i32]),
        "scc_ctx_kernel_time": (ctypes.c_int, [vp, ctypes.c_char_p, P(dbl), P(i64)]),
        "scc_ctx_reset_timers": (None, [vp]),
        "scc_dataset_create_csc": (ctypes.c_int, [vp, vp, vp, vp, i64, i64, i64, i32, P(vp)]),
        "scc_dataset_create_csr": (ctypes.c_int, [vp, vp, vp, vp, i64, i64, i64, i32, P(vp)]),
        "scc_dataset_create_dense": (ctypes.c_int, [vp, vp, i64, i64, i32, P(vp)]),
        "scc_dataset_destroy": (None, [vp]),
        "scc_dataset_read_csc": (ctypes.c_int, [vp, vp, vp, vp]),
        "scc_de_run": (ctypes.c_int, [vp, vp, vp, i32, P(DeParams), P(vp)]),
        "scc_de_shard_bytes": (i64, [i32, i64]),
        "scc_de_run_shard": (ctypes.c_int, [vp, vp, vp, i32, P(DeParams), i64, i64, vp]),
        "scc_de_finish": (ctypes.c_int, [vp, vp, vp, i32, P(DeParams), vp, P(vp)]),
        "scc_de_run_shard_records": (ctypes.c_int, [vp, vp, vp, i32, P(DeParams), i64, i64, vp, i64, P(i64)]),
        "scc_de_finish_records": (ctypes.c_int, [vp, vp, vp, i32, P(DeParams), vp, vp, i32, i64, P(vp)]),
        "scc_de_finish_records_pairs": (ctypes.c_int, [vp, vp, vp, i32, P(DeParams), vp, vp, i32, i64, i32, i32, vp]),
        "scc_de_union_first_occ": (ctypes.c_int, [vp, vp, i64, vp, P(i32)]),
        "scc_de_result_counts": (ctypes.c_int, [vp, P(i32), P(i64), P(i32)]),
        "scc_de_result_union": (ctypes.c_int, [vp, vp]),
        "scc_de_result_rows": (ctypes.c_int, [vp] + [vp] * 10),
        "scc_de_result_pair_vectors": (ctypes.c_int, [vp] + [vp] * 5),
        "scc_de_result_log_threshold": (ctypes.c_int, [vp, P(dbl)]),
        "scc_de_result_nodg": (ctypes.c_int, [vp, vp]),
        "scc_de_result_destroy": (None, [vp]),
        "scc_distance": (ctypes.c_int, [vp, vp, vp, i32, i32, i32, vp, i32, i32]),
        "scc_de_distance": (ctypes.c_int, [vp, vp, vp, i32, P(DeParams), i32, i32, vp, i32, i32, P(vp)]),
        "scc_distance_cols": (ctypes.c_int, [vp, vp, vp, i32, i32, i32, i64, i64, vp, i32, i32]),
        "scc_pca_shard_colsum": (ctypes.c_int, [vp, vp, vp, i32, i64, i64, vp]),
        "scc_pca_shard_gram": (ctypes.c_int, [vp, vp, i32, vp]),
        "scc_pca_shard_scores": (ctypes.c_int, [vp, vp, i32, vp]),
        "scc_pca_shard_eigen": (ctypes.c_int, [vp, vp, i32, vp]),
        "scc_pca_shard_project": (ctypes.c_int, [vp, vp, i32, vp]),
        "scc_distance_scores": (ctypes.c_int, [vp, vp, i64, i64, i64, vp, i32, i32]),
        "scc_silhouette": (ctypes.c_int, [vp, i64, vp, vp, i32, vp, vp, P(i32)]),
        "scc_last_pca_scores": (ctypes.c_int, [vp, vp, P(i32)]),
        "scc_hclust_ward_d2": (ctypes.c_int, [vp, i64, vp, vp, vp]),
        "scc_cutree_hybrid": (ctypes.c_int, [vp, vp, i64, vp, i32, i32, vp, P(dbl)]),
        "scc_diag_eigen_topk": (ctypes.c_int, [vp, i32, i32, i32, vp, vp, P(ctypes.c_int)]),
        "scc_diag_small_syev": (ctypes.c_int, [vp, i32, i32, i32, vp, vp, vp]),
        "scc_diag_cholinv": (ctypes.c_int, [vp, i32, dbl, vp, vp]),
        "scc_diag_eig_last_path": (ctypes.c_int, []),
        "scc_diag_small_syev_stamps": (ctypes.c_int, [vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def _ptr(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


@dataclass
class FastRows:
    pair_tested: np.ndarray
    row_pair: np.ndarray
    gene: np.ndarray
    p: np.ndarray
    q: np.ndarray
    avg_logfc: np.ndarray
    pct1: np.ndarray
    pct2: np.ndarray
    u2: np.ndarray
    ties: np.ndarray
    de: np.ndarray
    top: np.ndarray


@dataclass
class DeResult:
    mode: int
    K: int
    n_pairs: int
    union: np.ndarray
    nodg: np.ndarray
    rows: FastRows | None = None       # FAST
    p: np.ndarray | None = None        # [P, G]
    q: np.ndarray | None = None        # SLOW [P, G]
    logfc: np.ndarray | None = None    # [P, G]
    u2: np.ndarray | None = None       # [P, G]
    de: np.ndarray | None = None       # SLOW [P, G]
    log_thr: float = 0.0
    status: int = 0
    message: str = ""


class Dataset:
    def __init__(self, engine, handle, G, N):
        self.engine, self.handle, self.G, self.N = engine, handle, G, N
        _live_datasets.add(self)

    def close(self):
        if self.handle and not _shutdown:
            self.engine.lib.scc_dataset_destroy(self.handle)
        self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def device_count() -> int:
    n = ctypes.c_int32()
    load().scc_device_count(ctypes.byref(n))
    return n.value


class Engine:
    """One MI355X device (``device`` = HIP ordinal), or ONE job over a device
    list (``devices``: HIP ordinals, devices[0] the primary; scc_opts.devices)."""

    def __init__(self, device: int = 0, profile: bool = False, devices=None):
        self.lib = load()
        h = ctypes.c_void_p()
        o = Opts(device, 1 if profile else 0)
        if devices is not None and len(devices) > 1:
            self._devs = (ctypes.c_int32 * len(devices))(*[int(d) for d in devices])
            o.n_devices = len(devices)
            o.devices = self._devs
        rc = self.lib.scc_ctx_create(ctypes.byref(o), ctypes.byref(h))
        if rc != SCC_OK:
            raise SccError(rc, "scc_ctx_create failed (no HIP device?)")
        self.ctx = h
        _live_engines.add(self)

    def close(self):
        if self.ctx and not _shutdown:
            for d in list(_live_datasets):
                if d.engine is self:
                    d.close()
            self.lib.scc_ctx_destroy(self.ctx)
        self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != SCC_OK:
            raise SccError(rc, self.lib.scc_ctx_last_error(self.ctx).decode())

    # -------------------------------------------------------------- datasets
    def dataset_csc(self, indptr, rows, vals, G, N) -> Dataset:
        indptr = np.ascontiguousarray(indptr, np.int64)
        rows = np.ascontiguousarray(rows, np.int32)
        vals = np.ascontiguousarray(vals, np.float64)
        h = ctypes.c_void_p()
        self._check(self.lib.scc_dataset_create_csc(self.ctx, _ptr(indptr), _ptr(rows), _ptr(vals), G, N, len(vals),
                                                    SCC_PTR_HOST, ctypes.byref(h)))
        return Dataset(self, h, G, N)

    def dataset_csc_device(self, indptr_ptr, rows_ptr, vals_ptr, G, N, nnz) -> Dataset:
        h = ctypes.c_void_p()
        self._check(self.lib.scc_dataset_create_csc(self.ctx, ctypes.c_void_p(indptr_ptr), ctypes.c_void_p(rows_ptr),
                                                    ctypes.c_void_p(vals_ptr), G, N, nnz, SCC_PTR_DEVICE,
                                                    ctypes.byref(h)))
        return Dataset(self, h, G, N)

    def dataset_csr(self, indptr, cols, vals, G, N) -> Dataset:
        """Gene-major CSR (genes x cells: indptr[G+1], cell columns, values),
        transposed on the device into the resident dgCMatrix layout."""
        indptr = np.ascontiguousarray(indptr, np.int64)
        cols = np.ascontiguousarray(cols, np.int32)
        vals = np.ascontiguousarray(vals, np.float64)
        h = ctypes.c_void_p()
        self._check(self.lib.scc_dataset_create_csr(self.ctx, _ptr(indptr), _ptr(cols), _ptr(vals), G, N, len(vals),
                                                    SCC_PTR_HOST, ctypes.byref(h)))
        return Dataset(self, h, G, N)

    def dataset_csr_device(self, indptr_ptr, cols_ptr, vals_ptr, G, N, nnz) -> Dataset:
        h = ctypes.c_void_p()
        self._check(self.lib.scc_dataset_create_csr(self.ctx, ctypes.c_void_p(indptr_ptr), ctypes.c_void_p(cols_ptr),
                                                    ctypes.c_void_p(vals_ptr), G, N, nnz, SCC_PTR_DEVICE,
                                                    ctypes.byref(h)))
        return Dataset(self, h, G, N)

    def read_csc(self, ds: Dataset):
        """The dataset's resident dgCMatrix (indptr, rows, vals) on the host."""
        indptr = np.empty(ds.N + 1, np.int64)
        self._check(self.lib.scc_dataset_read_csc(ds.handle, _ptr(indptr), None, None))
        nnz = int(indptr[-1])
        rows = np.empty(max(nnz, 1), np.int32)
        vals = np.empty(max(nnz, 1), np.float64)
        self._check(self.lib.scc_dataset_read_csc(ds.handle, _ptr(indptr), _ptr(rows), _ptr(vals)))
        return indptr, rows[:nnz], vals[:nnz]

    def dataset_dense(self, X_gene_major) -> Dataset:
        """X as a genes x cells array; passed to the engine in R's column-major layout."""
        X = np.asarray(X_gene_major, np.float64)
        G, N = X.shape
        col = np.ascontiguousarray(X.T)  # N x G row-major == G x N column-major
        h = ctypes.c_void_p()
        self._check(self.lib.scc_dataset_create_dense(self.ctx, _ptr(col), G, N, SCC_PTR_HOST, ctypes.byref(h)))
        return Dataset(self, h, G, N)

    # -------------------------------------------------------------- DE
    def de_run(self, ds: Dataset, code, K, mode=SCC_DE_FAST, q_val_thrs=0.1, log_fc_thrs=0.5, min_per_cent=20.0,
               top_n=30, fc_thrs=1.5, mean_scaling_factor=5.0, fetch="all", test_all=None, test="wilcox") -> DeResult:
        """test_all (FAST): also compute U / p for the (pair, gene) cells the
        feature filters drop; default: only when the full per-pair vectors are
        fetched (fetch="all")."""
        code = np.ascontiguousarray(code, np.int32)
        prm = self._de_params(mode, q_val_thrs, log_fc_thrs, min_per_cent, top_n, fc_thrs, mean_scaling_factor,
                              fetch == "all" if test_all is None else test_all, test)
        r = ctypes.c_void_p()
        rc = self.lib.scc_de_run(self.ctx, ds.handle, _ptr(code), K, ctypes.byref(prm), ctypes.byref(r))
        return self._collect(r, rc, ds, mode, K, fetch)

    @staticmethod
    def _de_params(mode, q_val_thrs, log_fc_thrs, min_per_cent, top_n, fc_thrs, mean_scaling_factor, test_all,
                   test="wilcox"):
        if test not in ("wilcox", "t"):
            raise ValueError(f"test must be 'wilcox' or 't', not {test!r}")
        return DeParams(mode, top_n, q_val_thrs, log_fc_thrs, min_per_cent, fc_thrs, mean_scaling_factor,
                        1 if test_all else 0, SCC_TEST_T if test == "t" else SCC_TEST_WILCOX)

    def de_shard_bytes(self, K, G) -> int:
        return int(self.lib.scc_de_shard_bytes(K, G))

    def de_run_shard(self, ds: Dataset, code, K, gene_lo, gene_hi, shard_ptr, mode=SCC_DE_FAST, q_val_thrs=0.1,
                     log_fc_thrs=0.5, min_per_cent=20.0, top_n=30, fc_thrs=1.5, mean_scaling_factor=5.0,
                     test_all=False, test="wilcox"):
        """Per-(pair, gene) DE cells of genes [gene_lo, gene_hi) into the device
        buffer at shard_ptr (de_shard_bytes(K, G) bytes, zero outside the shard)."""
        code = np.ascontiguousarray(code, np.int32)
        prm = self._de_params(mode, q_val_thrs, log_fc_thrs, min_per_cent, top_n, fc_thrs, mean_scaling_factor,
                              test_all, test)
        self._check(self.lib.scc_de_run_shard(self.ctx, ds.handle, _ptr(code), K, ctypes.byref(prm), gene_lo,
                                              gene_hi, ctypes.c_void_p(shard_ptr)))

    def de_finish(self, ds: Dataset, code, K, shards_sum_ptr, mode=SCC_DE_FAST, q_val_thrs=0.1, log_fc_thrs=0.5,
                  min_per_cent=20.0, top_n=30, fc_thrs=1.5, mean_scaling_factor=5.0, fetch="all",
                  test_all=False, test="wilcox") -> DeResult:
        """Selection and union from the summed shards of every rank (device)."""
        code = np.ascontiguousarray(code, np.int32)
        prm = self._de_params(mode, q_val_thrs, log_fc_thrs, min_per_cent, top_n, fc_thrs, mean_scaling_factor,
                              test_all, test)
        r = ctypes.c_void_p()
        rc = self.lib.scc_de_finish(self.ctx, ds.handle, _ptr(code), K, ctypes.byref(prm),
                                    ctypes.c_void_p(shards_sum_ptr), ctypes.byref(r))
        return self._collect(r, rc, ds, mode, K, fetch)

    REC_BYTES = 64  # sizeof(scc_de_record)

    def de_run_shard_records(self, ds: Dataset, code, K, gene_lo, gene_hi, rec_ptr, cap, mode=SCC_DE_FAST,
                             q_val_thrs=0.1, log_fc_thrs=0.5, min_per_cent=20.0, top_n=30, fc_thrs=1.5,
                             mean_scaling_factor=5.0, test_all=False, test="wilcox") -> int:
        """Compact records (scc_de_record, 64 B) of the tested (pair, gene)
        cells of genes [gene_lo, gene_hi) into the device buffer at rec_ptr
        (capacity ``cap`` records); returns their number."""
        code = np.ascontiguousarray(code, np.int32)
        prm = self._de_params(mode, q_val_thrs, log_fc_thrs, min_per_cent, top_n, fc_thrs, mean_scaling_factor,
                              test_all, test)
        n = ctypes.c_int64()
        self._check(self.lib.scc_de_run_shard_records(self.ctx, ds.handle, _ptr(code), K, ctypes.byref(prm), gene_lo,
                                                      gene_hi, ctypes.c_void_p(rec_ptr), cap, ctypes.byref(n)))
        return n.value

    def de_finish_records(self, ds: Dataset, code, K, rec_ptr, counts, stride, mode=SCC_DE_FAST, q_val_thrs=0.1,
                          log_fc_thrs=0.5, min_per_cent=20.0, top_n=30, fc_thrs=1.5, mean_scaling_factor=5.0,
                          fetch="all", test_all=False, test="wilcox") -> DeResult:
        """Selection and union from the gathered records of every rank (device
        blocks ``stride`` records apart, ``counts[r]`` valid in block r)."""
        code = np.ascontiguousarray(code, np.int32)
        prm = self._de_params(mode, q_val_thrs, log_fc_thrs, min_per_cent, top_n, fc_thrs, mean_scaling_factor,
                              test_all, test)
        cnt = np.ascontiguousarray(counts, np.int64)
        r = ctypes.c_void_p()
        rc = self.lib.scc_de_finish_records(self.ctx, ds.handle, _ptr(code), K, ctypes.byref(prm),
                                            ctypes.c_void_p(rec_ptr or None), _ptr(cnt), len(cnt), int(stride),
                                            ctypes.byref(r))
        return self._collect(r, rc, ds, mode, K, fetch)

    def de_finish_records_pairs(self, ds: Dataset, code, K, rec_ptr, counts, stride, pair_lo, pair_hi, first_ptr,
                                q_val_thrs=0.1, log_fc_thrs=0.5, min_per_cent=20.0, top_n=30, test_all=False,
                                test="wilcox", **_):
        """FAST selection of the pairs [pair_lo, pair_hi) from the gathered
        records; the genes' first-occurrence keys go to ``first_ptr`` (device
        uint64 [G]; combine the ranks' arrays by MIN, then de_union_first_occ)."""
        code = np.ascontiguousarray(code, np.int32)
        prm = self._de_params(SCC_DE_FAST, q_val_thrs, log_fc_thrs, min_per_cent, top_n, 1.5, 5.0, test_all, test)
        cnt = np.ascontiguousarray(counts, np.int64)
        self._check(self.lib.scc_de_finish_records_pairs(self.ctx, ds.handle, _ptr(code), K, ctypes.byref(prm),
                                                         ctypes.c_void_p(rec_ptr or None), _ptr(cnt), len(cnt),
                                                         int(stride), int(pair_lo), int(pair_hi),
                                                         ctypes.c_void_p(first_ptr)))

    def de_union_first_occ(self, first_ptr, G):
        """deGeneUnion (reference order) from a combined first-occurrence array."""
        out = np.zeros(G, np.int32)
        nu = ctypes.c_int32()
        self._check(self.lib.scc_de_union_first_occ(self.ctx, ctypes.c_void_p(first_ptr), G, _ptr(out),
                                                    ctypes.byref(nu)))
        return out[: nu.value].copy()

    def _collect(self, r, rc, ds, mode, K, fetch) -> DeResult:
        msg = ""
        if rc != SCC_OK:
            msg = self.lib.scc_ctx_last_error(self.ctx).decode()
            if not r.value:
                raise SccError(rc, msg)
        try:
            npairs, nrows, nu = ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int32()
            self._check(self.lib.scc_de_result_counts(r, ctypes.byref(npairs), ctypes.byref(nrows), ctypes.byref(nu)))
            uni = np.zeros(nu.value, np.int32)
            self._check(self.lib.scc_de_result_union(r, _ptr(uni)))
            out = DeResult(mode, K, npairs.value, uni, np.zeros(0, np.int32), status=rc, message=msg)
            if fetch == "union":
                return out
            nodg = np.zeros(ds.N, np.int32)
            self._check(self.lib.scc_de_result_nodg(r, _ptr(nodg)))
            out.nodg = nodg
            if fetch == "nodg":  # what the R glue's C_scc_de_fast returns: the union and nodg
                return out
            P, G = npairs.value, ds.G
            if mode == SCC_DE_FAST:
                n = nrows.value
                tested = np.zeros(P, np.int32)
                a = dict(gene=np.zeros(n, np.int32), p=np.zeros(n), q=np.zeros(n), lfc=np.zeros(n),
                         pct1=np.zeros(n), pct2=np.zeros(n), u2=np.zeros(n, np.int64), t=np.zeros(n, np.int64),
                         fl=np.zeros(n, np.uint8))
                self._check(self.lib.scc_de_result_rows(r, _ptr(tested), _ptr(a["gene"]), _ptr(a["p"]), _ptr(a["q"]),
                                                        _ptr(a["lfc"]), _ptr(a["pct1"]), _ptr(a["pct2"]),
                                                        _ptr(a["u2"]), _ptr(a["t"]), _ptr(a["fl"])))
                out.rows = FastRows(tested, np.repeat(np.arange(P, dtype=np.int32), tested), a["gene"], a["p"],
                                    a["q"], a["lfc"], a["pct1"], a["pct2"], a["u2"], a["t"], (a["fl"] & 1) > 0,
                                    (a["fl"] & 2) > 0)
                if fetch == "all":
                    pv, lf, u2 = np.zeros((P, G)), np.zeros((P, G)), np.zeros((P, G), np.int64)
                    self._check(self.lib.scc_de_result_pair_vectors(r, _ptr(pv), None, _ptr(lf), _ptr(u2), None))
                    out.p, out.logfc, out.u2 = pv, lf, u2
            else:
                pv, qv, lf = np.zeros((P, G)), np.zeros((P, G)), np.zeros((P, G))
                u2, de = np.zeros((P, G), np.int64), np.zeros((P, G), np.uint8)
                self._check(self.lib.scc_de_result_pair_vectors(r, _ptr(pv), _ptr(qv), _ptr(lf), _ptr(u2), _ptr(de)))
                out.p, out.q, out.logfc, out.u2, out.de = pv, qv, lf, u2, de
                lt = ctypes.c_double()
                self._check(self.lib.scc_de_result_log_threshold(r, ctypes.byref(lt)))
                out.log_thr = lt.value
            return out
        finally:
            self.lib.scc_de_result_destroy(r)

    # -------------------------------------------------------------- distance
    def distance(self, ds: Dataset, genes, metric=SCC_DIST_PCA_EUCLID, ncomp=0, out=None, f32=False,
                 device_out_ptr=None):
        genes = np.ascontiguousarray(genes, np.int32)
        N = ds.N
        npairs = N * (N - 1) // 2
        if device_out_ptr is not None:  # 0 -> engine-owned HBM-resident output
            self._check(self.lib.scc_distance(self.ctx, ds.handle, _ptr(genes), len(genes), metric, ncomp,
                                              ctypes.c_void_p(device_out_ptr or None), SCC_PTR_DEVICE,
                                              1 if f32 else 0))
            return None
        if out is None:
            out = np.empty(npairs, np.float32 if f32 else np.float64)
        self._check(self.lib.scc_distance(self.ctx, ds.handle, _ptr(genes), len(genes), metric, ncomp, _ptr(out),
                                          SCC_PTR_HOST, 1 if f32 else 0))
        return out

    def de_distance(self, ds: Dataset, code, K, mode=SCC_DE_FAST, metric=SCC_DIST_PCA_EUCLID, ncomp=0, out=None,
                    f32=False, device_out_ptr=None, fetch="union", **de_kw):
        """scc_de_distance: the DE, then the distance over its union, in one
        C call.  Returns (DeResult, distance) — the distance None for device
        output (device_out_ptr; 0 keeps it in the engine)."""
        code = np.ascontiguousarray(code, np.int32)
        kw = dict(q_val_thrs=0.1, log_fc_thrs=0.5, min_per_cent=20.0, top_n=30, fc_thrs=1.5, mean_scaling_factor=5.0,
                  test_all=None, test="wilcox")
        unknown = set(de_kw) - set(kw)
        if unknown:
            raise TypeError(f"de_distance: unknown DE arguments {sorted(unknown)}")
        kw.update(de_kw)
        prm = self._de_params(mode, kw["q_val_thrs"], kw["log_fc_thrs"], kw["min_per_cent"], kw["top_n"],
                              kw["fc_thrs"], kw["mean_scaling_factor"],
                              fetch == "all" if kw["test_all"] is None else kw["test_all"], kw["test"])
        r = ctypes.c_void_p()
        if device_out_ptr is not None:
            dst, kind, res = ctypes.c_void_p(device_out_ptr or None), SCC_PTR_DEVICE, None
        else:
            res = out if out is not None else np.empty(ds.N * (ds.N - 1) // 2, np.float32 if f32 else np.float64)
            dst, kind = _ptr(res), SCC_PTR_HOST
        rc = self.lib.scc_de_distance(self.ctx, ds.handle, _ptr(code), K, ctypes.byref(prm), metric, ncomp, dst, kind,
                                      1 if f32 else 0, ctypes.byref(r))
        if rc != SCC_OK and r.value:  # the DE succeeded, the distance failed: free the result, raise
            self.lib.scc_de_result_destroy(r)
            self._check(rc)
        de = self._collect(r, rc, ds, mode, K, fetch)
        return de, res

    def distance_cols(self, ds: Dataset, genes, col_lo, col_hi, metric=SCC_DIST_PCA_EUCLID, ncomp=0, out=None,
                      f32=False, device_out_ptr=None):
        """Columns [col_lo, col_hi) of the packed distance vector (a contiguous slice)."""
        genes = np.ascontiguousarray(genes, np.int32)
        N = ds.N
        n = col_hi * (2 * N - col_hi - 1) // 2 - col_lo * (2 * N - col_lo - 1) // 2
        if device_out_ptr is not None:
            self._check(self.lib.scc_distance_cols(self.ctx, ds.handle, _ptr(genes), len(genes), metric, ncomp, col_lo,
                                                   col_hi, ctypes.c_void_p(device_out_ptr or None), SCC_PTR_DEVICE,
                                                   1 if f32 else 0))
            return None
        if out is None:
            out = np.empty(n, np.float32 if f32 else np.float64)
        self._check(self.lib.scc_distance_cols(self.ctx, ds.handle, _ptr(genes), len(genes), metric, ncomp, col_lo,
                                               col_hi, _ptr(out), SCC_PTR_HOST, 1 if f32 else 0))
        return out

    # ---------------------------------------------------------- sharded PCA
    def pca_shard_colsum(self, ds: Dataset, genes, cell_lo, cell_hi, part_ptr):
        genes = np.ascontiguousarray(genes, np.int32)
        self._check(self.lib.scc_pca_shard_colsum(self.ctx, ds.handle, _ptr(genes), len(genes), cell_lo, cell_hi,
                                                  ctypes.c_void_p(part_ptr)))

    def pca_shard_gram(self, parts_ptr, world, gram_ptr):
        self._check(self.lib.scc_pca_shard_gram(self.ctx, ctypes.c_void_p(parts_ptr), world, ctypes.c_void_p(gram_ptr)))

    def pca_shard_scores(self, gram_ptr, scores_ptr, ncomp=0):
        self._check(self.lib.scc_pca_shard_scores(self.ctx, ctypes.c_void_p(gram_ptr), ncomp,
                                                  ctypes.c_void_p(scores_ptr)))

    def pca_shard_eigen(self, gram_ptr, vecs_ptr, ncomp=0):
        self._check(self.lib.scc_pca_shard_eigen(self.ctx, ctypes.c_void_p(gram_ptr), ncomp, ctypes.c_void_p(vecs_ptr)))

    def pca_shard_project(self, vecs_ptr, scores_ptr, ncomp=0):
        self._check(self.lib.scc_pca_shard_project(self.ctx, ctypes.c_void_p(vecs_ptr), ncomp,
                                                   ctypes.c_void_p(scores_ptr)))

    def distance_scores(self, scores_ptr, N, col_lo, col_hi, out=None, f32=False, device_out_ptr=None):
        """Packed `dist` columns [col_lo, col_hi) from a device [N][16] score matrix."""
        n = col_hi * (2 * N - col_hi - 1) // 2 - col_lo * (2 * N - col_lo - 1) // 2
        if device_out_ptr is not None:
            self._check(self.lib.scc_distance_scores(self.ctx, ctypes.c_void_p(scores_ptr), N, col_lo, col_hi,
                                                     ctypes.c_void_p(device_out_ptr or None), SCC_PTR_DEVICE,
                                                     1 if f32 else 0))
            return None
        if out is None:
            out = np.empty(n, np.float32 if f32 else np.float64)
        self._check(self.lib.scc_distance_scores(self.ctx, ctypes.c_void_p(scores_ptr), N, col_lo, col_hi, _ptr(out),
                                                 SCC_PTR_HOST, 1 if f32 else 0))
        return out

    def silhouette(self, N, groups, dist_device_ptr=None, f32=False):
        """(widths [N], per-cluster average widths in sorted group order) of
        cluster::silhouette(groups, as.matrix(d)); d = the engine-kept output
        of the last full distance() call unless a device pointer is given."""
        groups = np.ascontiguousarray(groups, np.int32)
        C = len(np.unique(groups))
        w, ca, k = np.zeros(N), np.zeros(max(C, 1)), ctypes.c_int32()
        self._check(self.lib.scc_silhouette(self.ctx, N, _ptr(groups), ctypes.c_void_p(dist_device_ptr or None),
                                            1 if f32 else 0, _ptr(w), _ptr(ca), ctypes.byref(k)))
        return w, ca[:k.value]

    def last_pca_scores(self, N):
        k = ctypes.c_int32()
        self._check(self.lib.scc_last_pca_scores(self.ctx, None, ctypes.byref(k)))
        s = np.zeros((N, k.value))
        self._check(self.lib.scc_last_pca_scores(self.ctx, _ptr(s), ctypes.byref(k)))
        return s

    # -------------------------------------------------------------- timers
    def kernel_time(self, name):
        ms, n = ctypes.c_double(), ctypes.c_int64()
        self._check(self.lib.scc_ctx_kernel_time(self.ctx, name.encode(), ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def reset_timers(self):
        self.lib.scc_ctx_reset_timers(self.ctx)

    def synchronize(self):
        self._check(self.lib.scc_ctx_synchronize(self.ctx))

    def set_stream(self, stream_handle):
        """Launch on the caller's HIP stream (an int handle, e.g. torch's
        ``torch.cuda.current_stream().cuda_stream``; 0 is the legacy default
        stream); ``None``: back to the engine's own stream."""
        self._check(self.lib.scc_ctx_set_stream(self.ctx, ctypes.c_void_p(stream_handle or None),
                                                0 if stream_handle is None else 1))

    def on_stream(self, stream_handle):
        """Context manager: the engine's work goes on ``stream_handle`` inside."""
        eng = self

        class _On:
            def __enter__(self):
                eng.set_stream(stream_handle)
                return eng

            def __exit__(self, *exc):
                eng.set_stream(None)
                return False
        return _On()


# ---------------------------------------------------------------- host clustering
# Host functions of libscc (no device, no Engine): the reference keeps tree
# building and tree cutting on the host (Fast:406-427).

def hclust_ward_d2(dist_packed, n):
    """fastcluster::hclust(d, "ward.D2") -> (merge (n-1, 2) int32 in R's
    convention, height (n-1,), order (n,) 1-based)."""
    d = np.ascontiguousarray(dist_packed, np.float64)
    if d.shape != (n * (n - 1) // 2,):
        raise ValueError("dist_packed must hold n(n-1)/2 entries")
    merge = np.zeros(2 * (n - 1), np.int32)
    height = np.zeros(n - 1)
    order = np.zeros(n, np.int32)
    rc = load().scc_hclust_ward_d2(_ptr(d), n, _ptr(merge), _ptr(height), _ptr(order))
    if rc != SCC_OK:
        raise SccError(rc, "scc_hclust_ward_d2 failed")
    return merge.reshape(2, n - 1).T.copy(), height, order


def cutree_hybrid(merge, height, dist_packed, deep_split=1, min_cluster_size=20):
    """dynamicTreeCut::cutreeDynamic(method = "hybrid", pamStage = FALSE)
    labels (0 = unassigned) and the default cut height used."""
    merge = np.asarray(merge)
    n = merge.shape[0] + 1
    m = np.ascontiguousarray(merge.T.reshape(-1), np.int32)
    h = np.ascontiguousarray(height, np.float64)
    d = np.ascontiguousarray(dist_packed, np.float64)
    if d.shape != (n * (n - 1) // 2,) or h.shape != (n - 1,):
        raise ValueError("shape mismatch between merge, height and dist_packed")
    lab = np.zeros(n, np.int32)
    cut = ctypes.c_double()
    rc = load().scc_cutree_hybrid(_ptr(m), _ptr(h), n, _ptr(d), int(deep_split), int(min_cluster_size), _ptr(lab),
                                  ctypes.byref(cut))
    if rc != SCC_OK:
        raise SccError(rc, "scc_cutree_hybrid failed (deepSplit must be 0..4)")
    return lab, cut.value
