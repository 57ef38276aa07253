// scc_distance.cpp — C ABI for stage 3 (include/scc.h: scc_distance).
//
// PCA path (parity default, reference Fast:398-400): gather X[U, ] for ALL
// cells, centre columns (R colMeans), fp64 MFMA Gram C = Xc^T Xc, top-k
// eigenpairs of the |U| x |U| Gram (Householder + multisection + inverse
// iteration, exact to fp64 backward error), scores
// P = Xc V_k, then the packed Euclidean `dist`.  The eigensolve is this
// engine's own multi-workgroup dense solver (scc_eigen.hip), no vendor BLAS.  The exact truncated SVD is
// the deterministic quantity irlba approximates.
// Pearson path (reference Fast:403, commented out there): per-cell z-scores
// over U and an FP32 MFMA Gram with the 1 - r epilogue fused into the store.
#include "scc_internal.hpp"

using namespace scc_rt;

extern "C" {
hipError_t scc_launch_union_map(int* umap, int G, const int* genes, int nu, hipStream_t st);
hipError_t scc_launch_gather(const long long* indptr, const int* rows, const double* vals, const double* dense,
                             int G, int N, const int* umap, const int* genes, int nu, int ld, double* Xc,
                             hipStream_t st);
hipError_t scc_launch_center(double* Xc, int N, int nu, int ld, dd* part, int nchunk, double* mean, hipStream_t st);
hipError_t scc_launch_gram(const double* Xc, int Npad, int ld, int nchunk, double* slabs, double* C, hipStream_t st);
hipError_t scc_launch_scores(const double* Xc, int N, int nu, int ld, const double* Z16, int k, double* P,
                             hipStream_t st);
size_t scc_sil_scratch_doubles(int N, int C);
hipError_t scc_launch_silhouette(const void* D, int f32, int N, const int* lab, const int* cnt, int C, double* part,
                                 double* width, hipStream_t st);
hipError_t scc_launch_dist_euclid(const double* P, int N, int c_lo, int c_hi, void* out, int f32, hipStream_t st);
hipError_t scc_launch_zscore(const double* Xc, int N, int nu, int ld, float* Z, int ldz, hipStream_t st);
hipError_t scc_launch_pearson(const double* Xc, int N, int nu, int ld, float* Z, int ldz, int c_lo, int c_hi,
                              void* out, int f32, hipStream_t st);
}

extern "C" void scc_distance_release(scc_ctx*) {}

// columns [col_lo, col_hi) of the packed output (the whole matrix: [0, N))
static int dist_impl(scc_ctx* c, const scc_dataset* ds, const int32_t* genes, int32_t nu, int32_t metric,
                     int32_t ncomp, int64_t col_lo, int64_t col_hi, void* dist_out, int32_t out_kind, int32_t out_f32)
{
    if (!c || !ds || !genes) return fail(c, SCC_ERR_INVALID, "scc_distance: null argument");
    if (!dist_out && out_kind != SCC_PTR_DEVICE) return fail(c, SCC_ERR_INVALID, "scc_distance: null output");
    if (ds->ctx != c) return fail(c, SCC_ERR_INVALID, "dataset belongs to another context");
    if (nu < 1) return fail(c, SCC_ERR_INVALID, "empty gene union");
    if (metric != SCC_DIST_PCA_EUCLID && metric != SCC_DIST_PEARSON) return fail(c, SCC_ERR_INVALID, "bad metric");
    const int G = (int)ds->G, N = (int)ds->N;
    if (N < 2) return fail(c, SCC_ERR_INVALID, "need at least two cells");
    for (int u = 0; u < nu; ++u)
        if (genes[u] < 0 || genes[u] >= G) return fail(c, SCC_ERR_INVALID, "gene index out of range");
    int k = ncomp > 0 ? ncomp : std::min(nu, 15);
    if (k > 16 || k > nu) return fail(c, SCC_ERR_UNSUPPORTED, "ncomp must be <= min(16, |U|)");
    hipSetDevice(c->device);
    hipStream_t s0 = c->s0;
    const int ld = (nu + 63) & ~63;
    const int Npad = (N + 15) & ~15;
    if (col_lo < 0 || col_hi > N || col_lo > col_hi) return fail(c, SCC_ERR_INVALID, "column slice out of range");
    auto colbase = [&](int64_t j) { return (size_t)j * (2 * (size_t)N - j - 1) / 2; };
    const size_t npairs = colbase(col_hi) - colbase(col_lo);  // the slice's packed entries
    int rc;
    int *d_genes, *d_umap;
    double *d_X, *d_mean;
    void* d_part;
#define WS(name, n, ptr)                                       \
    do {                                                       \
        if ((rc = ws(c, name, (size_t)(n), &(ptr)))) return rc; \
    } while (0)
    WS("d_genes", nu, d_genes);
    WS("d_umap", G, d_umap);
    WS("d_X", (size_t)Npad * ld, d_X);
    WS("d_mean", ld, d_mean);
    const int nchunk_mean = 512;  // 2 x 512 workgroups over the column sums
    if ((rc = ws_get(c, "d_part", sizeof(double) * 2 * (size_t)nchunk_mean * ld, &d_part))) return rc;
    void* d_out = dist_out;
    if (out_kind == SCC_PTR_HOST || !dist_out) {  // NULL device output: keep it in the workspace
        if ((rc = ws_get(c, "d_dist", npairs * (out_f32 ? 4 : 8), &d_out))) return rc;
    }
    HIPCHK(c, hipMemcpyAsync(d_genes, genes, sizeof(int) * nu, hipMemcpyHostToDevice, s0));
    {
        Scope sc(c, "gather", s0);
        HIPCHK(c, hipMemsetAsync(d_X, 0, sizeof(double) * (size_t)Npad * ld, s0));
        HIPCHK(c, scc_launch_union_map(d_umap, G, d_genes, nu, s0));
        HIPCHK(c, scc_launch_gather(ds->d_indptr, ds->d_rows, ds->d_vals, ds->d_dense, G, N, d_umap, d_genes, nu, ld,
                                    d_X, s0));
    }
    if (metric == SCC_DIST_PCA_EUCLID) {
        double *d_slabs, *d_C, *d_W, *d_Z, *d_P, *d_escr;
        const int nchunk = std::max(1, std::min(32, Npad / 512));
        WS("d_slabs", (size_t)nchunk * ld * ld, d_slabs);
        WS("d_C", (size_t)ld * ld, d_C);
        WS("d_W", ld, d_W);
        WS("d_Z", (size_t)ld * 16, d_Z);
        WS("d_P", (size_t)N * 16, d_P);
        WS("d_escr", scc_eigen_scratch_doubles(nu, ld, k), d_escr);
        {
            Scope sc(c, "center", s0);
            HIPCHK(c, scc_launch_center(d_X, N, nu, ld, (dd*)d_part, nchunk_mean, d_mean, s0));
        }
        {
            Scope sc(c, "gram", s0);
            HIPCHK(c, scc_launch_gram(d_X, Npad, ld, nchunk, d_slabs, d_C, s0));
        }
        unsigned int* d_eig_err = nullptr;
        {
            Scope sc(c, "eigen", s0);
            hipEvent_t mk[6];
            hipEvent_t* marks = nullptr;
            if (c->profile) {  // per-kernel split of the eigensolve
                for (auto& m : mk) m = ev_take(c);
                marks = mk;
            }
            unsigned long long* st_buf = nullptr;
            if (env_int("SCC_STAMPS", 0)) WS("d_estamps", 8, st_buf);
            int nwg_used = 0;
            HIPCHK(c, scc_launch_eigen_topk(d_C, nu, ld, k, d_escr, d_Z, d_W, &d_eig_err, &nwg_used, marks, st_buf, s0));
            if (st_buf) {
                unsigned long long h[8];
                HIPCHK(c, hipMemcpyAsync(h, st_buf, sizeof(h), hipMemcpyDeviceToHost, s0));
                HIPCHK(c, hipStreamSynchronize(s0));
                fprintf(stderr, "[scc stamps] tridiag n=%d nwg=%d: phase B %llu (wave 0 rows %llu), hand-off wait %llu, "
                        "phase C %llu cycles\n", nu, nwg_used, h[0], h[7], h[1], h[2]);
                fprintf(stderr, "[scc stamps] vectors (eigenpair 0): bisection %llu, LU %llu, inverse iteration %llu, "
                        "back-transform %llu cycles\n", h[3], h[4], h[5], h[6]);
            }
            if (marks) {
                c->pending.push_back({"eig_tridiag", mk[0], mk[1]});
                c->pending.push_back({"eig_vec", mk[2], mk[3]});
                c->pending.push_back({"eig_fin", mk[4], mk[5]});
            }
        }
        HIPCHK(c, hipMemcpyAsync(&c->eig_err, d_eig_err, sizeof(unsigned int), hipMemcpyDeviceToHost, s0));
        if (env_int("SCC_EIG_DUMP", 0)) {  // debug: eigenvalues and vectors on stderr
            std::vector<double> w(k), z((size_t)nu * 16);
            HIPCHK(c, hipMemcpyAsync(w.data(), d_W, sizeof(double) * k, hipMemcpyDeviceToHost, s0));
            HIPCHK(c, hipMemcpyAsync(z.data(), d_Z, sizeof(double) * z.size(), hipMemcpyDeviceToHost, s0));
            HIPCHK(c, hipStreamSynchronize(s0));
            fprintf(stderr, "[scc eig] n=%d k=%d err=%u W:", nu, k, c->eig_err);
            for (int q = 0; q < k; ++q) fprintf(stderr, " %.6g", w[q]);
            fprintf(stderr, "\n");
            for (int u = 0; u < std::min(nu, 8); ++u) {
                fprintf(stderr, "[scc eig] Z[%d]:", u);
                for (int q = 0; q < k; ++q) fprintf(stderr, " %.4g", z[(size_t)u * 16 + q]);
                fprintf(stderr, "\n");
            }
        }
        {
            Scope sc(c, "scores", s0);
            HIPCHK(c, scc_launch_scores(d_X, N, nu, ld, d_Z, k, d_P, s0));
        }
        {
            Scope sc(c, "dist", s0);
            HIPCHK(c, scc_launch_dist_euclid(d_P, N, (int)col_lo, (int)col_hi, d_out, out_f32, s0));
        }
        c->d_last_scores = d_P;
        c->last_n = N;
        c->last_ncomp = k;
    } else {
        float* d_Zp;
        // rows padded to 8 floats (k_pearson_mfma's fragment group); its 32-float
        // staging reads run up to 24 floats past a row, so the last row has slack
        const int ldz = (nu + 7) & ~7;
        WS("d_Zp", (size_t)N * ldz + 32, d_Zp);
        {
            Scope sz(c, "zscore", s0);
            HIPCHK(c, scc_launch_zscore(d_X, N, nu, ld, d_Zp, ldz, s0));
        }
        Scope sc(c, "pearson", s0);
        HIPCHK(c, scc_launch_pearson(d_X, N, nu, ld, d_Zp, ldz, (int)col_lo, (int)col_hi, d_out, out_f32, s0));
    }
    if (out_kind == SCC_PTR_HOST) {
        HIPCHK(c, hipMemcpyAsync(dist_out, d_out, npairs * (out_f32 ? 4 : 8), hipMemcpyDeviceToHost, s0));
    }
    c->d_last_dist = (col_lo == 0 && col_hi == N) ? d_out : nullptr;  // what scc_silhouette(dist = NULL) reads
    c->last_dist_n = N;
    c->last_dist_f32 = out_f32 ? 1 : 0;
    HIPCHK(c, hipStreamSynchronize(s0));
    if (metric == SCC_DIST_PCA_EUCLID && c->eig_err)
        return fail(c, SCC_ERR_HIP, "scc_distance: eigensolver workgroup hand-off timed out");
    return SCC_OK;
#undef WS
}

extern "C" int scc_distance(scc_ctx* c, const scc_dataset* ds, const int32_t* genes, int32_t nu, int32_t metric,
                            int32_t ncomp, void* dist_out, int32_t out_kind, int32_t out_f32)
{
    return dist_impl(c, ds, genes, nu, metric, ncomp, 0, ds ? ds->N : 0, dist_out, out_kind, out_f32);
}

extern "C" int scc_distance_cols(scc_ctx* c, const scc_dataset* ds, const int32_t* genes, int32_t nu, int32_t metric,
                                 int32_t ncomp, int64_t col_lo, int64_t col_hi, void* dist_out, int32_t out_kind,
                                 int32_t out_f32)
{
    return dist_impl(c, ds, genes, nu, metric, ncomp, col_lo, col_hi, dist_out, out_kind, out_f32);
}

extern "C" int scc_silhouette(scc_ctx* c, int64_t n_cells, const int32_t* groups, const void* dist, int32_t dist_f32,
                              double* widths, double* clus_avg, int32_t* n_groups)
{
    if (!c || !groups) return fail(c, SCC_ERR_INVALID, "scc_silhouette: null argument");
    const int N = (int)n_cells;
    if (N < 2) return fail(c, SCC_ERR_INVALID, "scc_silhouette: need at least two cells");
    const void* D = dist;
    int f32 = dist_f32 ? 1 : 0;
    if (!D) {
        if (!c->d_last_dist || c->last_dist_n != N)
            return fail(c, SCC_ERR_INVALID, "scc_silhouette: no full scc_distance output of this size is kept");
        D = c->d_last_dist;
        f32 = c->last_dist_f32;
    }
    // cluster codes in increasing id order (silhouette's sorted clusters)
    std::vector<int32_t> ids(groups, groups + N);
    std::sort(ids.begin(), ids.end());
    ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
    const int C = (int)ids.size();
    if (n_groups) *n_groups = C;
    if (C < 2 || C >= N) return fail(c, SCC_ERR_INVALID, "silhouette needs 2 <= clusters < cells (R returns NA)");
    std::vector<int> lab(N), cnt(C, 0);
    for (int i = 0; i < N; ++i) {
        lab[i] = (int)(std::lower_bound(ids.begin(), ids.end(), groups[i]) - ids.begin());
        cnt[lab[i]]++;
    }
    hipSetDevice(c->device);
    hipStream_t s0 = c->s0;
    int rc;
    int *d_lab, *d_cnt;
    double *d_part, *d_w;
    if ((rc = ws(c, "sil_lab", N, &d_lab))) return rc;
    if ((rc = ws(c, "sil_cnt", C, &d_cnt))) return rc;
    if ((rc = ws(c, "sil_part", scc_sil_scratch_doubles(N, C), &d_part))) return rc;
    if ((rc = ws(c, "sil_w", N, &d_w))) return rc;
    HIPCHK(c, hipMemcpyAsync(d_lab, lab.data(), sizeof(int) * N, hipMemcpyHostToDevice, s0));
    HIPCHK(c, hipMemcpyAsync(d_cnt, cnt.data(), sizeof(int) * C, hipMemcpyHostToDevice, s0));
    {
        Scope sc(c, "silhouette", s0);
        HIPCHK(c, scc_launch_silhouette(D, f32, N, d_lab, d_cnt, C, d_part, d_w, s0));
    }
    std::vector<double> w(N);
    HIPCHK(c, hipMemcpyAsync(w.data(), d_w, sizeof(double) * N, hipMemcpyDeviceToHost, s0));
    HIPCHK(c, hipStreamSynchronize(s0));
    if (widths) std::copy(w.begin(), w.end(), widths);
    if (clus_avg) {  // summary(.)$clus.avg.widths: mean width per cluster (long double sums, R mean)
        std::vector<long double> sum(C, 0.0L);
        for (int i = 0; i < N; ++i) sum[lab[i]] += w[i];
        for (int k = 0; k < C; ++k) clus_avg[k] = (double)(sum[k] / cnt[k]);
    }
    return SCC_OK;
}

extern "C" int scc_last_pca_scores(const scc_ctx* c, double* scores, int32_t* ncomp)
{
    if (!c) return SCC_ERR_INVALID;
    if (ncomp) *ncomp = c->last_ncomp;
    if (scores && c->last_ncomp > 0 && c->d_last_scores) {
        scc_ctx* cc = const_cast<scc_ctx*>(c);
        hipSetDevice(c->device);
        std::vector<double> buf((size_t)c->last_n * 16);
        HIPCHK(cc, hipMemcpy(buf.data(), c->d_last_scores, sizeof(double) * buf.size(), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < (size_t)c->last_n; ++i)
            for (int q = 0; q < c->last_ncomp; ++q) scores[i * c->last_ncomp + q] = buf[i * 16 + q];
    }
    return SCC_OK;
}
