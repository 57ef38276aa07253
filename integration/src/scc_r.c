/*
 * scc_r.c — R `.Call` glue for libscc (include/scc.h).  Compiled only where R
 * headers exist (R CMD INSTALL of the scConsensus package with this file in
 * src/; R is absent from the build container).  The glue never lets a C++
 * frame unwind through R: every libscc entry point returns an int status, and
 * Rf_error() is raised only here, after the library call returned.
 *
 * Bindings (reference call sites they replace):
 *   C_scc_dataset   as.matrix(dataMatrix) per pair (Fast:368) / dataIn (slow:32):
 *                   ONE upload per call of the R function, held as an external
 *                   pointer that the DE and distance calls share
 *   C_scc_de_fast   R/reclusterDEConsensusFast.R:57-392 (pair loop, ComputePairWiseDE, top_n, unique)
 *   C_scc_de_slow   R/reclusterDEConsensus.R:32-227
 *   C_scc_distance  R/reclusterDEConsensusFast.R:398-400 (prcomp_irlba + dist), :403 (1 - cor)
 *   C_scc_release   frees the device copy early (the finalizer does it otherwise)
 *   C_scc_devices   nCores (Fast:33,61-65) -> the context's device list
 *   C_scc_si        deepSplitInfo's silhouette SI (Fast:433) on the engine-kept dist
 *   C_scc_cutree    dynamicTreeCut::cutreeDynamic(..., distM = as.matrix(d), pamStage = FALSE)
 *                   (Fast:421-427) on the packed dist: no N x N host matrix
 *                   (options(scConsensus.engineCut = TRUE))
 *   C_scc_hclust    hclust(d, "ward.D2") (Fast:406-411) restated in C++
 *                   (options(scConsensus.engineTree = TRUE))
 */
#include <R.h>
#include <Rinternals.h>
#include <R_ext/Rdynload.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "scc.h"

static scc_ctx* g_ctx = NULL;
static int g_ndev = 1;  /* devices of g_ctx: 0 .. g_ndev - 1 */

static void ensure_ctx(void)
{
    if (g_ctx) return;
    scc_opts o;
    memset(&o, 0, sizeof(o));
    int32_t devs[64];
    if (g_ndev > 1) {
        for (int k = 0; k < g_ndev; ++k) devs[k] = k;
        o.n_devices = g_ndev;
        o.devices = devs;
    }
    if (scc_ctx_create(&o, &g_ctx) != SCC_OK) Rf_error("scConsensus engine: no MI355X (HIP) device available");
}

/* nCores (Fast:33, the PSOCK workers of Fast:61-65) -> the engine's device
 * list: min(nCores, visible GPUs) devices, ONE job sharded over them (gene
 * blocks for the DE, column slices for dist).  Recreates the context when
 * the count changes (datasets of the old context must be released first:
 * the wrappers hold one only inside a call). */
SEXP C_scc_devices(SEXP n_cores)
{
    int32_t nvis = 0;
    scc_device_count(&nvis);
    if (nvis < 1) Rf_error("scConsensus engine: no MI355X (HIP) device available");
    int want = Rf_asInteger(n_cores);
    if (want == NA_INTEGER || want < 1) want = 1;
    if (want > nvis) want = nvis;
    if (want > 64) want = 64;
    if (g_ctx && want != g_ndev) {
        scc_ctx_destroy(g_ctx);
        g_ctx = NULL;
    }
    g_ndev = want;
    ensure_ctx();
    return Rf_ScalarInteger(want);
}

static void check(int rc)
{
    if (rc != SCC_OK) Rf_error("scConsensus engine error %d: %s", rc, scc_ctx_last_error(g_ctx));
}

/* ---- the dataset handle: external pointer tagged "scc_dataset", its
 * protected slot holding c(G, N) */
static SEXP ds_tag(void) { return Rf_install("scc_dataset"); }

static void ds_finalize(SEXP h)
{
    scc_dataset* ds = (scc_dataset*)R_ExternalPtrAddr(h);
    if (ds) {
        scc_dataset_destroy(ds);
        R_ClearExternalPtr(h);
    }
}

static scc_dataset* ds_of(SEXP h, int* G, int* N)
{
    if (TYPEOF(h) != EXTPTRSXP || R_ExternalPtrTag(h) != ds_tag())
        Rf_error("scConsensus engine: not a dataset handle (use C_scc_dataset)");
    scc_dataset* ds = (scc_dataset*)R_ExternalPtrAddr(h);
    if (!ds) Rf_error("scConsensus engine: the dataset handle was released");
    SEXP dims = R_ExternalPtrProtected(h);
    if (G) *G = INTEGER(dims)[0];
    if (N) *N = INTEGER(dims)[1];
    return ds;
}

/* dgCMatrix slots (@p int, @i int, @x double), dgRMatrix slots (@p, @j, @x;
 * dim has a third entry 1) or a base double matrix -> device-resident dataset */
SEXP C_scc_dataset(SEXP x, SEXP p, SEXP i, SEXP dim)
{
    ensure_ctx();
    scc_dataset* ds = NULL;
    const int G = INTEGER(dim)[0], N = INTEGER(dim)[1];
    if (Rf_isNull(p)) {
        check(scc_dataset_create_dense(g_ctx, REAL(x), G, N, SCC_PTR_HOST, &ds));
    } else if (XLENGTH(dim) > 2 && INTEGER(dim)[2] == 1) {
        /* dgRMatrix @p is int[G+1] over genes, @j the cell columns */
        int64_t* p64 = (int64_t*)R_alloc((size_t)G + 1, sizeof(int64_t));
        for (int g = 0; g <= G; ++g) p64[g] = INTEGER(p)[g];
        check(scc_dataset_create_csr(g_ctx, p64, INTEGER(i), REAL(x), G, N, (int64_t)XLENGTH(x), SCC_PTR_HOST, &ds));
    } else {
        /* dgCMatrix @p is int[N+1]: widen to int64 once */
        int64_t* p64 = (int64_t*)R_alloc((size_t)N + 1, sizeof(int64_t));
        for (int c = 0; c <= N; ++c) p64[c] = INTEGER(p)[c];
        check(scc_dataset_create_csc(g_ctx, p64, INTEGER(i), REAL(x), G, N, (int64_t)XLENGTH(x), SCC_PTR_HOST, &ds));
    }
    SEXP dims = PROTECT(Rf_allocVector(INTSXP, 2));
    INTEGER(dims)[0] = G;
    INTEGER(dims)[1] = N;
    SEXP h = PROTECT(R_MakeExternalPtr(ds, ds_tag(), dims));
    R_RegisterCFinalizerEx(h, ds_finalize, TRUE);
    UNPROTECT(2);
    return h;
}

SEXP C_scc_release(SEXP h)
{
    if (TYPEOF(h) == EXTPTRSXP && R_ExternalPtrTag(h) == ds_tag()) ds_finalize(h);
    return R_NilValue;
}

/* returns list(union = int (1-based gene rows), nodg = int[N]) */
SEXP C_scc_de_fast(SEXP h, SEXP code, SEXP K, SEXP qthr, SEXP lfc, SEXP minpct, SEXP topn, SEXP ttest)
{
    ensure_ctx();
    int N = 0;
    scc_dataset* ds = ds_of(h, NULL, &N);
    if (XLENGTH(code) != N) Rf_error("scConsensus engine: %d cluster codes for %d cells", (int)XLENGTH(code), N);
    scc_de_params prm;
    memset(&prm, 0, sizeof(prm));
    prm.mode = SCC_DE_FAST;
    prm.q_val_thrs = Rf_asReal(qthr);
    prm.log_fc_thrs = Rf_asReal(lfc);
    prm.min_per_cent = Rf_asReal(minpct);
    prm.top_n = Rf_asInteger(topn);
    prm.test = Rf_asInteger(ttest) ? SCC_TEST_T : SCC_TEST_WILCOX; /* test.use = method (Fast:372) */
    scc_de_result* r = NULL;
    int rc = scc_de_run(g_ctx, ds, INTEGER(code), Rf_asInteger(K), &prm, &r);
    if (rc != SCC_OK && !r) check(rc);
    int32_t npairs = 0, nu = 0;
    int64_t nrows = 0;
    scc_de_result_counts(r, &npairs, &nrows, &nu);
    SEXP uni = PROTECT(Rf_allocVector(INTSXP, nu));
    scc_de_result_union(r, INTEGER(uni));
    for (int k = 0; k < nu; ++k) INTEGER(uni)[k] += 1;
    SEXP nodg = PROTECT(Rf_allocVector(INTSXP, N));
    scc_de_result_nodg(r, INTEGER(nodg));
    scc_de_result_destroy(r);
    if (rc != SCC_OK) {
        UNPROTECT(2);
        check(rc);
    }
    SEXP out = PROTECT(Rf_allocVector(VECSXP, 2));
    SET_VECTOR_ELT(out, 0, uni);
    SET_VECTOR_ELT(out, 1, nodg);
    UNPROTECT(3);
    return out;
}

/* returns list(union, q = matrix[G, P], logfc = matrix[G, P], de = raw matrix, nodg) */
SEXP C_scc_de_slow(SEXP h, SEXP code, SEXP K, SEXP qthr, SEXP fc, SEXP msf)
{
    ensure_ctx();
    int G = 0, N = 0;
    scc_dataset* ds = ds_of(h, &G, &N);
    if (XLENGTH(code) != N) Rf_error("scConsensus engine: %d cluster codes for %d cells", (int)XLENGTH(code), N);
    scc_de_params prm;
    memset(&prm, 0, sizeof(prm));
    prm.mode = SCC_DE_SLOW;
    prm.top_n = 30;
    prm.q_val_thrs = Rf_asReal(qthr);
    prm.fc_thrs = Rf_asReal(fc);
    prm.mean_scaling_factor = Rf_asReal(msf);
    scc_de_result* r = NULL;
    int rc = scc_de_run(g_ctx, ds, INTEGER(code), Rf_asInteger(K), &prm, &r);
    if (rc != SCC_OK) { /* includes SCC_ERR_RSTOP: R itself would stop() here */
        if (r) scc_de_result_destroy(r);
        check(rc);
    }
    int32_t npairs = 0, nu = 0;
    int64_t nrows = 0;
    scc_de_result_counts(r, &npairs, &nrows, &nu);
    SEXP uni = PROTECT(Rf_allocVector(INTSXP, nu));
    scc_de_result_union(r, INTEGER(uni));
    for (int k = 0; k < nu; ++k) INTEGER(uni)[k] += 1;
    SEXP q = PROTECT(Rf_allocMatrix(REALSXP, G, npairs));
    SEXP lf = PROTECT(Rf_allocMatrix(REALSXP, G, npairs));
    SEXP de = PROTECT(Rf_allocMatrix(RAWSXP, G, npairs));
    scc_de_result_pair_vectors(r, NULL, REAL(q), REAL(lf), NULL, RAW(de));
    SEXP nodg = PROTECT(Rf_allocVector(INTSXP, N));
    scc_de_result_nodg(r, INTEGER(nodg));
    scc_de_result_destroy(r);
    SEXP out = PROTECT(Rf_allocVector(VECSXP, 5));
    SET_VECTOR_ELT(out, 0, uni);
    SET_VECTOR_ELT(out, 1, q);
    SET_VECTOR_ELT(out, 2, lf);
    SET_VECTOR_ELT(out, 3, de);
    SET_VECTOR_ELT(out, 4, nodg);
    UNPROTECT(6);
    return out;
}

/* returns a "dist" object body (double vector, N(N-1)/2, R order); the R
 * wrapper sets the Size/Diag/Upper/method attributes and class "dist".  The
 * engine streams it from HBM into this vector in column tiles (pageable
 * memory: a pinned staging ring). */
SEXP C_scc_distance(SEXP h, SEXP genes, SEXP metric, SEXP ncomp)
{
    ensure_ctx();
    int G = 0, N = 0;
    scc_dataset* ds = ds_of(h, &G, &N);
    const int nu = LENGTH(genes);
    int32_t* g0 = (int32_t*)R_alloc((size_t)nu, sizeof(int32_t));
    for (int k = 0; k < nu; ++k) {
        g0[k] = INTEGER(genes)[k] - 1;
        if (g0[k] < 0 || g0[k] >= G) Rf_error("scConsensus engine: gene row %d out of range", g0[k] + 1);
    }
    SEXP d = PROTECT(Rf_allocVector(REALSXP, (R_xlen_t)N * (N - 1) / 2));
    int rc = scc_distance(g_ctx, ds, g0, nu, Rf_asInteger(metric), Rf_asInteger(ncomp), REAL(d), SCC_PTR_HOST, 0);
    if (rc != SCC_OK) {
        UNPROTECT(1);
        check(rc);
    }
    UNPROTECT(1);
    return d;
}

/* mean(summary(cluster::silhouette(groups, as.matrix(d)))$clus.avg.widths)
 * (Fast:433) on the engine-kept output of the last C_scc_distance call.
 * R's silhouette() returns NA for fewer than 2 groups or as many groups as
 * cells, and summary(NA)$clus.avg.widths then stops ("$ operator is invalid
 * for atomic vectors"): the same stop here.  Any other failure (no kept
 * distance of this size, a HIP error) is an error too, never a silent NA. */
SEXP C_scc_si(SEXP groups)
{
    ensure_ctx();
    const int N = LENGTH(groups);
    int32_t* g = (int32_t*)R_alloc((size_t)N, sizeof(int32_t));
    for (int k = 0; k < N; ++k) g[k] = INTEGER(groups)[k];
    double* avg = (double*)R_alloc((size_t)N, sizeof(double));
    int32_t ng = 0;
    int rc = scc_silhouette(g_ctx, N, g, NULL, 0, NULL, avg, &ng);
    if (rc == SCC_ERR_INVALID && ng > 0 && (ng < 2 || ng >= N))
        Rf_error("$ operator is invalid for atomic vectors");
    check(rc);
    double s = 0.0;
    for (int k = 0; k < ng; ++k) s += avg[k];
    return Rf_ScalarReal(s / ng);
}

/* n from the length of a "dist" body, n (n - 1) / 2 */
static int64_t dist_n(SEXP d)
{
    const double nd = (double)XLENGTH(d);
    int64_t n = (int64_t)((1.0 + sqrt(1.0 + 8.0 * nd)) / 2.0 + 0.5);
    if (n * (n - 1) / 2 != (int64_t)XLENGTH(d)) Rf_error("scConsensus engine: not a dist body (length %.0f)", nd);
    return n;
}

/* cutreeDynamic(dendro, distM = as.matrix(d), deepSplit, pamStage = FALSE,
 * minClusterSize) with method "hybrid" and the default cut height
 * (Fast:421-427), on the packed d: merge is the hclust merge matrix ((n-1) x 2
 * integer, column-major as R stores it), height its heights.  Returns the
 * integer labels (0 = unassigned, 1.. by decreasing size), as cutreeDynamic. */
SEXP C_scc_cutree(SEXP merge, SEXP height, SEXP d, SEXP deep, SEXP minsize)
{
    const int64_t n = dist_n(d);
    if (XLENGTH(merge) != 2 * (n - 1) || XLENGTH(height) != n - 1)
        Rf_error("scConsensus engine: merge / height do not match the dist of %lld cells", (long long)n);
    SEXP m = PROTECT(Rf_coerceVector(merge, INTSXP));
    SEXP lab = PROTECT(Rf_allocVector(INTSXP, n));
    const int rc = scc_cutree_hybrid(INTEGER(m), REAL(height), n, REAL(d), Rf_asInteger(deep), Rf_asInteger(minsize),
                                     INTEGER(lab), NULL);
    UNPROTECT(2);
    if (rc != SCC_OK) Rf_error("scConsensus engine: cutree failed (%d)", rc);
    return lab;
}

/* hclust(d, method = "ward.D2") (Fast:406-411): list(merge, height, order) of
 * an R hclust object (the wrapper adds labels / method / call / dist.method) */
SEXP C_scc_hclust(SEXP d)
{
    const int64_t n = dist_n(d);
    SEXP merge = PROTECT(Rf_allocMatrix(INTSXP, (int)(n - 1), 2));
    SEXP height = PROTECT(Rf_allocVector(REALSXP, n - 1));
    SEXP order = PROTECT(Rf_allocVector(INTSXP, n));
    const int rc = scc_hclust_ward_d2(REAL(d), n, INTEGER(merge), REAL(height), INTEGER(order));
    if (rc != SCC_OK) {
        UNPROTECT(3);
        Rf_error("scConsensus engine: hclust failed (%d)", rc);
    }
    SEXP out = PROTECT(Rf_allocVector(VECSXP, 3));
    SET_VECTOR_ELT(out, 0, merge);
    SET_VECTOR_ELT(out, 1, height);
    SET_VECTOR_ELT(out, 2, order);
    UNPROTECT(4);
    return out;
}

static const R_CallMethodDef call_methods[] = {
    {"C_scc_dataset", (DL_FUNC)&C_scc_dataset, 4},
    {"C_scc_release", (DL_FUNC)&C_scc_release, 1},
    {"C_scc_de_fast", (DL_FUNC)&C_scc_de_fast, 8},
    {"C_scc_de_slow", (DL_FUNC)&C_scc_de_slow, 6},
    {"C_scc_distance", (DL_FUNC)&C_scc_distance, 4},
    {"C_scc_si", (DL_FUNC)&C_scc_si, 1},
    {"C_scc_devices", (DL_FUNC)&C_scc_devices, 1},
    {"C_scc_cutree", (DL_FUNC)&C_scc_cutree, 5},
    {"C_scc_hclust", (DL_FUNC)&C_scc_hclust, 1},
    {NULL, NULL, 0}};

/* the package is scConsensus (NAMESPACE: useDynLib(scConsensus, .registration = TRUE)) */
void R_init_scConsensus(DllInfo* dll)
{
    R_registerRoutines(dll, NULL, call_methods, NULL, NULL);
    R_useDynamicSymbols(dll, FALSE);
}
