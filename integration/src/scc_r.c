/*
 * scc_r.c — R `.Call` glue for libscc (include/scc.h).  Compiled only where R
 * headers exist (R CMD INSTALL of the wrapper package; R is absent from the
 * build container).  The glue never lets a C++ frame unwind through R: every
 * libscc entry point returns an int status, and Rf_error() is raised only
 * here, after the library call returned.
 *
 * Bindings (reference call sites they replace):
 *   C_scc_de_fast   R/reclusterDEConsensusFast.R:57-392 (pair loop, ComputePairWiseDE, top_n, unique)
 *   C_scc_de_slow   R/reclusterDEConsensus.R:32-227
 *   C_scc_distance  R/reclusterDEConsensusFast.R:398-400 (prcomp_irlba + dist), :403 (1 - cor)
 */
#include <R.h>
#include <Rinternals.h>
#include <R_ext/Rdynload.h>
#include <stdint.h>
#include <string.h>

#include "scc.h"

static scc_ctx* g_ctx = NULL;

static void ensure_ctx(void)
{
    if (g_ctx) return;
    scc_opts o;
    memset(&o, 0, sizeof(o));
    if (scc_ctx_create(&o, &g_ctx) != SCC_OK) Rf_error("scConsensus engine: no MI355X (HIP) device available");
}

static void check(int rc)
{
    if (rc != SCC_OK) Rf_error("scConsensus engine error %d: %s", rc, scc_ctx_last_error(g_ctx));
}

/* dgCMatrix slots (@p int, @i int, @x double), dgRMatrix slots (@p, @j, @x;
 * dim has a third entry 1) or a base double matrix */
static scc_dataset* dataset_from(SEXP x, SEXP p, SEXP i, SEXP dim)
{
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
    return ds;
}

/* returns list(union = int (1-based gene rows), nodg = int[N]) */
SEXP C_scc_de_fast(SEXP x, SEXP p, SEXP i, SEXP dim, SEXP code, SEXP K, SEXP qthr, SEXP lfc, SEXP minpct, SEXP topn,
                   SEXP ttest)
{
    ensure_ctx();
    scc_dataset* ds = dataset_from(x, p, i, dim);
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
    if (rc != SCC_OK && !r) {
        scc_dataset_destroy(ds);
        check(rc);
    }
    int32_t npairs = 0, nu = 0;
    int64_t nrows = 0;
    scc_de_result_counts(r, &npairs, &nrows, &nu);
    SEXP uni = PROTECT(Rf_allocVector(INTSXP, nu));
    scc_de_result_union(r, INTEGER(uni));
    for (int k = 0; k < nu; ++k) INTEGER(uni)[k] += 1;
    SEXP nodg = PROTECT(Rf_allocVector(INTSXP, INTEGER(dim)[1]));
    scc_de_result_nodg(r, INTEGER(nodg));
    scc_de_result_destroy(r);
    scc_dataset_destroy(ds);
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

/* returns list(union, q = matrix[G, P], logfc = matrix[G, P], de = logical matrix, nodg) */
SEXP C_scc_de_slow(SEXP x, SEXP p, SEXP i, SEXP dim, SEXP code, SEXP K, SEXP qthr, SEXP fc, SEXP msf)
{
    ensure_ctx();
    scc_dataset* ds = dataset_from(x, p, i, dim);
    scc_de_params prm;
    memset(&prm, 0, sizeof(prm));
    prm.mode = SCC_DE_SLOW;
    prm.top_n = 30;
    prm.q_val_thrs = Rf_asReal(qthr);
    prm.fc_thrs = Rf_asReal(fc);
    prm.mean_scaling_factor = Rf_asReal(msf);
    scc_de_result* r = NULL;
    int rc = scc_de_run(g_ctx, ds, INTEGER(code), Rf_asInteger(K), &prm, &r);
    if (rc != SCC_OK) {  /* includes SCC_ERR_RSTOP: R itself would stop() here */
        if (r) scc_de_result_destroy(r);
        scc_dataset_destroy(ds);
        check(rc);
    }
    const int G = INTEGER(dim)[0];
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
    SEXP nodg = PROTECT(Rf_allocVector(INTSXP, INTEGER(dim)[1]));
    scc_de_result_nodg(r, INTEGER(nodg));
    scc_de_result_destroy(r);
    scc_dataset_destroy(ds);
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
 * wrapper sets the Size/Diag/Upper/method attributes and class "dist". */
SEXP C_scc_distance(SEXP x, SEXP p, SEXP i, SEXP dim, SEXP genes, SEXP metric, SEXP ncomp)
{
    ensure_ctx();
    scc_dataset* ds = dataset_from(x, p, i, dim);
    const int N = INTEGER(dim)[1];
    const int nu = LENGTH(genes);
    int32_t* g0 = (int32_t*)R_alloc((size_t)nu, sizeof(int32_t));
    for (int k = 0; k < nu; ++k) g0[k] = INTEGER(genes)[k] - 1;
    SEXP d = PROTECT(Rf_allocVector(REALSXP, (R_xlen_t)N * (N - 1) / 2));
    int rc = scc_distance(g_ctx, ds, g0, nu, Rf_asInteger(metric), Rf_asInteger(ncomp), REAL(d), SCC_PTR_HOST, 0);
    scc_dataset_destroy(ds);
    if (rc != SCC_OK) {
        UNPROTECT(1);
        check(rc);
    }
    UNPROTECT(1);
    return d;
}

static const R_CallMethodDef call_methods[] = {
    {"C_scc_de_fast", (DL_FUNC)&C_scc_de_fast, 11},
    {"C_scc_de_slow", (DL_FUNC)&C_scc_de_slow, 9},
    {"C_scc_distance", (DL_FUNC)&C_scc_distance, 7},
    {NULL, NULL, 0}};

void R_init_scConsensusAMD(DllInfo* dll)
{
    R_registerRoutines(dll, NULL, call_methods, NULL, NULL);
    R_useDynamicSymbols(dll, FALSE);
}
