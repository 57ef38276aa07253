/*
 * oracle/scc_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference R semantics of the scConsensus hot path
 * (pairwise Wilcoxon DE + BH + filters + top-N union).  It exists to CHECK the
 * MI355X engine (scconsensus_amd/); it is never linked into, loaded by, or
 * called from the product path.  Only tests/, __graft_entry__.smoke() and the
 * bench.py `cpu_baseline` leg may load it.
 *
 * It deliberately mirrors the reference's algorithm step for step (per pair:
 * gather both clusters, per gene a full average-tie rank of n_i+n_j doubles,
 * R's wilcox.test normal/exact rule, BH, filters) and NOT the engine's
 * count-based algorithm, so a match between the two is evidence.
 *
 * Reference call sites restated (paths relative to the reference repo):
 *   R/reclusterDEConsensusFast.R:40-53   cluster selection (done by the caller; codes in)
 *   R/reclusterDEConsensusFast.R:229-291 pct / log-mean-expm1 / logFC feature filters
 *   R/reclusterDEConsensusFast.R:78-91   WilcoxDETest -> stats::wilcox.test(x ~ group)
 *   R/reclusterDEConsensusFast.R:185-196 DiffTTest -> stats::t.test(x, y) (Welch), test.use = "t"
 *   R/reclusterDEConsensusFast.R:335-351 order(p, -avg_logFC); p.adjust(.,"BH")
 *   R/reclusterDEConsensusFast.R:359-392 pair loop, dim>1 rule, q filter, top_n, unique
 *   R/reclusterDEConsensus.R:32-36       global mean(expm1(X)) threshold
 *   R/reclusterDEConsensus.R:69-187      per-gene wilcox.test, mean diff, gate, BH n=G, DE rule
 *   R/reclusterDEConsensus.R:206-227     sort(|logfc|, decreasing) first 30, union
 *   R/reclusterDEConsensus(Fast).R:440-443 nodg
 *
 * The arithmetic itself lives in R base (not vendored, R absent from the build
 * container): src/main/summary.c (mean: LDOUBLE two-pass), src/main/sort.c
 * (rank "average"), src/library/stats/R/wilcox.test.R, src/nmath/wilcox.c
 * (cwilcox/pwilcox), src/nmath/pnorm.c (Cody 1993, ACM TOMS 715),
 * src/library/stats/R/p.adjust.R, src/nmath/choose.c.  These are restated
 * from the published algorithms; deviations are marked DEVIATION below.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>

#define ORC_OK 0
#define ORC_ERR_ALLOC 1
#define ORC_ERR_RSTOP 5 /* a condition under which the R code would stop() */

/* ---------------------------------------------------------------- R mean */
/* R summary.c: LDOUBLE s = sum; s /= n; if finite: t = sum(x - s); s += t/n */
double orc_r_mean(const double *x, long n)
{
    long double s = 0.0L;
    for (long i = 0; i < n; ++i) s += x[i];
    s /= (long double)n;
    if (isfinite((double)s)) {
        long double t = 0.0L;
        for (long i = 0; i < n; ++i) t += (x[i] - s);
        s += t / (long double)n;
    }
    return (double)s;
}

/* ---------------------------------------------------------------- rank */
typedef struct { double v; int i; } orc_vi;

static int cmp_vi(const void *a, const void *b)
{
    const orc_vi *x = (const orc_vi *)a, *y = (const orc_vi *)b;
    if (x->v < y->v) return -1;
    if (x->v > y->v) return 1;
    return (x->i < y->i) ? -1 : (x->i > y->i);
}

/* R rank(x, ties.method = "average") (sort.c do_rank): rk = (i + j + 2) / 2.
 * Returns the tie term sum(NTIES^3 - NTIES) accumulated as R's sum() does
 * (LDOUBLE over double terms) and whether any tie exists. */
static double rank_average(const double *v, int n, double *rk, orc_vi *scr, int *has_ties)
{
    for (int i = 0; i < n; ++i) { scr[i].v = v[i]; scr[i].i = i; }
    qsort(scr, (size_t)n, sizeof(orc_vi), cmp_vi);
    long double tsum = 0.0L;
    *has_ties = 0;
    for (int i = 0; i < n;) {
        int j = i;
        while (j < n - 1 && scr[j + 1].v == scr[i].v) ++j;
        double r = (double)(i + j + 2) / 2.0;
        for (int k = i; k <= j; ++k) rk[scr[k].i] = r;
        double t = (double)(j - i + 1);
        tsum += (long double)(t * t * t - t);
        if (j > i) *has_ties = 1;
        i = j + 1;
    }
    return (double)tsum;
}

/* ---------------------------------------------------------------- pnorm */
/* R nmath/pnorm.c pnorm_both (Cody's rational Chebyshev approximations). */
static const double PN_A[5] = {2.2352520354606839287, 161.02823106855587881, 1067.6894854603709582,
                               18154.981253343561249, 0.065682337918207449113};
static const double PN_B[4] = {47.20258190468824187, 976.09855173777669322, 10260.932208618978205,
                               45507.789335026729956};
static const double PN_C[9] = {0.39894151208813466764, 8.8831497943883759412, 93.506656132177855979,
                               597.27027639480026226, 2494.5375852903726711, 6848.1904505362823326,
                               11602.651437647350124, 9842.7148383839780218, 1.0765576773720192317e-8};
static const double PN_D[8] = {22.266688044328115691, 235.38790178262499861, 1519.377599407554805,
                               6485.558298266760755, 18615.571640885098091, 34900.952721145977266,
                               38912.003286093271411, 19685.429676859990727};
static const double PN_P[6] = {0.21589853405795699, 0.1274011611602473639, 0.022235277870649807,
                               0.001421619193227893466, 2.9112874951168792e-5, 0.02307344176494017303};
static const double PN_Q[5] = {1.28426009614491121, 0.468238212480865118, 0.0659881378689285515,
                               0.00378239633202758244, 7.29751555083966205e-5};
#define PN_SQRT_32 5.656854249492380195206754896838
#define PN_1_SQRT_2PI 0.398942280401432677939946059934

/* i_tail: 0 = lower only, 1 = upper only, 2 = both (R's convention). */
void orc_pnorm_both(double x, double *cum, double *ccum, int i_tail)
{
    double xden, xnum, temp, del, xsq, y;
    const double eps = DBL_EPSILON * 0.5;
    int lower = i_tail != 1, upper = i_tail != 0;
    y = fabs(x);
    if (y <= 0.67448975) {
        if (y > eps) {
            xsq = x * x;
            xnum = PN_A[4] * xsq;
            xden = xsq;
            for (int i = 0; i < 3; ++i) {
                xnum = (xnum + PN_A[i]) * xsq;
                xden = (xden + PN_B[i]) * xsq;
            }
        } else {
            xnum = xden = 0.0;
        }
        temp = x * (xnum + PN_A[3]) / (xden + PN_B[3]);
        if (lower) *cum = 0.5 + temp;
        if (upper) *ccum = 0.5 - temp;
    } else if (y <= PN_SQRT_32) {
        xnum = PN_C[8] * y;
        xden = y;
        for (int i = 0; i < 7; ++i) {
            xnum = (xnum + PN_C[i]) * y;
            xden = (xden + PN_D[i]) * y;
        }
        temp = (xnum + PN_C[7]) / (xden + PN_D[7]);
        xsq = trunc(y * 16.0) / 16.0;
        del = (y - xsq) * (y + xsq);
        *cum = exp(-xsq * xsq * 0.5) * exp(-del * 0.5) * temp;
        *ccum = 1.0 - *cum;
        if (x > 0.) { temp = *cum; if (lower) *cum = *ccum; *ccum = temp; }
    } else if ((lower && -37.5193 < x && x < 8.2924) || (upper && -8.2924 < x && x < 37.5193)) {
        xsq = 1.0 / (x * x);
        xnum = PN_P[5] * xsq;
        xden = xsq;
        for (int i = 0; i < 4; ++i) {
            xnum = (xnum + PN_P[i]) * xsq;
            xden = (xden + PN_Q[i]) * xsq;
        }
        temp = xsq * (xnum + PN_P[4]) / (xden + PN_Q[4]);
        temp = (PN_1_SQRT_2PI - temp) / y;
        xsq = trunc(x * 16.0) / 16.0;
        del = (x - xsq) * (x + xsq);
        *cum = exp(-xsq * xsq * 0.5) * exp(-del * 0.5) * temp;
        *ccum = 1.0 - *cum;
        if (x > 0.) { temp = *cum; if (lower) *cum = *ccum; *ccum = temp; }
    } else {
        if (x > 0) { *cum = 1.0; *ccum = 0.0; }
        else { *cum = 0.0; *ccum = 1.0; }
    }
}

double orc_pnorm(double x, int lower_tail)
{
    double p = 0, cp = 0;
    if (isnan(x)) return x;
    orc_pnorm_both(x, &p, &cp, lower_tail ? 0 : 1);
    return lower_tail ? p : cp;
}

/* ---------------------------------------------------------------- pwilcox */
/* R nmath/wilcox.c cwilcox with memo w[i][j][k] (i <= j, k <= floor(i*j/2)). */
#define WMAX 50
static double *orc_w[WMAX + 1][WMAX + 1];

static double cwilcox(int k, int m, int n)
{
    int u = m * n;
    if (k < 0 || k > u) return 0;
    int c = u / 2;
    if (k > c) k = u - k;
    int i, j;
    if (m < n) { i = m; j = n; } else { i = n; j = m; }
    if (j == 0) return (k == 0);
    if (j > 0 && k < j) return cwilcox(k, i, k);
    if (orc_w[i][j] == NULL) {
        orc_w[i][j] = (double *)malloc(sizeof(double) * (size_t)(c + 1));
        for (int l = 0; l <= c; ++l) orc_w[i][j][l] = -1;
    }
    if (orc_w[i][j][k] < 0) {
        orc_w[i][j][k] = cwilcox(k - j, i - 1, j) + cwilcox(k, i, j - 1);
    }
    return orc_w[i][j][k];
}

/* DEVIATION: R's choose() switches to exp(lfastchoose()) rounded when both
 * k and n-k are >= 30; we use the k<30 product formula for every k (relative
 * difference ~1e-14, far inside the 1e-6 p-value tolerance). */
double orc_choose(double n, double k)
{
    if (n - k < k) k = n - k;
    if (k < 0) return 0;
    if (k == 0) return 1;
    double r = n;
    for (int j = 2; j <= (int)k; ++j) r *= (n - j + 1) / j;
    return nearbyint(r);
}

double orc_pwilcox(double q, int m, int n, int lower_tail)
{
    q = floor(q + 1e-7);
    if (q < 0.0) return lower_tail ? 0.0 : 1.0;
    if (q >= (double)m * n) return lower_tail ? 1.0 : 0.0;
    double c = orc_choose((double)m + n, (double)n);
    double p = 0;
    if (q <= ((double)m * n / 2)) {
        for (int i = 0; i <= (int)q; ++i) p += cwilcox(i, m, n) / c;
    } else {
        q = (double)m * n - q;
        for (int i = 0; i < (int)q; ++i) p += cwilcox(i, m, n) / c;
        lower_tail = !lower_tail;
    }
    return lower_tail ? p : (0.5 - p + 0.5);
}

void orc_wilcox_free(void)
{
    for (int i = 0; i <= WMAX; ++i)
        for (int j = 0; j <= WMAX; ++j) { free(orc_w[i][j]); orc_w[i][j] = NULL; }
}

/* ---------------------------------------------------------------- wilcox.test */
/* stats:::wilcox.test.default(x, y, alternative = "two.sided", mu = 0,
 * exact = NULL, correct = TRUE) — p.value.  Outputs W (the STATISTIC) and the
 * tie term sum(NTIES^3 - NTIES); *method = 1 exact, 0 normal approximation. */
double orc_wilcox_p_scratch(const double *x, int nx, const double *y, int ny, double *W_out,
                            double *ties_out, int *method, double *buf, double *rk, orc_vi *scr)
{
    int n = nx + ny;
    for (int i = 0; i < nx; ++i) buf[i] = x[i];
    for (int i = 0; i < ny; ++i) buf[nx + i] = y[i];
    int has_ties = 0;
    double tsum = rank_average(buf, n, rk, scr, &has_ties);
    long double rs = 0.0L;
    for (int i = 0; i < nx; ++i) rs += rk[i];
    double dnx = (double)nx, dny = (double)ny;
    double W = (double)rs - dnx * (dnx + 1) / 2;
    if (W_out) *W_out = W;
    if (ties_out) *ties_out = tsum;
    int exact = (nx < 50) && (ny < 50);
    if (exact && !has_ties) {
        if (method) *method = 1;
        double p;
        if (W > (dnx * dny / 2))
            p = orc_pwilcox(W - 1, nx, ny, 0);
        else
            p = orc_pwilcox(W, nx, ny, 1);
        return fmin(2 * p, 1.0);
    }
    if (method) *method = 0;
    double z = W - dnx * dny / 2;
    double sigma = sqrt((dnx * dny / 12) * ((dnx + dny + 1) - tsum / ((dnx + dny) * (dnx + dny - 1))));
    double corr = (z > 0) ? 0.5 : ((z < 0) ? -0.5 : 0.0);
    z = (z - corr) / sigma;
    double pl = orc_pnorm(z, 1), pu = orc_pnorm(z, 0);
    if (isnan(pl) || isnan(pu)) return NAN;
    return 2 * fmin(pl, pu);
}

double orc_wilcox_p(const double *x, int nx, const double *y, int ny, double *W_out, double *ties_out,
                    int *method)
{
    int n = nx + ny;
    double *buf = (double *)malloc(sizeof(double) * (size_t)n * 2);
    orc_vi *scr = (orc_vi *)malloc(sizeof(orc_vi) * (size_t)n);
    double p = orc_wilcox_p_scratch(x, nx, y, ny, W_out, ties_out, method, buf, buf + n, scr);
    free(buf);
    free(scr);
    return p;
}

/* ---------------------------------------------------------------- p.adjust */
typedef struct { double p; int i; } orc_pi;

static int cmp_p_desc(const void *a, const void *b)
{
    const orc_pi *x = (const orc_pi *)a, *y = (const orc_pi *)b;
    if (x->p > y->p) return -1;
    if (x->p < y->p) return 1;
    return (x->i < y->i) ? -1 : (x->i > y->i); /* stable, as R's radix order */
}

/* stats::p.adjust(p, "BH", n): NaN/NA entries excluded from ranking and kept NA;
 * n < 0 means the lazy default (number of non-NA entries). */
void orc_p_adjust_bh(const double *p, int len, long n, double *q)
{
    int lp = 0;
    orc_pi *v = (orc_pi *)malloc(sizeof(orc_pi) * (size_t)(len > 0 ? len : 1));
    for (int i = 0; i < len; ++i) {
        if (!isnan(p[i])) { v[lp].p = p[i]; v[lp].i = i; ++lp; }
        q[i] = NAN;
    }
    if (n < 0) n = lp;
    qsort(v, (size_t)lp, sizeof(orc_pi), cmp_p_desc);
    double cm = INFINITY;
    for (int t = 0; t < lp; ++t) {
        double rank = (double)(lp - t); /* i <- lp:1L */
        double val = ((double)n / rank) * v[t].p;
        if (val < cm) cm = val;
        q[v[t].i] = fmin(1.0, cm);
    }
    free(v);
}

/* ---------------------------------------------------------------- t test */
/* R var() (src/library/stats/src/cov.c, one complete vector): long double
 * mean, then the long double sum of squared deviations / (n - 1). */
double orc_r_var(const double *x, long n, double mean)
{
    long double s = 0.0L;
    for (long i = 0; i < n; ++i) s += ((long double)x[i] - mean) * ((long double)x[i] - mean);
    return (double)(s / (long double)(n - 1));
}

/* Stirling-series correction lgamma(x) - [(x - 1/2) log x - x + log sqrt(2 pi)], x >= 10 */
static double lgammacor(double x)
{
    const double r = 1.0 / (x * x);
    return (1.0 / 12 - r * (1.0 / 360 - r * (1.0 / 1260 - r * (1.0 / 1680 - r * (1.0 / 1188 -
            r * (691.0 / 360360 - r / 156)))))) / x;
}

/* log B(a, b) in R nmath/lbeta.c's three regimes (no lgamma cancellation for
 * large arguments) */
static double orc_lbeta(double a, double b)
{
    const double p = fmin(a, b), q = fmax(a, b);
    const double ln_sqrt_2pi = 0.918938533204672741780329736406;
    if (p >= 10) {
        const double corr = lgammacor(p) + lgammacor(q) - lgammacor(p + q);
        return log(q) * -0.5 + ln_sqrt_2pi + corr + (p - 0.5) * log(p / (p + q)) + q * log1p(-p / (p + q));
    }
    if (q >= 10) {
        const double corr = lgammacor(q) - lgammacor(p + q);
        return lgamma(p) + corr + p - p * log(p + q) + (q - 0.5) * log1p(-p / (p + q));
    }
    return lgamma(p) + lgamma(q) - lgamma(p + q);
}

/* log B(a, b) in long double (the series' prefactor) */
static long double lbeta_l(long double a, long double b)
{
    return lgammal(a) + lgammal(b) - lgammal(a + b);
}

/* I_x(a, b) by its hypergeometric power series (DLMF 8.17.8, 15.2.1):
 *   I_x(a, b) = x^a (1-x)^b / (a B(a, b)) * sum_{n >= 0} (a+b)_n / (a+1)_n x^n,
 * every term positive, summed in long double until a term no longer moves the
 * sum.  lx = log x, l1x = log(1 - x), both from the caller's cancellation-free
 * x and 1 - x.  This is deliberately NOT the continued fraction the GPU kernel
 * evaluates (scc_select.hip ibeta_cf_den), so the oracle checks the kernel with
 * an independent algorithm (and both are pinned to scipy in the tests). */
static long double ibeta_series(long double a, long double b, long double x, long double lx, long double l1x)
{
    long double sum = 1.0L, term = 1.0L;
    for (long k = 0; k < 40000000L; ++k) {
        term *= (a + b + (long double)k) / (a + 1.0L + (long double)k) * x;
        const long double s2 = sum + term;
        if (s2 == sum) break;
        sum = s2;
    }
    return expl(a * lx + b * l1x - lbeta_l(a, b)) / a * sum;
}

/* I_x(a, b) (lower = 1) or 1 - I_x(a, b) (lower = 0), x given with its
 * complement y = 1 - x computed by the caller without cancellation.  The
 * smaller tail (x below or above the mean a / (a + b)) is summed directly:
 * its series decreases from the first term; the other tail is 1 minus it.
 * DEVIATION: R's pbeta is TOMS 708 (bratio); Student t tails agree with scipy
 * to ~1e-12 relative (tests/test_oracle.py). */
static double orc_pbeta2(double x, double y, double a, double b, int lower)
{
    if (x <= 0.0) return lower ? 0.0 : 1.0;
    if (y <= 0.0) return lower ? 1.0 : 0.0;
    const long double lx = x > 0.5 ? log1pl(-(long double)y) : logl((long double)x);
    const long double ly = y > 0.5 ? log1pl(-(long double)x) : logl((long double)y);
    if ((long double)x * (a + b) <= (long double)a) { /* lower tail the smaller */
        const long double lo = ibeta_series(a, b, x, lx, ly);
        return (double)(lower ? lo : 1.0L - lo);
    }
    const long double up = ibeta_series(b, a, y, ly, lx); /* 1 - I_x(a, b) = I_y(b, a) */
    return (double)(lower ? 1.0L - up : up);
}

/* R nmath/pt.c, lower_tail, non-log */
double orc_pt(double x, double n, int lower_tail)
{
    if (n > 4e5) {
        const double val = 1.0 / (4.0 * n);
        return orc_pnorm(x * (1.0 - val) / sqrt(1.0 + x * x * 2.0 * val), lower_tail);
    }
    const double nx = 1 + (x / n) * x;
    double val;
    if (nx > 1e100) {
        const double lval = -0.5 * n * (2 * log(fabs(x)) - log(n)) - orc_lbeta(0.5 * n, 0.5) - log(0.5 * n);
        val = exp(lval);
    } else {
        val = (n > x * x) ? orc_pbeta2(x * x / (n + x * x), n / (n + x * x), 0.5, n / 2.0, 0)
                          : orc_pbeta2(1.0 / nx, (x / n) * x / nx, n / 2.0, 0.5, 1);
    }
    if (x <= 0.0) lower_tail = !lower_tail;
    val /= 2.0;
    return lower_tail ? (0.5 - val + 0.5) : val;
}

/* stats::t.test(x, y)$p.value (Welch, two-sided, mu = 0; R/t.test.R).
 * *constant = 1 where R stops with "data are essentially constant". */
double orc_t_test_p(const double *x, int nx, const double *y, int ny, double *tstat, int *constant)
{
    const double mx = orc_r_mean(x, nx), my = orc_r_mean(y, ny);
    const double vx = orc_r_var(x, nx, mx), vy = orc_r_var(y, ny, my);
    const double sx = sqrt(vx / nx), sy = sqrt(vy / ny);
    const double se = sqrt(sx * sx + sy * sy);
    const double df = pow(se, 4) / (pow(sx, 4) / (nx - 1) + pow(sy, 4) / (ny - 1));
    *constant = se < 10 * DBL_EPSILON * fmax(fabs(mx), fabs(my));
    const double t = (mx - my) / se;
    if (tstat) *tstat = t;
    return 2 * orc_pt(-fabs(t), df, 1);
}

/* ---------------------------------------------------------------- Fast driver */
typedef struct {
    double q_val_thrs;   /* qValThrs */
    double log_fc_thrs;  /* logFCThrs (natural log) */
    double min_per_cent; /* minPerCent */
    int top_n;           /* NumbertopDEGenes */
    int test;            /* 0: wilcox (Fast:78-91), 1: t (DiffTTest, Fast:185-196) */
    int status;          /* out: ORC_ERR_RSTOP where R's t.test stops (constant data) */
} orc_fast_params;

typedef struct {
    int gene;
    double p, nlfc; /* order keys: p asc (NA last), -avg_logFC asc */
} orc_row_key;

static int cmp_row_key(const void *a, const void *b)
{
    const orc_row_key *x = (const orc_row_key *)a, *y = (const orc_row_key *)b;
    int xn = isnan(x->p), yn = isnan(y->p);
    if (xn != yn) return xn - yn;
    if (!xn) {
        if (x->p < y->p) return -1;
        if (x->p > y->p) return 1;
    }
    if (x->nlfc < y->nlfc) return -1;
    if (x->nlfc > y->nlfc) return 1;
    return (x->gene < y->gene) ? -1 : (x->gene > y->gene);
}

/* X: gene-major dense, X[g*N + c]; code[c] in [0,K) or -1 (excluded).
 * Rows are written pair-major in R's row order (tested features of pair (i,j),
 * ordered by order(p, -avg_logFC)).  Capacity of the row arrays must be
 * >= P*G.  Returns the number of rows; union[] gets unique(Gene) of the
 * top_n-filtered DE rows.  Per-pair tested counts go to pair_tested[P]. */
long orc_de_fast(const double *X, int G, int N, const int *code, int K, const orc_fast_params *prm,
                 int *pair_tested, int *row_gene, double *row_p, double *row_q, double *row_lfc,
                 double *row_pct1, double *row_pct2, double *row_W, double *row_ties,
                 uint8_t *row_flags, int *union_genes, int *n_union)
{
    int *cells = (int *)malloc(sizeof(int) * (size_t)N);
    int *cstart = (int *)calloc((size_t)K + 1, sizeof(int));
    for (int c = 0; c < N; ++c)
        if (code[c] >= 0) cstart[code[c] + 1]++;
    for (int a = 0; a < K; ++a) cstart[a + 1] += cstart[a];
    int *fill = (int *)malloc(sizeof(int) * (size_t)K);
    memcpy(fill, cstart, sizeof(int) * (size_t)K);
    for (int c = 0; c < N; ++c)
        if (code[c] >= 0) cells[fill[code[c]]++] = c; /* which(labels == cl): ascending */
    free(fill);
    int nmax = 0;
    for (int a = 0; a < K; ++a)
        if (cstart[a + 1] - cstart[a] > nmax) nmax = cstart[a + 1] - cstart[a];

    double *xi = (double *)malloc(sizeof(double) * (size_t)(2 * nmax + 1));
    double *yj = xi + nmax;
    double *tmp = (double *)malloc(sizeof(double) * (size_t)(4 * nmax + 2));
    orc_vi *scr = (orc_vi *)malloc(sizeof(orc_vi) * (size_t)(2 * nmax + 1));
    orc_row_key *keys = (orc_row_key *)malloc(sizeof(orc_row_key) * (size_t)G);
    double *pct1 = (double *)malloc(sizeof(double) * (size_t)G * 6);
    double *pct2 = pct1 + G, *m1 = pct1 + 2 * (size_t)G, *m2 = pct1 + 3 * (size_t)G;
    double *pv = pct1 + 4 * (size_t)G, *qv = pct1 + 5 * (size_t)G;
    double *Wv = (double *)malloc(sizeof(double) * (size_t)G * 2), *Tv = Wv + G;
    int *feat = (int *)malloc(sizeof(int) * (size_t)G);
    long nrows = 0;
    int pidx = 0;
    /* union bookkeeping */
    uint8_t *in_union = (uint8_t *)calloc((size_t)G, 1);
    int nu = 0;

    for (int i = 0; i < K - 1; ++i) {
        for (int j = i + 1; j < K; ++j, ++pidx) {
            const int *ci = cells + cstart[i], *cj = cells + cstart[j];
            int ni = cstart[i + 1] - cstart[i], nj = cstart[j + 1] - cstart[j];
            /* Fast:229-256 pct filter (round(., 16) is the identity for these values) */
            int nf = 0;
            for (int g = 0; g < G; ++g) {
                const double *row = X + (size_t)g * N;
                double s1 = 0, s2 = 0;
                for (int k = 0; k < ni; ++k) s1 += (row[ci[k]] > 0);
                for (int k = 0; k < nj; ++k) s2 += (row[cj[k]] > 0);
                pct1[g] = 100 * s1 / ni;
                pct2[g] = 100 * s2 / nj;
                double amax = fmax(pct1[g], pct2[g]);
                if (amax > prm->min_per_cent) feat[nf++] = g;
            }
            /* Fast:259-291: log(mean(expm1(x)) + 1); expm1 gate; |diff| > thr */
            int nt = 0;
            for (int f = 0; f < nf; ++f) {
                int g = feat[f];
                const double *row = X + (size_t)g * N;
                for (int k = 0; k < ni; ++k) tmp[k] = expm1(row[ci[k]]);
                m1[g] = log(orc_r_mean(tmp, ni) + 1);
                for (int k = 0; k < nj; ++k) tmp[k] = expm1(row[cj[k]]);
                m2[g] = log(orc_r_mean(tmp, nj) + 1);
                double d = m1[g] - m2[g];
                int pass_expr = (expm1(m1[g]) > 0) || (expm1(m2[g]) > 0);
                if (pass_expr && fabs(d) > prm->log_fc_thrs) feat[nt++] = g;
            }
            pair_tested[pidx] = nt;
            /* Fast:78-91 wilcox on tested features; x = cells.1 (cluster i) */
            for (int f = 0; f < nt; ++f) {
                int g = feat[f];
                const double *row = X + (size_t)g * N;
                for (int k = 0; k < ni; ++k) xi[k] = row[ci[k]];
                for (int k = 0; k < nj; ++k) yj[k] = row[cj[k]];
                if (prm->test == 1) { /* DiffTTest: t.test(x = cells.1, y = cells.2)$p.value */
                    int constant = 0;
                    pv[g] = orc_t_test_p(xi, ni, yj, nj, NULL, &constant);
                    if (constant) ((orc_fast_params *)prm)->status = ORC_ERR_RSTOP;
                    Wv[g] = Tv[g] = 0.0;
                } else {
                    int meth;
                    pv[g] = orc_wilcox_p_scratch(xi, ni, yj, nj, &Wv[g], &Tv[g], &meth, tmp,
                                                 tmp + ni + nj, scr);
                }
                keys[f].gene = g;
                keys[f].p = pv[g];
                keys[f].nlfc = -(m1[g] - m2[g]);
            }
            /* Fast:346-350 order(p, -avg_logFC) then BH with lazy n */
            qsort(keys, (size_t)nt, sizeof(orc_row_key), cmp_row_key);
            for (int f = 0; f < nt; ++f) tmp[f] = keys[f].p;
            orc_p_adjust_bh(tmp, nt, -1, qv);
            /* Fast:376-378: keep the pair only if > 1 rows; rows with q < thr */
            long row0 = nrows;
            int nde = 0;
            for (int f = 0; f < nt; ++f) {
                int g = keys[f].gene;
                row_gene[nrows] = g;
                row_p[nrows] = pv[g];
                row_q[nrows] = qv[f];
                row_lfc[nrows] = m1[g] - m2[g];
                row_pct1[nrows] = pct1[g];
                row_pct2[nrows] = pct2[g];
                row_W[nrows] = Wv[g];
                row_ties[nrows] = Tv[g];
                uint8_t fl = 0;
                if (nt > 1 && qv[f] < prm->q_val_thrs) { fl |= 1; ++nde; }
                row_flags[nrows] = fl;
                ++nrows;
            }
            /* Fast:386-392 top_n(N, |avg_logFC|): min_rank(desc(w)) <= N, ties kept */
            for (long r = row0; r < nrows; ++r) {
                if (!(row_flags[r] & 1)) continue;
                double w = fabs(row_lfc[r]);
                int above = 0;
                for (long s = row0; s < nrows; ++s)
                    if ((row_flags[s] & 1) && fabs(row_lfc[s]) > w) ++above;
                if (above + 1 <= prm->top_n) {
                    row_flags[r] |= 2;
                    if (!in_union[row_gene[r]]) {
                        in_union[row_gene[r]] = 1;
                        union_genes[nu++] = row_gene[r];
                    }
                }
            }
            (void)nde;
        }
    }
    *n_union = nu;
    free(cells); free(cstart); free(xi); free(tmp); free(scr); free(keys); free(pct1);
    free(Wv); free(feat); free(in_union);
    return nrows;
}

/* ---------------------------------------------------------------- Slow driver */
typedef struct {
    double q_val_thrs;          /* qValThrs */
    double fc_thrs;             /* fcThrs (compared as log(fcThrs)) */
    double mean_scaling_factor; /* meanScalingFactor */
} orc_slow_params;

typedef struct { double a; int g; } orc_abs_key;

static int cmp_abs_desc(const void *a, const void *b)
{
    const orc_abs_key *x = (const orc_abs_key *)a, *y = (const orc_abs_key *)b;
    if (x->a > y->a) return -1;
    if (x->a < y->a) return 1;
    return (x->g < y->g) ? -1 : (x->g > y->g);
}

/* Outputs per pair (pair-major, G each): p, q, logfc, W, ties, de (0/1);
 * union; *log_thr gets log(meanScalingFactor * mean(expm1(X))).
 * Returns ORC_ERR_RSTOP when the R code would stop() (NA in the DE vector). */
int orc_de_slow(const double *X, int G, int N, const int *code, int K, const orc_slow_params *prm,
                double *out_p, double *out_q, double *out_lfc, double *out_W, double *out_T,
                uint8_t *out_de, int *union_genes, int *n_union, double *log_thr)
{
    /* slow:36 meanExprsThrs = meanScalingFactor * mean(expm1(dataIn)) — R takes
     * the mean over the column-major G x N matrix; restated over all entries. */
    long double s = 0.0L;
    size_t tot = (size_t)G * (size_t)N;
    for (size_t e = 0; e < tot; ++e) s += expm1(X[e]);
    s /= (long double)tot;
    if (isfinite((double)s)) {
        long double t = 0.0L;
        for (size_t e = 0; e < tot; ++e) t += (expm1(X[e]) - s);
        s += t / (long double)tot;
    }
    double thr = prm->mean_scaling_factor * (double)s;
    double lthr = log(thr);
    *log_thr = lthr;
    double lfc_cut = log(prm->fc_thrs);

    int *cells = (int *)malloc(sizeof(int) * (size_t)N);
    int *cstart = (int *)calloc((size_t)K + 1, sizeof(int));
    for (int c = 0; c < N; ++c)
        if (code[c] >= 0) cstart[code[c] + 1]++;
    for (int a = 0; a < K; ++a) cstart[a + 1] += cstart[a];
    int *fill = (int *)malloc(sizeof(int) * (size_t)K);
    memcpy(fill, cstart, sizeof(int) * (size_t)K);
    for (int c = 0; c < N; ++c)
        if (code[c] >= 0) cells[fill[code[c]]++] = c;
    free(fill);
    int nmax = 0;
    for (int a = 0; a < K; ++a)
        if (cstart[a + 1] - cstart[a] > nmax) nmax = cstart[a + 1] - cstart[a];
    double *xi = (double *)malloc(sizeof(double) * (size_t)(2 * nmax + 1));
    double *yj = xi + nmax;
    double *tmp = (double *)malloc(sizeof(double) * (size_t)(4 * nmax + 2));
    orc_vi *scr = (orc_vi *)malloc(sizeof(orc_vi) * (size_t)(2 * nmax + 1));
    orc_abs_key *ak = (orc_abs_key *)malloc(sizeof(orc_abs_key) * (size_t)G);
    uint8_t *in_union = (uint8_t *)calloc((size_t)G, 1);
    int nu = 0, rc = ORC_OK;
    int pidx = 0;
    for (int i = 0; i < K - 1; ++i) {
        for (int j = i + 1; j < K; ++j, ++pidx) {
            const int *ci = cells + cstart[i], *cj = cells + cstart[j];
            int ni = cstart[i + 1] - cstart[i], nj = cstart[j + 1] - cstart[j];
            double *P = out_p + (size_t)pidx * G, *Q = out_q + (size_t)pidx * G;
            double *L = out_lfc + (size_t)pidx * G;
            double *Wp = out_W + (size_t)pidx * G, *Tp = out_T + (size_t)pidx * G;
            uint8_t *D = out_de + (size_t)pidx * G;
            uint8_t *gate = (uint8_t *)malloc((size_t)G);
            for (int g = 0; g < G; ++g) {
                const double *row = X + (size_t)g * N;
                for (int k = 0; k < ni; ++k) xi[k] = row[ci[k]];
                for (int k = 0; k < nj; ++k) yj[k] = row[cj[k]];
                int meth;
                P[g] = orc_wilcox_p_scratch(xi, ni, yj, nj, &Wp[g], &Tp[g], &meth, tmp, tmp + ni + nj, scr);
                double mi = orc_r_mean(xi, ni), mj = orc_r_mean(yj, nj);
                L[g] = mi - mj;
                gate[g] = (mi > lthr) || (mj > lthr);
            }
            orc_p_adjust_bh(P, G, G, Q);
            int nde = 0;
            for (int g = 0; g < G; ++g) {
                /* qval < thr & abs(logfc) > log(fcThrs) & gate, with R's NA logic */
                int b = (fabs(L[g]) > lfc_cut) && gate[g];
                if (isnan(Q[g])) {
                    if (b) { D[g] = 2; rc = ORC_ERR_RSTOP; } /* NA -> R stops at if(sum<=1) */
                    else D[g] = 0;
                } else {
                    D[g] = (Q[g] < prm->q_val_thrs) && b;
                }
                nde += (D[g] == 1);
            }
            free(gate);
            /* slow:214-225 sort(|logfc| of DE genes, decreasing) first 30, union */
            int nk = 0;
            for (int g = 0; g < G; ++g)
                if (D[g] == 1) { ak[nk].a = fabs(L[g]); ak[nk].g = g; ++nk; }
            qsort(ak, (size_t)nk, sizeof(orc_abs_key), cmp_abs_desc);
            int take = nk > 30 ? 30 : nk;
            for (int t = 0; t < take; ++t)
                if (!in_union[ak[t].g]) { in_union[ak[t].g] = 1; union_genes[nu++] = ak[t].g; }
            (void)nde;
        }
    }
    *n_union = nu;
    free(cells); free(cstart); free(xi); free(tmp); free(scr); free(ak); free(in_union);
    return rc;
}

/* nodg (Fast:440-443): number of genes with x > 0 per cell */
void orc_nodg(const double *X, int G, int N, int *nodg)
{
    for (int c = 0; c < N; ++c) nodg[c] = 0;
    for (int g = 0; g < G; ++g) {
        const double *row = X + (size_t)g * N;
        for (int c = 0; c < N; ++c) nodg[c] += (row[c] > 0);
    }
}
