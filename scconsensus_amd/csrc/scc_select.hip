// scc_select.hip — per-(pair, gene) test epilogue and per-pair selection.
//
//  k_wilcox_table   R's cwilcox counts (nmath/wilcox.c recursion, memo table
//                   w[i][j][k]) for the exact test, built once per context.
//  k_pair_test      per (pair, gene): Fast feature filters (Fast:229-291) or
//                   slow mean-diff + expression gate (slow:104-113), and the
//                   wilcox.test p-value (exact / normal rule) from exact 2U, T.
//  k_pair_select    per pair: R's row order order(p, -avg_logFC) (Fast:346),
//                   BH (Fast:347 lazy n / slow:116-121 n = G), q filter and
//                   the dim > 1 rule (Fast:376-378), top_n with ties
//                   (Fast:391) / first-30 of sort(|logfc|) (slow:214-222),
//                   and first-occurrence keys for the union.
//  k_union          unique(Gene) in row order (Fast:392) / union() (slow:224).
#include "scc_common.hpp"
#include "scc_kernels.hpp"
#include "scc_sort.hpp"

#define WT_DIM 50  // exact test when both clusters < 50 cells
#define SEL_T 1024

// -------------------------------------------------------- cwilcox table
__device__ inline double cw_lookup(int k, int m, int n, const double* W, const int* woff)
{
    for (;;) {
        const int u = m * n;
        if (k < 0 || k > u) return 0.0;
        const int c = u / 2;
        if (k > c) k = u - k;
        const int i = m < n ? m : n, j = m < n ? n : m;
        if (j == 0) return (k == 0) ? 1.0 : 0.0;
        if (k < j) {  // cwilcox(k, i, k)
            m = i;
            n = k;
            continue;
        }
        return W[woff[i * WT_DIM + j] + k];
    }
}

// single workgroup; level s = i + j ascending, every entry of a level (all
// its (i, j) rows at once, flattened over the threads) in parallel.  Only the
// sizes i <= j <= mmax are built: the exact test runs for a pair of clusters
// that both hold fewer than 50 cells (wilcox.test.default's rule), and
// cwilcox(k, m, n) reads only rows with i <= m, j <= n.
__global__ void __launch_bounds__(1024) k_wilcox_table(double* W, const int* woff, int mmax)
{
    for (int s = 2; s <= 2 * mmax; ++s) {
        const int ilo = max(1, s - mmax), ihi = s / 2;  // rows (i, s - i) with i <= j <= mmax
        int tot = 0;
        for (int i = ilo; i <= ihi; ++i) tot += (i * (s - i)) / 2 + 1;
        for (int f = threadIdx.x; f < tot; f += blockDim.x) {
            int i = ilo, k = f;
            for (;;) {
                const int len = (i * (s - i)) / 2 + 1;
                if (k < len) break;
                k -= len;
                ++i;
            }
            const int j = s - i;
            double* row = W + woff[i * WT_DIM + j];
            if (k < j)
                row[k] = -1.0;  // never read (reduced to cwilcox(k, i, k))
            else
                row[k] = cw_lookup(k - j, i - 1, j, W, woff) + cw_lookup(k, i, j - 1, W, woff);
        }
        __syncthreads();
    }
}

__device__ inline double r_choose(double n, double k)
{
    if (n - k < k) k = n - k;
    if (k < 0) return 0.0;
    if (k == 0) return 1.0;
    double r = n;
    for (int j = 2; j <= (int)k; ++j) r *= (n - j + 1) / j;
    return rint(r);
}

__device__ inline double r_pwilcox(double q, int m, int n, bool lower, const double* W, const int* woff)
{
    q = floor(q + 1e-7);
    const double mn = (double)m * n;
    if (q < 0.0) return lower ? 0.0 : 1.0;
    if (q >= mn) return lower ? 1.0 : 0.0;
    const double c = r_choose((double)m + n, (double)n);
    double p = 0.0;
    if (q <= mn / 2) {
        for (int i = 0; i <= (int)q; ++i) p += cw_lookup(i, m, n, W, woff) / c;
    } else {
        q = mn - q;
        for (int i = 0; i < (int)q; ++i) p += cw_lookup(i, m, n, W, woff) / c;
        lower = !lower;
    }
    return lower ? p : (0.5 - p + 0.5);
}

// stats:::wilcox.test.default two-sided, correct = TRUE, exact = NULL, from
// the exact statistic W = 2U/2 and tie term T = sum(NTIES^3 - NTIES).
__device__ inline double wilcox_p(i64 u2, i64 tie, int nx, int ny, const double* W, const int* woff, u8* exact_used)
{
    const double dnx = (double)nx, dny = (double)ny;
    const double stat = (double)u2 * 0.5;
    if (nx < 50 && ny < 50 && tie == 0) {
        *exact_used = 1;
        double p;
        if (stat > (dnx * dny / 2))
            p = r_pwilcox(stat - 1, nx, ny, false, W, woff);
        else
            p = r_pwilcox(stat, nx, ny, true, W, woff);
        return fmin(2 * p, 1.0);
    }
    *exact_used = 0;
    double z = stat - dnx * dny / 2;
    const double sigma =
        sqrt((dnx * dny / 12) * ((dnx + dny + 1) - (double)tie / ((dnx + dny) * (dnx + dny - 1))));
    const double corr = (z > 0) ? 0.5 : ((z < 0) ? -0.5 : 0.0);
    z = (z - corr) / sigma;
    return 2 * scc_pnorm_small_tail(z);
}

// -------------------------------------------------------- Welch t test
// stats::t.test(x, y)$p.value (R/t.test.R, two-sided, var.equal = FALSE) for
// the DiffTTest path (Fast:185-196): 2 * pt(-|t|, df) with R nmath/pt.c's
// regimes; pbeta by the continued fraction below with R's lbeta (R's own
// pbeta is TOMS 708; the oracle checks this with the power series and both are
// pinned to scipy).
__device__ inline double t_lgammacor(double x)
{
    const double r = 1.0 / (x * x);
    return (1.0 / 12 - r * (1.0 / 360 - r * (1.0 / 1260 - r * (1.0 / 1680 - r * (1.0 / 1188 -
            r * (691.0 / 360360 - r / 156)))))) / x;
}

__device__ inline double t_lbeta(double a, double b)
{
    const double p = fmin(a, b), q = fmax(a, b);
    const double ln_sqrt_2pi = 0.918938533204672741780329736406;
    if (p >= 10) {
        const double corr = t_lgammacor(p) + t_lgammacor(q) - t_lgammacor(p + q);
        return log(q) * -0.5 + ln_sqrt_2pi + corr + (p - 0.5) * log(p / (p + q)) + q * log1p(-p / (p + q));
    }
    if (q >= 10) {
        const double corr = t_lgammacor(q) - t_lgammacor(p + q);
        return lgamma(p) + corr + p - p * log(p + q) + (q - 0.5) * log1p(-p / (p + q));
    }
    return lgamma(p) + lgamma(q) - lgamma(p + q);
}

// The continued fraction of I_x(a, b) (DLMF 8.17.22):
//   I_x(a, b) = x^a (1-x)^b / (a B(a, b)) / K,  K = 1 + d_1 / (1 + d_2 / (1 + ...)),
//   d_{2m+1} = -(a+m)(a+b+m) x / ((a+2m)(a+2m+1)),  d_{2m} = m(b-m) x / ((a+2m-1)(a+2m)),
// evaluated forward by the modified Lentz method (Thompson & Barnett 1986):
// K_j = K_{j-1} C_j D_j, C_j = 1 + d_j / C_{j-1}, D_j = 1 / (1 + d_j D_{j-1})
// (C_0 = K_0 = 1, D_0 = 0), one coefficient per step, until C_j D_j = 1 to
// working precision.  Returns K.  (The oracle sums the power series instead.)
__device__ inline double ibeta_cf_den(double a, double b, double x)
{
    const double tiny = 1e-300;
    double K = 1.0, C = 1.0, D = 0.0;
    for (int j = 1; j <= 20000; ++j) {
        const int m = j >> 1;
        const double dj = (j & 1) ? -(a + m) * (a + b + m) * x / ((a + 2 * m) * (a + 2 * m + 1))
                                  : m * (b - m) * x / ((a + 2 * m - 1) * (a + 2 * m));
        D = 1.0 + dj * D;
        D = 1.0 / (fabs(D) < tiny ? tiny : D);
        C = 1.0 + dj / C;
        if (fabs(C) < tiny) C = tiny;
        const double cd = C * D;
        K *= cd;
        if (fabs(cd - 1.0) < 1e-16) break;
    }
    return K;
}

// I_x(a, b) (lower) or 1 - I_x(a, b), with y = 1 - x from the caller
__device__ inline double t_pbeta2(double x, double y, double a, double b, bool lower)
{
    if (x <= 0.0) return lower ? 0.0 : 1.0;
    if (y <= 0.0) return lower ? 1.0 : 0.0;
    const double lx = x > 0.5 ? log1p(-y) : log(x), ly = y > 0.5 ? log1p(-x) : log(y);
    const double lbt = a * lx + b * ly - t_lbeta(a, b);
    if (x < (a + 1.0) / (a + b + 2.0)) {
        const double v = exp(lbt) / (a * ibeta_cf_den(a, b, x));
        return lower ? v : 1.0 - v;
    }
    const double v = exp(lbt) / (b * ibeta_cf_den(b, a, y));
    return lower ? 1.0 - v : v;
}

// 2 * pt(-|t|, n): the upper tail beyond |t| twice (R nmath/pt.c)
__device__ inline double t_two_sided(double t, double n)
{
    const double x = -fabs(t);
    if (n > 4e5) {
        const double val = 1.0 / (4.0 * n);
        return 2 * scc_pnorm_small_tail(x * (1.0 - val) / sqrt(1.0 + x * x * 2.0 * val));
    }
    const double nx = 1 + (x / n) * x;
    double val;
    if (nx > 1e100)
        val = exp(-0.5 * n * (2 * log(fabs(x)) - log(n)) - t_lbeta(0.5 * n, 0.5) - log(0.5 * n));
    else
        val = (n > x * x) ? t_pbeta2(x * x / (n + x * x), n / (n + x * x), 0.5, n / 2.0, false)
                          : t_pbeta2(1.0 / nx, (x / n) * x / nx, n / 2.0, 0.5, true);
    return 2 * (val / 2.0);  // x <= 0: pt(x, lower) = val / 2
}

// -------------------------------------------------------- per (pair, gene)
__device__ inline u64 f_tie3(u64 c) { return c * c * c - c; }

// Feature filters before the rank stage: FAST keeps only the features
// ComputePairWiseDE tests (Fast:229-291), so the rank engine never sorts a
// gene no pair tests; SLOW tests every gene (slow:90) and records the gate.
// flags bit0 tested, bit1 expression gate (SLOW).
__global__ void __launch_bounds__(256) k_pair_filter(ScTestLaunch A)
{
    const int g = A.glo + blockIdx.x * blockDim.x + threadIdx.x;  // the run's gene shard only
    const int p = blockIdx.y;
    if (g >= A.ghi) return;
    int a, b;
    {
        a = 0;
        int rem = p;
        while (rem >= A.K - 1 - a) {
            rem -= A.K - 1 - a;
            ++a;
        }
        b = a + 1 + rem;
    }
    const size_t pg = (size_t)p * A.G + g;
    const int na = A.n_clu[a], nb = A.n_clu[b];
    u8 fl = 0;
    double lfc;
    if (A.mode == SCC_DE_FAST) {
        // Fast:230-239  round(100 * rowSums(x > 0) / n, 16): the round is the identity here
        const double pct1 = (100.0 * (double)A.cnt_pos[(size_t)a * A.G + g]) / (double)na;
        const double pct2 = (100.0 * (double)A.cnt_pos[(size_t)b * A.G + g]) / (double)nb;
        const double amax = pct1 > pct2 ? pct1 : pct2;
        // Fast:259-272 log(mean(expm1(x)) + 1)
        const double m1 = log(A.mean_e[(size_t)a * A.G + g] + 1.0);
        const double m2 = log(A.mean_e[(size_t)b * A.G + g] + 1.0);
        lfc = m1 - m2;
        const bool pass_pct = amax > A.min_pct;
        const bool pass_expr = (expm1(m1) > 0.0) || (expm1(m2) > 0.0);  // Fast:275
        const bool pass_fc = fabs(lfc) > A.lfc_thr;                       // Fast:285
        if (pass_pct && pass_expr && pass_fc) fl |= 1;
        A.out_pct1[pg] = pct1;
        A.out_pct2[pg] = pct2;
    } else {
        const double mi = A.mean_x[(size_t)a * A.G + g], mj = A.mean_x[(size_t)b * A.G + g];
        lfc = mi - mj;  // slow:105
        fl |= 1;
        if (mi > A.log_thr || mj > A.log_thr) fl |= 2;  // slow:110-113
    }
    A.out_lfc[pg] = lfc;
    A.out_flags[pg] = fl;
}

// After the rank stage: exact 2U and tie term (the implicit zero group in
// closed form) and the wilcox.test p-value of every tested (pair, gene).
// Untested cells (FAST, not requested) carry u2 = t = -1 and p = NaN.
__global__ void __launch_bounds__(256) k_pair_test(ScTestLaunch A)
{
    const int g = A.glo + blockIdx.x * blockDim.x + threadIdx.x;  // the run's gene shard only
    const int p = blockIdx.y;
    if (g >= A.ghi) return;
    int a, b;
    {
        a = 0;
        int rem = p;
        while (rem >= A.K - 1 - a) {
            rem -= A.K - 1 - a;
            ++a;
        }
        b = a + 1 + rem;
    }
    const size_t pg = (size_t)p * A.G + g;
    u8 fl = A.out_flags[pg];
    if (!(fl & 1) && !A.all_pairs) {
        A.out_p[pg] = __longlong_as_double(0x7ff8000000000000ll);
        A.out_u2[pg] = -1;
        A.out_t[pg] = -1;
        return;
    }
    const int na = A.n_clu[a], nb = A.n_clu[b];
    if (A.test == SCC_TEST_T) {  // DiffTTest: t.test(x = cluster a, y = cluster b)
        const double mx = A.mean_x[(size_t)a * A.G + g], my = A.mean_x[(size_t)b * A.G + g];
        const double vx = A.var_x[(size_t)a * A.G + g], vy = A.var_x[(size_t)b * A.G + g];
        const double sx = sqrt(vx / na), sy = sqrt(vy / nb);
        const double se = sqrt(sx * sx + sy * sy);
        const double df = pow(se, 4.0) / (pow(sx, 4.0) / (na - 1) + pow(sy, 4.0) / (nb - 1));
        double pv = __longlong_as_double(0x7ff8000000000000ll);
        if (se < 10 * 2.220446049250313e-16 * fmax(fabs(mx), fabs(my)))
            atomicOr(A.err, 8);  // R: stop("data are essentially constant")
        else
            pv = t_two_sided((mx - my) / se, df);
        A.out_p[pg] = pv;
        A.out_u2[pg] = 0;
        A.out_t[pg] = 0;
        return;
    }
    const u64 pa = A.cnt_pos[(size_t)a * A.G + g], ga = A.cnt_neg[(size_t)a * A.G + g];
    const u64 pb = A.cnt_pos[(size_t)b * A.G + g], gb = A.cnt_neg[(size_t)b * A.G + g];
    const u64 za = (u64)na - pa - ga, zb = (u64)nb - pb - gb;
    const u64 S = A.accS[pg] + za * gb + pa * zb;  // x > y, zeros included
    const u64 u2 = 2 * S + za * zb + A.accE[pg];
    const u64 t = A.accF[(size_t)a * A.G + g] + A.accF[(size_t)b * A.G + g] + f_tie3(za) + f_tie3(zb) +
                  3 * za * zb * (za + zb) + 3 * A.accX[pg];
    u8 ex = 0;
    const double pv = wilcox_p((i64)u2, (i64)t, na, nb, A.wtab, A.woff, &ex);
    A.out_p[pg] = pv;
    A.out_u2[pg] = (i64)u2;
    A.out_t[pg] = (i64)t;
    A.out_flags[pg] = (u8)(fl | (ex << 2));
}

// -------------------------------------------------------- per pair counts
__global__ void __launch_bounds__(256) k_count_tested(const u8* flags, int G, int* tested)
{
    const int p = blockIdx.x;
    int c = 0;
    for (int g = threadIdx.x; g < G; g += blockDim.x) c += flags[(size_t)p * G + g] & 1;
    c = (int)u32_wave_sum((u32)c);
    __shared__ int s[4];
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) tested[p] = s[0] + s[1] + s[2] + s[3];
}

// exclusive prefix over P pair counts (single block; P <= a few thousand)
__global__ void __launch_bounds__(1024) k_prefix_pairs(const int* cnt, int P, i64* off)
{
    __shared__ i64 s[1024];
    i64 carry = 0;
    for (int base = 0; base < P; base += 1024) {
        const int i = base + threadIdx.x;
        const i64 v = (i < P) ? cnt[i] : 0;
        s[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {
            const i64 t = ((int)threadIdx.x >= o) ? s[threadIdx.x - o] : 0;
            __syncthreads();
            s[threadIdx.x] += t;
            __syncthreads();
        }
        if (i < P) off[i] = carry + s[threadIdx.x] - v;
        const i64 blk = s[1023];
        __syncthreads();
        carry += blk;
    }
    if (threadIdx.x == 0) off[P] = carry;
}

// -------------------------------------------------------- per pair selection
// Record order = R's order(p, -avg_logFC) with NA last, ties by gene index
// (the original feature order: R's radix order is stable).
struct RowRec {
    u64 k1;  // orderable p (NaN -> max)
    u64 k2;  // orderable -logFC (FAST) / 0 (SLOW)
    u32 g;
    u32 pad;
    __device__ bool operator<(const RowRec& o) const
    {
        if (k1 != o.k1) return k1 < o.k1;
        if (k2 != o.k2) return k2 < o.k2;
        return g < o.g;
    }
};

struct KeyRec {  // (u64 key, u32 payload) ascending by key then payload
    u64 k;
    u32 g;
    u32 pad;
    __device__ bool operator<(const KeyRec& o) const { return k != o.k ? k < o.k : g < o.g; }
};

__device__ inline u64 p_key(double p) { return (p != p) ? ~0ull : scc_key_of(p + 0.0); }

struct SelectArgs {
    int K, G, P, mode, top_n, cap;
    int plo;                 // first pair of this launch (blockIdx.x = p - plo)
    double q_thr;
    double lfc_cut;          // SLOW: log(fcThrs)
    const double* p;         // [P][G]
    const double* lfc;
    const double* pct1;
    const double* pct2;
    const i64* u2;
    const i64* t;
    const u8* flags;
    const i64* row_off;      // [P+1] (FAST rows = tested genes per pair)
    RowRec* rec_scratch;     // [P][G] global scratch for large pairs
    KeyRec* key_scratch;     // [P][G]
    // FAST row outputs
    int* row_gene;
    double* row_p;
    double* row_q;
    double* row_lfc;
    double* row_pct1;
    double* row_pct2;
    i64* row_u2;
    i64* row_t;
    u8* row_flags;           // bit0 DE (q < thr and pair kept), bit1 top_n survivor
    // SLOW outputs [P][G]
    double* slow_q;
    u8* slow_de;             // 0/1, 2 = NA (R would stop())
    u64* first_occ;          // [G] (pair << 32 | rank), min-reduced
    int* err;
};

// block-wide exclusive scan helper (T threads, returns exclusive prefix, total)
template <int T>
__device__ int block_excl_scan(int v, int* s, int& total)
{
    // wave scans (shuffles) + one exchange of the wave totals: 2 barriers
    // (the Hillis-Steele form took 2 log2 T)
    constexpr int W = T / 64;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    int inc = v;
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
    }
    if (lane == 63) s[w] = inc;
    __syncthreads();
    int pre = 0, tot = 0;
#pragma unroll
    for (int q = 0; q < W; ++q) {
        const int x = s[q];
        pre += q < w ? x : 0;
        tot += x;
    }
    total = tot;
    __syncthreads();  // s is reused by the next call
    return pre + inc - v;
}

// Order-preserving compaction of [0, n): thread tid owns the contiguous
// indices [tid * per, tid * per + per), counts its hits, one block scan gives
// its output offset, then it emits them in order.  One barrier pair in all
// (a T-wide chunk per scan took n / T dependent load + scan rounds: 40 at
// G = 10,000).  Returns the number of hits.
template <int T, class Pred, class Emit>
__device__ int block_compact(int n, int* s, Pred pred, Emit emit)
{
    const int per = (n + T - 1) / T;
    const int i0 = min(n, (int)threadIdx.x * per), i1 = min(n, i0 + per);
    int c = 0;
    for (int i = i0; i < i1; ++i) c += pred(i) ? 1 : 0;
    int tot;
    int o = block_excl_scan<T>(c, s, tot);
    for (int i = i0; i < i1; ++i)
        if (pred(i)) emit(i, o++);
    return tot;
}

template <int T>
__global__ void __launch_bounds__(T) k_pair_select(SelectArgs A)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // dynamic LDS: RowRec[cap] | KeyRec[cap] | sred[T] | sc[T] | sthr
    const size_t tail = (size_t)A.cap * (sizeof(RowRec) + sizeof(KeyRec));
    double* sred = (double*)(smem + tail);
    int* sc = (int*)(smem + tail + sizeof(double) * T);
    u64& sthr = *(u64*)(smem + tail + (sizeof(double) + sizeof(int)) * T);
    const int p = A.plo + blockIdx.x, tid = threadIdx.x;
    const int G = A.G;
    const size_t pb = (size_t)p * G;
    // 1) compact tested genes (gene order) into records (HBM scratch when
    // they outgrow the LDS: counted first).  SLOW (every gene, no second key)
    // sorts 16-B (p key, gene) records instead of 24-B rows, with the whole
    // record LDS as their staging (4096 of them in the 2048-row budget): a
    // pair's 20k genes at config D took 10 passes over 24-B records through
    // HBM / L2, now 6 over 16-B ones.  Same order (p, then gene): same results.
    int m = 0;
    const bool fast = (A.mode == SCC_DE_FAST);
    RowRec* rec = (RowRec*)smem;
    KeyRec* krec = (KeyRec*)smem;
    int chk = 1;  // SLOW: KeyRec staging capacity (a power of two)
    while (2 * chk * sizeof(KeyRec) <= (size_t)A.cap * (sizeof(RowRec) + sizeof(KeyRec))) chk *= 2;
    const int per = (G + T - 1) / T;
    {
        const int g0 = min(G, tid * per), g1 = min(G, g0 + per);
        int c = 0;
        for (int g = g0; g < g1; ++g) c += A.flags[pb + g] & 1;
        int o = block_excl_scan<T>(c, sc, m);
        if (fast && m > A.cap) rec = A.rec_scratch + pb;
        if (!fast && m > chk) krec = A.key_scratch + pb;
        for (int g = g0; g < g1; ++g) {
            if (A.flags[pb + g] & 1) {
                if (fast) {
                    RowRec r;
                    r.k1 = p_key(A.p[pb + g]);
                    r.k2 = scc_key_of(-A.lfc[pb + g] + 0.0);
                    r.g = (u32)g;
                    r.pad = 0;
                    rec[o++] = r;
                } else {
                    KeyRec r;
                    r.k = p_key(A.p[pb + g]);
                    r.g = (u32)g;
                    r.pad = 0;
                    krec[o++] = r;
                }
            }
        }
    }
    __syncthreads();
    // 2) sort into R's row order
    if (fast) {
        if (m > A.cap) {
            AccAoS<RowRec> gacc{rec}, sacc{(RowRec*)smem};
            block_bitonic_staged(gacc, m, sacc, A.cap, tid, T);
        } else {
            AccAoS<RowRec> acc{rec};
            block_bitonic(acc, m, tid, T);
        }
    } else {
        if (m > chk) {
            AccAoS<KeyRec> gacc{krec}, sacc{(KeyRec*)smem};
            block_bitonic_staged(gacc, m, sacc, chk, tid, T);
        } else {
            AccAoS<KeyRec> acc{krec};
            block_bitonic(acc, m, tid, T);
        }
    }
    auto key_at = [&](int i) { return fast ? rec[i].k1 : krec[i].k; };
    auto gene_at = [&](int i) { return fast ? rec[i].g : krec[i].g; };
    // 3) BH: non-NaN prefix length, then suffix-min of (n / rank) * p
    int mnn = 0;
    {
        int c = 0;
        for (int i = tid; i < m; i += T) c += (key_at(i) != ~0ull);
        int tot;
        block_excl_scan<T>(c, sc, tot);
        mnn = tot;
    }
    const double nbh = fast ? (double)mnn : (double)G;
    // suffix min processed in chunks of T from the end; carry = min so far
    double carry = INFINITY;
    const int nchunks = (mnn + T - 1) / T;
    for (int cidx = nchunks - 1; cidx >= 0; --cidx) {
        const int i = cidx * T + tid;
        double v = INFINITY;
        double pv = 0.0;
        u32 gg = 0;
        if (i < mnn) {
            gg = gene_at(i);
            pv = A.p[pb + gg];
            v = (nbh / (double)(i + 1)) * pv;
        }
        // inclusive suffix min within the chunk: wave suffix mins by shuffles,
        // then the later waves' minima (fmin is exact: order-free)
        double wm = v;
        for (int o = 1; o < 64; o <<= 1) {
            const double y = __shfl_down(wm, o, 64);
            if ((tid & 63) + o < 64) wm = fmin(wm, y);
        }
        if ((tid & 63) == 0) sred[tid >> 6] = wm;
        __syncthreads();
        double suf = wm;
        for (int q = (tid >> 6) + 1; q < T / 64; ++q) suf = fmin(suf, sred[q]);
        const double sm = fmin(suf, carry);
        const double q = fmin(1.0, sm);
        if (i < mnn) {
            if (fast) {
                A.row_q[A.row_off[p] + i] = q;
            } else {
                A.slow_q[pb + gg] = q;
            }
        }
        double chunk_min = sred[0];
        for (int q = 1; q < T / 64; ++q) chunk_min = fmin(chunk_min, sred[q]);
        const double cmin = fmin(chunk_min, carry);
        __syncthreads();
        carry = cmin;
    }
    for (int i = mnn + tid; i < m; i += T) {
        if (fast) A.row_q[A.row_off[p] + i] = NAN;
        else A.slow_q[pb + gene_at(i)] = NAN;
    }
    __syncthreads();
    __threadfence_block();
    if (fast) {
        // 4) rows in R order, DE flag (q < thr, pair kept only when > 1 row)
        const i64 ro = A.row_off[p];
        int nde = 0;
        for (int i = tid; i < m; i += T) {
            const u32 g = rec[i].g;
            const double q = A.row_q[ro + i];
            const bool de = (m > 1) && (q < A.q_thr);
            A.row_gene[ro + i] = (int)g;
            A.row_p[ro + i] = A.p[pb + g];
            A.row_lfc[ro + i] = A.lfc[pb + g];
            A.row_pct1[ro + i] = A.pct1[pb + g];
            A.row_pct2[ro + i] = A.pct2[pb + g];
            A.row_u2[ro + i] = A.u2[pb + g];
            A.row_t[ro + i] = A.t[pb + g];
            A.row_flags[ro + i] = de ? 1 : 0;
            nde += de;
            if (m > 1 && q != q) atomicOr(A.err, 0x100);  // NA q in a kept pair: R builds an NA row (informational)
        }
        int d;
        block_excl_scan<T>(nde, sc, d);
        // 5) top_n: keep DE rows with min_rank(desc(|lfc|)) <= top_n  <=>  w >= v,
        //    v = top_n-th largest |lfc| among DE rows (all kept when d <= top_n)
        if (tid == 0) sthr = 0ull;
        __syncthreads();
        if (d > A.top_n) {
            // sort |lfc| keys of DE rows (ascending) in the record buffer's KeyRec view
            KeyRec* kr = (d <= A.cap) ? (KeyRec*)(smem + (size_t)A.cap * sizeof(RowRec))
                                      : (A.key_scratch + pb);
            block_compact<T>(
                m, sc, [&](int i) { return (A.row_flags[ro + i] & 1) != 0; },
                [&](int i, int o) {
                    KeyRec r;
                    r.k = scc_key_of(fabs(A.row_lfc[ro + i]));
                    r.g = (u32)i;
                    r.pad = 0;
                    kr[o] = r;
                });
            __syncthreads();
            if (d <= A.cap) {
                AccAoS<KeyRec> acc{kr};
                block_bitonic(acc, d, tid, T);
            } else {
                AccAoS<KeyRec> gacc{kr}, sacc{(KeyRec*)smem};
                block_bitonic_staged(gacc, d, sacc, A.cap, tid, T);
            }
            if (tid == 0) sthr = kr[d - A.top_n].k;
            __syncthreads();
        }
        const u64 thr = sthr;
        for (int i = tid; i < m; i += T) {
            if (A.row_flags[ro + i] & 1) {
                const u64 w = scc_key_of(fabs(A.row_lfc[ro + i]));
                if (w >= thr) {
                    A.row_flags[ro + i] |= 2;
                    atomicMin((unsigned long long*)&A.first_occ[A.row_gene[ro + i]],
                              (unsigned long long)(((u64)p << 32) | (u64)i));
                }
            }
        }
    } else {
        // SLOW: DE = q < thr & |logfc| > log(fcThrs) & gate (R NA logic), then
        // first 30 of sort(|logfc|, decreasing) (stable: gene order on ties)
        int nde = 0;
        for (int g = tid; g < G; g += T) {
            const double q = A.slow_q[pb + g];
            const bool bterm = (fabs(A.lfc[pb + g]) > A.lfc_cut) && (A.flags[pb + g] & 2);
            u8 de;
            if (q != q) {
                de = bterm ? 2 : 0;
                if (bterm) atomicOr(A.err, 0x200);  // informational
            } else {
                de = (q < A.q_thr) && bterm;
            }
            A.slow_de[pb + g] = de;
            nde += (de == 1);
        }
        int d;
        block_excl_scan<T>(nde, sc, d);
        __syncthreads();
        KeyRec* kr = (d <= A.cap) ? (KeyRec*)(smem + (size_t)A.cap * sizeof(RowRec)) : (A.key_scratch + pb);
        block_compact<T>(
            G, sc, [&](int g) { return A.slow_de[pb + g] == 1; },
            [&](int g, int o) {
                KeyRec r;
                // descending |logfc| -> ascending key of -|logfc|; ties by gene (stable)
                r.k = scc_key_of(-fabs(A.lfc[pb + g]));
                r.g = (u32)g;
                r.pad = 0;
                kr[o] = r;
            });
        __syncthreads();
        if (d <= A.cap) {
            AccAoS<KeyRec> acc{kr};
            block_bitonic(acc, d, tid, T);
        } else {
            AccAoS<KeyRec> gacc{kr}, sacc{(KeyRec*)smem};
            block_bitonic_staged(gacc, d, sacc, A.cap, tid, T);
        }
        const int take = d < 30 ? d : 30;
        for (int i = tid; i < take; i += T)
            atomicMin((unsigned long long*)&A.first_occ[kr[i].g], (unsigned long long)(((u64)p << 32) | (u64)i));
    }
}

// -------------------------------------------------------- union
template <int T>
__global__ void __launch_bounds__(T) k_union(const u64* first_occ, int G, KeyRec* scratch, int cap, int* out,
                                             int* n_out)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    int* sc = (int*)(smem + (size_t)cap * sizeof(KeyRec));
    const int tid = threadIdx.x;
    // the genes in some pair's selection, in gene order (one compaction scan)
    const int per = (G + T - 1) / T;
    const int g0 = min(G, tid * per), g1 = min(G, g0 + per);
    int c = 0;
    for (int g = g0; g < g1; ++g) c += (first_occ[g] != ~0ull);
    int nu;
    int o = block_excl_scan<T>(c, sc, nu);
    KeyRec* kr = (nu <= cap) ? (KeyRec*)smem : scratch;
    for (int g = g0; g < g1; ++g) {
        const u64 f = first_occ[g];
        if (f != ~0ull) {
            KeyRec r;
            r.k = f;
            r.g = (u32)g;
            r.pad = 0;
            kr[o++] = r;
        }
    }
    __syncthreads();
    if (nu <= cap) {
        AccAoS<KeyRec> acc{kr};
        block_bitonic(acc, nu, tid, T);
    } else {
        AccAoS<KeyRec> gacc{kr}, sacc{(KeyRec*)smem};
        block_bitonic_staged(gacc, nu, sacc, cap, tid, T);
    }
    for (int i = tid; i < nu; i += T) out[i] = (int)kr[i].g;
    if (tid == 0) *n_out = nu;
}

// -------------------------------------------------------- launchers
extern "C" hipError_t scc_launch_wilcox_table(double* W, const int* woff, int mmax, hipStream_t st)
{
    if (mmax < 1) return hipSuccess;
    hipLaunchKernelGGL(k_wilcox_table, dim3(1), dim3(1024), 0, st, W, woff, min(mmax, WT_DIM - 1));
    return hipGetLastError();
}

extern "C" int scc_wilcox_table_layout(int* woff /* WT_DIM*WT_DIM */)
{
    int o = 0;
    for (int i = 0; i < WT_DIM; ++i)
        for (int j = 0; j < WT_DIM; ++j) {
            if (i >= 1 && j >= i) {
                woff[i * WT_DIM + j] = o;
                o += (i * j) / 2 + 1;
            } else {
                woff[i * WT_DIM + j] = 0;
            }
        }
    return o;
}

extern "C" hipError_t scc_launch_pair_filter(const ScTestLaunch* L, hipStream_t st)
{
    if (L->ghi <= L->glo) return hipSuccess;
    hipLaunchKernelGGL(k_pair_filter, dim3((L->ghi - L->glo + 255) / 256, L->P), dim3(256), 0, st, *L);
    return hipGetLastError();
}

extern "C" hipError_t scc_launch_pair_test(const ScTestLaunch* L, hipStream_t st)
{
    if (L->ghi <= L->glo) return hipSuccess;
    hipLaunchKernelGGL(k_pair_test, dim3((L->ghi - L->glo + 255) / 256, L->P), dim3(256), 0, st, *L);
    return hipGetLastError();
}

extern "C" hipError_t scc_launch_count_tested(const u8* flags, int G, int P, int* tested, i64* row_off,
                                              hipStream_t st)
{
    hipLaunchKernelGGL(k_count_tested, dim3(P), dim3(256), 0, st, flags, G, tested);
    hipLaunchKernelGGL(k_prefix_pairs, dim3(1), dim3(1024), 0, st, tested, P, row_off);
    return hipGetLastError();
}

extern "C" size_t scc_select_lds_bytes(int cap)
{
    return (size_t)cap * (sizeof(RowRec) + sizeof(KeyRec)) + (sizeof(double) + sizeof(int)) * SEL_T + 16;
}
extern "C" size_t scc_select_rec_bytes(void) { return sizeof(RowRec); }
extern "C" size_t scc_select_key_bytes(void) { return sizeof(KeyRec); }

extern "C" hipError_t scc_launch_pair_select(const ScSelectLaunch* L, hipStream_t st)
{
    SelectArgs A;
    A.K = L->K;
    A.G = L->G;
    A.P = L->P;
    A.plo = L->plo;
    A.mode = L->mode;
    A.top_n = L->top_n;
    A.cap = L->cap;
    A.q_thr = L->q_thr;
    A.lfc_cut = L->lfc_cut;
    A.p = L->p;
    A.lfc = L->lfc;
    A.pct1 = L->pct1;
    A.pct2 = L->pct2;
    A.u2 = L->u2;
    A.t = L->t;
    A.flags = L->flags;
    A.row_off = L->row_off;
    A.rec_scratch = (RowRec*)L->rec_scratch;
    A.key_scratch = (KeyRec*)L->key_scratch;
    A.row_gene = L->row_gene;
    A.row_p = L->row_p;
    A.row_q = L->row_q;
    A.row_lfc = L->row_lfc;
    A.row_pct1 = L->row_pct1;
    A.row_pct2 = L->row_pct2;
    A.row_u2 = L->row_u2;
    A.row_t = L->row_t;
    A.row_flags = L->row_flags;
    A.slow_q = L->slow_q;
    A.slow_de = L->slow_de;
    A.first_occ = L->first_occ;
    A.err = L->err;
    const size_t lds = scc_select_lds_bytes(L->cap);
    scc_set_lds((const void*)k_pair_select<SEL_T>, (int)lds);
    if (L->phi <= L->plo) return hipSuccess;
    hipLaunchKernelGGL(k_pair_select<SEL_T>, dim3(L->phi - L->plo), dim3(SEL_T), lds, st, A);
    return hipGetLastError();
}

extern "C" hipError_t scc_launch_union(const u64* first_occ, int G, void* scratch, int cap, int* out, int* n_out,
                                       hipStream_t st)
{
    // one workgroup over all G genes: 1024 threads (a quarter of the chunk rounds of 256)
    constexpr int UT = 1024;
    const size_t lds = (size_t)cap * sizeof(KeyRec) + sizeof(int) * UT;
    scc_set_lds((const void*)k_union<UT>, (int)lds);
    hipLaunchKernelGGL(k_union<UT>, dim3(1), dim3(UT), lds, st, first_occ, G, (KeyRec*)scratch, cap, out, n_out);
    return hipGetLastError();
}

// The DE result header in one launch, written straight into the context's
// pinned host staging buffer (host-mapped): [0] |U|, [1] error bits, [2..3]
// FAST row count (i64), [4, 4 + P) tested rows per pair, then the |U| union
// genes.  Replaces five small device-to-host copies (~15 us of copy-engine
// latency each) with one kernel and the final synchronisation.
__global__ void __launch_bounds__(256) k_stage_pack(const int* __restrict__ nu, const int* __restrict__ err,
                                                    const long long* __restrict__ nrows,
                                                    const int* __restrict__ tested, int P, const int* __restrict__ uni,
                                                    int G, int* __restrict__ out)
{
    const int n = min(max(*nu, 0), G);
    const int tot = 4 + P + n;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += gridDim.x * blockDim.x) {
        int v;
        if (i == 0) v = *nu;
        else if (i == 1) v = *err;
        else if (i < 4) v = nrows ? (int)(((unsigned long long)*nrows) >> (32 * (i - 2))) : 0;
        else if (i < 4 + P) v = tested ? tested[i - 4] : 0;
        else v = uni[i - 4 - P];
        out[i] = v;
    }
}

extern "C" hipError_t scc_launch_stage_pack(const int* nu, const int* err, const long long* nrows, const int* tested,
                                            int P, const int* uni, int G, int* out_dev, hipStream_t st)
{
    hipLaunchKernelGGL(k_stage_pack, dim3(std::min(64, (4 + P + G + 255) / 256)), dim3(256), 0, st, nu, err, nrows,
                       tested, P, uni, G, out_dev);
    return hipGetLastError();
}

// one u32 flag ORed into mapped pinned host memory (a kernel instead of a
// small device-to-host copy: ~5 instead of ~30 us; sticky until the host reads
// and clears it)
__global__ void k_flag_copy(const unsigned int* __restrict__ src, unsigned int* __restrict__ dst) { *dst |= *src; }

extern "C" hipError_t scc_launch_flag_copy(const unsigned int* src, unsigned int* dst_dev, hipStream_t st)
{
    hipLaunchKernelGGL(k_flag_copy, dim3(1), dim3(1), 0, st, src, dst_dev);
    return hipGetLastError();
}
