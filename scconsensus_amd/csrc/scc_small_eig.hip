// scc_small_eig.hip — small dense kernels of the filtered subspace iteration
// (scc_subspace.hip), each ONE launch on one CU:
//
//   k_small_syev   top-k eigenpairs of a symmetric n x n matrix, n <= 64: the
//                  Rayleigh-Ritz matrix H = V^T C V of the 64-column basis
//                  (reference: irlba::prcomp_irlba, R/reclusterDEConsensusFast.R:398).
//                  Householder tridiagonalisation in LDS (LAPACK dsytd2 order),
//                  multisection on Sturm counts, inverse iteration (dgttrf /
//                  dgttrs order, one lane per eigenpair), Gram-Schmidt inside
//                  eigenvalue clusters (dstein's 1e-3 ||T|| rule), Rayleigh
//                  quotient, back-transformation by the reflectors.  The hand-off
//                  solver of scc_eigen.hip spends ~3 us per column on cross-CU
//                  hand-offs; here every column costs three workgroup barriers.
//   k_fsi_cholinv  T = R^{-1} for G + s I = R^T R (the CholQR step of a 64-column
//                  block): one wave, lane = row, the pivot column broadcast
//                  through LDS, no cross-lane register traffic but one readlane
//                  per step.
#include "scc_common.hpp"
#include "scc.h"
#include <mutex>

#define SE_N 64
#define SE_T 256
#define SE_MAXK 16

static constexpr double kSeEps = 2.220446049250313e-16;

__device__ inline double se_wave_sum(double v)
{
    v += scc_xor_lane_f64<32>(v);
    v += scc_xor_lane_f64<16>(v);
    v += scc_xor_lane_f64<8>(v);
    v += scc_xor_lane_f64<4>(v);
    v += scc_xor_lane_f64<2>(v);
    return v + scc_xor_lane_f64<1>(v);
}
__device__ inline double se_wave_min(double v)
{
    v = fmin(v, scc_xor_lane_f64<32>(v));
    v = fmin(v, scc_xor_lane_f64<16>(v));
    v = fmin(v, scc_xor_lane_f64<8>(v));
    v = fmin(v, scc_xor_lane_f64<4>(v));
    v = fmin(v, scc_xor_lane_f64<2>(v));
    return fmin(v, scc_xor_lane_f64<1>(v));
}
__device__ inline double se_wave_max(double v)
{
    v = fmax(v, scc_xor_lane_f64<32>(v));
    v = fmax(v, scc_xor_lane_f64<16>(v));
    v = fmax(v, scc_xor_lane_f64<8>(v));
    v = fmax(v, scc_xor_lane_f64<4>(v));
    v = fmax(v, scc_xor_lane_f64<2>(v));
    return fmax(v, scc_xor_lane_f64<1>(v));
}
// uniform value of lane l (compile-time or wave-uniform) of a lane-varying double
__device__ __forceinline__ double se_readlane(double x, int l)
{
    const u64 b = (u64)__double_as_longlong(x);
    const u32 lo = (u32)__builtin_amdgcn_readlane((int)(u32)b, l);
    const u32 hi = (u32)__builtin_amdgcn_readlane((int)(u32)(b >> 32), l);
    return __longlong_as_double((long long)(((u64)hi << 32) | lo));
}

// number of eigenvalues of T (d, e^2) below x: signs of the leading principal
// minors p_i = (d_i - x) p_{i-1} - e_{i-1}^2 p_{i-2} (one FMA on the dependent
// chain, no division), a zero pivot counted negative (LAPACK dstebz's
// -pivmin), the pair rescaled by a power of two every 8 steps
__device__ inline int se_count(const double* dg, const double* e2, int n, double x, double pivmin)
{
    double pp = 1.0, pc = dg[0] - x;
    if (pc == 0.0) pc = -pivmin;
    int neg = pc < 0.0;
    for (int i = 1; i < n; ++i) {
        double pn = fma(dg[i] - x, pc, -e2[i - 1] * pp);
        pn = (pn == 0.0) ? -pivmin * pc : pn;
        neg += (pn < 0.0) != (pc < 0.0);
        pp = pc;
        pc = pn;
        if ((i & 7) == 0) {
            const int ex = ilogb(pc);
            if (ex > 256 || ex < -256) {
                pc = ldexp(pc, -ex);
                pp = ldexp(pp, -ex);
            }
        }
    }
    return neg;
}

// dynamic LDS of k_small_syev (doubles)
#define SE_LDS_A 0                              // [64][65] the matrix, updated in place
#define SE_LDS_V (SE_LDS_A + SE_N * (SE_N + 1)) // [64][64] reflector i in row i
#define SE_LUS (5 * SE_N + 2)                  // per-eigenpair LU stride (padded: lanes on distinct banks)
#define SE_YS (SE_N + 2)                       // tridiagonal eigenvector stride (padded likewise)
#define SE_LDS_LU (SE_LDS_V + SE_N * SE_N)      // [16][SE_LUS] LU factors per eigenpair
#define SE_LDS_Y (SE_LDS_LU + SE_MAXK * SE_LUS)  // [16][SE_YS] tridiagonal eigenvectors
#define SE_LDS_TOTAL (SE_LDS_Y + SE_MAXK * SE_YS)

extern "C" size_t scc_small_syev_lds_bytes() { return sizeof(double) * SE_LDS_TOTAL; }

// H: n x n (ldh), symmetrised on load; k <= 16 wanted.  Y[r * 16 + q]: the
// q-th largest eigenvector (q < k; columns k..15 zero), theta[q] its Rayleigh
// quotient.  flag |= 16 when a value is not finite or a cluster's vectors are
// dependent.
__global__ void __launch_bounds__(SE_T) k_small_syev(const double* __restrict__ H, int n, int ldh, int k,
                                                    double* __restrict__ Y, double* __restrict__ theta,
                                                    u32* __restrict__ flag)
{
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double(*A)[SE_N + 1] = (double(*)[SE_N + 1])(sm + SE_LDS_A);
    double(*Vr)[SE_N] = (double(*)[SE_N])(sm + SE_LDS_V);
    double* LU = sm + SE_LDS_LU;
    double(*Yt)[SE_YS] = (double(*)[SE_YS])(sm + SE_LDS_Y);
    __shared__ double dg[SE_N], eo[SE_N], e2[SE_N], ta[SE_N], pv[SE_N], vc[SE_N], th[SE_MAXK];
    __shared__ double blo[SE_MAXK], bhi[SE_MAXK], gsc[4];
    __shared__ int cnt[SE_T];
    __shared__ int s_bad;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (tid == 0) s_bad = 0;
    for (int e = tid; e < n * n; e += SE_T) {
        const int i = e / n, j = e - i * n;
        A[i][j] = 0.5 * (H[(size_t)i * ldh + j] + H[(size_t)j * ldh + i]);
    }
    __syncthreads();
    // ---- tridiagonalisation: reflector of column i from wave 0, p = tau A22 v
    // (4 threads per row), w = p - (tau/2)(p.v) v, A22 -= v w^T + w v^T
    for (int i = 0; i + 2 < n; ++i) {
        if (wv == 0) {
            const int r = i + 1 + lane;
            const double x = (r < n) ? A[min(r, n - 1)][i] : 0.0;
            const double alpha = A[i + 1][i];
            const double s = se_wave_sum((r >= i + 2 && r < n) ? x * x : 0.0);
            double beta = alpha, t = 0.0, scal = 0.0;
            if (s > 0.0) {
                beta = -copysign(sqrt(alpha * alpha + s), alpha);
                t = (beta - alpha) / beta;
                scal = 1.0 / (alpha - beta);
            }
            if (r < n) {
                const double v = (r == i + 1) ? 1.0 : x * scal;
                vc[r] = v;
                Vr[i][r] = v;
            }
            if (lane == 0) {
                dg[i] = A[i][i];
                eo[i] = beta;
                ta[i] = t;
            }
        }
        __syncthreads();
        const double t = ta[i];
        const int r = i + 1 + (tid >> 2), q = tid & 3;
        double part = 0.0;
        if (r < n)
            for (int c = i + 1 + q; c < n; c += 4) part = fma(A[r][c], vc[c], part);
        part += scc_xor_lane_f64<1>(part);
        part += scc_xor_lane_f64<2>(part);
        if (q == 0 && r < n) pv[r] = t * part;
        __syncthreads();
        const int rr = i + 1 + lane;
        const double K = -0.5 * t * se_wave_sum(rr < n ? pv[min(rr, n - 1)] * vc[min(rr, n - 1)] : 0.0);
        if (r < n) {
            const double vr = vc[r], wr = fma(K, vr, pv[r]);
            for (int c = i + 1 + q; c < n; c += 4) {
                const double vcc = vc[c], wc = fma(K, vcc, pv[c]);
                A[r][c] = fma(-vr, wc, fma(-wr, vcc, A[r][c]));
            }
        }
        __syncthreads();
    }
    if (tid == 0) {
        if (n >= 2) {
            dg[n - 2] = A[n - 2][n - 2];
            eo[n - 2] = A[n - 1][n - 2];
            ta[n - 2] = 0.0;
        }
        dg[n - 1] = A[n - 1][n - 1];
        eo[n - 1] = 0.0;
        ta[n - 1] = 0.0;
    }
    __syncthreads();
    // ---- Gershgorin bounds, pivmin (LAPACK dstebz)
    if (wv == 0) {
        const int i = lane;
        double gl = INFINITY, gu = -INFINITY, em = 0.0;
        if (i < n) {
            const double ei = eo[i];
            e2[i] = ei * ei;
            const double rad = (i > 0 ? fabs(eo[i - 1]) : 0.0) + (i < n - 1 ? fabs(ei) : 0.0);
            gl = dg[i] - rad;
            gu = dg[i] + rad;
            if (i < n - 1) em = ei * ei;
        }
        gl = se_wave_min(gl);
        gu = se_wave_max(gu);
        em = se_wave_max(em);
        if (lane == 0) {
            gsc[0] = gl;
            gsc[1] = gu;
            gsc[2] = em;
        }
    }
    __syncthreads();
    const double tnorm = fmax(fabs(gsc[0]), fabs(gsc[1]));
    const double pivmin = fmax(2.2250738585072014e-308 * fmax(1.0, gsc[2]), 1e-300);
    const double glo = gsc[0] - 2.0 * tnorm * kSeEps * n - 1e-300;
    const double ghi = gsc[1] + 2.0 * tnorm * kSeEps * n + 1e-300;
    // ---- eigenvalues: one shared round of 256 points, then 16 points per
    // wanted eigenvalue per round until the bracket is below
    // max(1e-12 |lambda|, 2 eps ||T||) (inverse iteration's need; the value
    // returned is the Rayleigh quotient)
    {
        const double x = glo + (ghi - glo) * (double)(tid + 1) / (double)(SE_T + 1);
        cnt[tid] = se_count(dg, e2, n, x, pivmin);
    }
    __syncthreads();
    const int qg = tid >> 4, jg = tid & 15;
    const int idx = n - 1 - qg;  // ascending index of the qg-th largest
    const bool want = qg < k;
    if (want && jg == 0) {
        // first point with cnt > idx (cnt is nondecreasing in the point)
        int lo = 0, hi = SE_T;
        while (lo < hi) {
            const int m = (lo + hi) >> 1;
            if (cnt[m] > idx)
                hi = m;
            else
                lo = m + 1;
        }
        blo[qg] = (lo == 0) ? glo : glo + (ghi - glo) * (double)lo / (double)(SE_T + 1);
        bhi[qg] = (lo == SE_T) ? ghi : glo + (ghi - glo) * (double)(lo + 1) / (double)(SE_T + 1);
    }
    __syncthreads();
    bool done = !want;
    for (int it = 0; it < 24; ++it) {
        if (!__syncthreads_or(!done)) break;
        double lo = want ? blo[qg] : 0.0, hi = want ? bhi[qg] : 0.0;
        if (!done) {
            const double x = lo + (hi - lo) * (double)(jg + 1) / 17.0;
            const int c = se_count(dg, e2, n, x, pivmin);
            const u64 m = __ballot(c > idx);
            const u32 bits = (u32)(m >> (16 * ((tid >> 4) & 3))) & 0xffffu;
            const int js = bits ? __builtin_ctz(bits) : 16;
            const double nlo = (js == 0) ? lo : lo + (hi - lo) * (double)js / 17.0;
            const double nhi = (js == 16) ? hi : lo + (hi - lo) * (double)(js + 1) / 17.0;
            if (jg == 0) {
                blo[qg] = nlo;
                bhi[qg] = nhi;
            }
            if (nhi - nlo <= fmax(1e-12 * fmax(fabs(nlo), fabs(nhi)), 2.0 * kSeEps * tnorm) + pivmin ||
                (nlo == lo && nhi == hi))
                done = true;
        }
    }
    __syncthreads();
    // ---- inverse iteration: eigenpair q on lane q of wave 0 (LU with partial
    // pivoting of T - lambda I, two solves from a pseudo-random start)
    if (wv == 0 && lane < k) {
        const int q = lane;
        const double lam = 0.5 * (blo[q] + bhi[q]);
        double* fdr = LU + (size_t)q * SE_LUS;  // 1 / U diagonal
        double* fu = fdr + SE_N;
        double* fu2 = fu + SE_N;
        double* fl = fu2 + SE_N;
        double* fp = fl + SE_N;
        double* y = Yt[q];
        const double tiny = kSeEps * tnorm + 1e-300;
        double dcur = dg[0] - lam, ucur = (n > 1) ? eo[0] : 0.0;
        for (int i = 0; i < n - 1; ++i) {
            const double li = eo[i], dn = dg[i + 1] - lam, un = (i < n - 2) ? eo[i + 1] : 0.0;
            const bool piv = fabs(dcur) < fabs(li);
            const double dc = (!piv && dcur == 0.0) ? tiny : dcur;
            const double den = piv ? li : dc;
            // (piv ? dc : li) / den through a refined hardware reciprocal (a few ulp)
            const double r0 = __builtin_amdgcn_rcp(den);
            const double rd = fma(fma(-den, r0, 1.0), r0, r0);
            const double f = (piv ? dc : li) * rd;
            fl[i] = f;
            fdr[i] = rd;
            const double ua = piv ? dn : ucur, ub = piv ? ucur : dn;
            fu[i] = ua;
            fu2[i] = piv ? un : 0.0;
            fp[i] = piv ? 1.0 : 0.0;
            dcur = fma(-f, ua, ub);
            ucur = piv ? -f * un : un;
        }
        if (dcur == 0.0) dcur = tiny;
        fdr[n - 1] = 1.0 / dcur;
        fu[n - 1] = 0.0;
        fu2[n - 1] = 0.0;
        for (int i = 0; i < n; ++i) {
            unsigned h = (unsigned)i * 2654435761u ^ ((unsigned)q * 40503u + 12345u);
            h ^= h >> 13;
            h *= 0x5bd1e995u;
            h ^= h >> 15;
            y[i] = 0.5 + (double)(h & 0xffff) / 65536.0;
        }
        for (int iter = 0; iter < 2; ++iter) {
            double bi = y[0];  // y <- L^-1 P y (in place)
            for (int i = 0; i < n - 1; ++i) {
                const double bn = y[i + 1];
                const bool piv = fp[i] != 0.0;
                const double xa = piv ? bn : bi, xb = piv ? bi : bn;
                y[i] = xa;
                bi = fma(-fl[i], xa, xb);
            }
            y[n - 1] = bi;
            double z1 = 0.0, z2 = 0.0;  // y <- U^-1 y from the bottom
            for (int i = n - 1; i >= 0; --i) {
                const double z0 = fma(-fu[i], z2, fma(-fu2[i], z1, y[i])) * fdr[i];
                y[i] = z0;
                z1 = z2;
                z2 = z0;
            }
            double mx = 0.0;
            for (int i = 0; i < n; ++i) mx = fmax(mx, fabs(y[i]));
            const double sc = (mx > 0.0 && mx < INFINITY) ? 1.0 / mx : 1.0;
            double s = 0.0;
            for (int i = 0; i < n; ++i) {
                const double v = y[i] * sc;
                s = fma(v, v, s);
            }
            const double inv = sc / sqrt(s);
            for (int i = 0; i < n; ++i) y[i] *= inv;
        }
    }
    __syncthreads();
    // ---- Gram-Schmidt inside clusters (|lambda_p - lambda_q| <= 1e-3 ||T||,
    // LAPACK dstein), in order, then the Rayleigh quotients y^T T y (wave 0,
    // lane = entry)
    if (wv == 0) {
        const int i = lane;
        const int ic = min(i, n - 1);
        for (int q = 0; q < k; ++q) {
            double yq = (i < n) ? Yt[q][ic] : 0.0;
            const double lq = 0.5 * (blo[q] + bhi[q]);
            bool touched = false;
            for (int p = 0; p < q; ++p) {
                const double lp = 0.5 * (blo[p] + bhi[p]);
                if (fabs(lp - lq) > 1e-3 * tnorm) continue;
                const double yp = (i < n) ? Yt[p][ic] : 0.0;
                const double d = se_wave_sum(yp * yq);
                yq = fma(-d, yp, yq);
                touched = true;
            }
            if (touched) {
                const double s = se_wave_sum(yq * yq);
                if (!(s > 1e-6)) s_bad = 1;  // the cluster's vectors were (nearly) dependent
                yq *= 1.0 / sqrt(s);
            }
            if (i < n) Yt[q][i] = yq;
            const double tv = (i < n) ? yq * dg[ic] + (i + 1 < n ? eo[ic] * Yt[q][min(i + 1, n - 1)] : 0.0) +
                                            (i > 0 ? eo[max(i - 1, 0)] * Yt[q][max(i - 1, 0)] : 0.0)
                                      : 0.0;
            const double rq = se_wave_sum(yq * tv);  // (the neighbours' entries of q were stored above)
            if (lane == 0) th[q] = rq;
        }
    }
    __syncthreads();
    // ---- back-transformation y <- H_0 ... H_{n-3} y: group qg (16 lanes) holds
    // eigenvector qg, entries r = jg + 16 u in registers
    double yv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int r = jg + 16 * u;
        yv[u] = (want && r < n) ? Yt[qg][min(r, n - 1)] : 0.0;
    }
    for (int i = n - 3; i >= 0; --i) {
        double d = 0.0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int r = jg + 16 * u;
            const double v = Vr[i][min(r, n - 1)];
            d = fma((r > i && r < n) ? v : 0.0, yv[u], d);
        }
        d += scc_xor_lane_f64<1>(d);
        d += scc_xor_lane_f64<2>(d);
        d += scc_xor_lane_f64<4>(d);
        d += scc_xor_lane_f64<8>(d);
        const double td = ta[i] * d;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int r = jg + 16 * u;
            const double v = Vr[i][min(r, n - 1)];
            yv[u] = fma(-td, (r > i && r < n) ? v : 0.0, yv[u]);
        }
    }
    bool bad = false;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int r = jg + 16 * u;
        if (r < n) Y[(size_t)r * 16 + qg] = want ? yv[u] : 0.0;
        bad |= !(fabs(yv[u]) < INFINITY);
    }
    if (want && jg == 0) {
        theta[qg] = th[qg];
        bad |= !(fabs(th[qg]) < INFINITY);
    }
    if ((bad || (tid == 0 && s_bad)) && flag) atomicOr(flag, 16u);
}

// the dynamic-LDS attribute, set once per process before any launch or capture
extern "C" void scc_small_syev_prepare()
{
    static std::once_flag once;
    std::call_once(once, [] {
        (void)hipFuncSetAttribute((const void*)k_small_syev, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)scc_small_syev_lds_bytes());
    });
}

extern "C" hipError_t scc_launch_small_syev(const double* H, int n, int ldh, int k, double* Y, double* theta,
                                            u32* flag, hipStream_t st)
{
    if (n < 1 || n > SE_N || k < 1 || k > SE_MAXK || k > n) return hipErrorInvalidValue;
    const size_t lds = scc_small_syev_lds_bytes();
    hipLaunchKernelGGL(k_small_syev, dim3(1), dim3(SE_T), lds, st, H, n, ldh, k, Y, theta, flag);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// T = R^{-1} with G + shift I = R^T R (R upper), shift = shift_rel * tr(G):
// one wave; lane i holds row i of G in registers.  Step k: the pivot from lane
// k by readlane, rsq + one Newton step, column k of L scaled in every lane and
// written to LDS, the trailing update reads it back as broadcasts.  Then lane j
// solves column j of T against the stored L (R_im = L_mi).  flag |= 1 when a
// pivot is not positive (the block is rank deficient beyond the shift).
template <int P>
__global__ void __launch_bounds__(64) k_fsi_cholinv(const double* __restrict__ G, double shift_rel,
                                                    double* __restrict__ T, u32* __restrict__ flag)
{
    static_assert(P <= 64, "one lane per row");
    __shared__ double Lc[P][P];  // Lc[k][i] = L_ik
    __shared__ double Ri[P];     // 1 / L_kk
    const int i = threadIdx.x;
    const int ic = min(i, P - 1);
    double a[P];
    const double gii = G[(size_t)ic * P + ic];
    const double tr = se_wave_sum(i < P ? gii : 0.0);
    const double shift = shift_rel * tr;
#pragma unroll
    for (int j = 0; j < P; ++j) {
        const double g = (j >= ic) ? G[(size_t)ic * P + j] : G[(size_t)j * P + ic];
        a[j] = (i < P) ? g + (j == i ? shift : 0.0) : 0.0;
    }
    bool bad = !(tr >= 0.0) || !(tr < INFINITY);
#pragma unroll
    for (int k = 0; k < P; ++k) {
        const double d = se_readlane(a[k], k);
        bad |= !(d > 0.0);
        const double dd = d > 0.0 ? d : 1.0;
        double g = __builtin_amdgcn_rsq(dd);
        g = g * fma(-0.5 * dd * g, g, 1.5);  // Newton step on 1/sqrt
        const double lkk = dd * g;
        const double lik = (i > k) ? a[k] * g : (i == k ? lkk : 0.0);
        a[k] = lik;
        if (i < P) Lc[k][i] = lik;
        if (i == 0) Ri[k] = g;
#pragma unroll
        for (int j = k + 1; j < P; ++j) a[j] = fma(-lik, Lc[k][j], a[j]);
    }
    __syncthreads();
    // column j = i of T: for m descending, t_m = (delta_mj - sum_{l > m} L_lm t_l) / L_mm
    double t[P];
#pragma unroll
    for (int m = P - 1; m >= 0; --m) {
        double s = (m == i) ? 1.0 : 0.0;
#pragma unroll
        for (int l = m + 1; l < P; ++l) s = fma(-Lc[m][l], t[l], s);
        t[m] = s * Ri[m];
    }
    if (i < P) {
#pragma unroll
        for (int m = 0; m < P; ++m) T[(size_t)m * P + i] = t[m];
    }
    if (bad && i == 0 && flag) atomicOr(flag, 1u);
}

extern "C" hipError_t scc_launch_fsi_cholinv(const double* G, int P, double shift_rel, double* T, u32* flag,
                                             hipStream_t st)
{
    if (P == 64)
        hipLaunchKernelGGL(k_fsi_cholinv<64>, dim3(1), dim3(64), 0, st, G, shift_rel, T, flag);
    else if (P == 48)
        hipLaunchKernelGGL(k_fsi_cholinv<48>, dim3(1), dim3(64), 0, st, G, shift_rel, T, flag);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

// diagnostics (device pointers): the two small solvers alone, for tests
extern "C" SCC_API int scc_diag_small_syev(const double* H, int n, int ldh, int k,
                                                                          double* Y, double* theta, unsigned* flag)
{
    scc_small_syev_prepare();
    if (scc_launch_small_syev(H, n, ldh, k, Y, theta, flag, nullptr) != hipSuccess) return 1;
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
extern "C" SCC_API int scc_diag_cholinv(const double* G, int P, double shift_rel,
                                                                       double* T, unsigned* flag)
{
    if (scc_launch_fsi_cholinv(G, P, shift_rel, T, flag, nullptr) != hipSuccess) return 1;
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
