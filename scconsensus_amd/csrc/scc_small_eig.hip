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
#include "scc_fsi_dev.hpp"
#include "scc.h"
#include <mutex>

#define SE_N 64
#define SE_T 256
#define SE_MAXK 16

static constexpr double kSeEps = 2.220446049250313e-16;

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
// number of eigenvalues of the 64 x 64 tridiagonal T (d, e^2) below x: signs
// of the leading principal minors p_i = (d_i - x) p_{i-1} - e_{i-1}^2 p_{i-2}
// (one FMA on the dependent chain, no division), a zero pivot counted negative
// (LAPACK dstebz's -pivmin), the pair rescaled by a power of two every 8
// steps.  Fixed length: the loop unrolls completely and its LDS loads are
// issued ahead of the chain (a bound check per step made every step wait on
// its load, ~190 cycles a step).
__device__ __forceinline__ int se_count64(const double* dg, const double* e2, double x, double pivmin)
{
    double pp = 1.0, pc = dg[0] - x;
    if (pc == 0.0) pc = -pivmin;
    int neg = pc < 0.0;
#pragma unroll
    for (int i0 = 1; i0 < SE_N; i0 += 9) {
        double dv[9], ev[9];
#pragma unroll
        for (int u = 0; u < 9; ++u) {
            dv[u] = dg[min(i0 + u, SE_N - 1)];
            ev[u] = e2[min(i0 + u, SE_N - 1) - 1];
        }
#pragma unroll
        for (int u = 0; u < 9; ++u) {
            if (i0 + u >= SE_N) break;  // compile-time
            double pn = fma(dv[u] - x, pc, -ev[u] * pp);
            pn = (pn == 0.0) ? -pivmin * pc : pn;
            neg += (pn < 0.0) != (pc < 0.0);
            pp = pc;
            pc = pn;
        }
        const int ex = ilogb(pc);
        if (ex > 256 || ex < -256) {
            pc = ldexp(pc, -ex);
            pp = ldexp(pp, -ex);
        }
    }
    return neg;
}

// phase stamps of the last k_small_syev (s_memtime at the start of each phase;
// diagnostic, read by scc_diag_small_syev_stamps)
__device__ u64 g_se_stamps[8];

// dynamic LDS of k_small_syev (doubles)
#define SE_LUS (5 * SE_N + 2)                   // per-eigenpair LU stride (padded: lanes on distinct banks)
#define SE_YS (SE_N + 2)                        // tridiagonal eigenvector stride (padded likewise)
#define SE_LDS_V 0                              // [64][64] reflector i in row i
#define SE_LDS_LU (SE_LDS_V + SE_N * SE_N)      // [16][SE_LUS] LU factors per eigenpair
#define SE_LDS_Y (SE_LDS_LU + SE_MAXK * SE_LUS) // [16][SE_YS] tridiagonal eigenvectors
#define SE_LDS_TOTAL (SE_LDS_Y + SE_MAXK * SE_YS)

extern "C" size_t scc_small_syev_lds_bytes() { return sizeof(double) * SE_LDS_TOTAL; }

// H: n x n (ldh, n <= 64), symmetrised on load; k <= min(16, n) wanted.
// Y[r * 16 + q]: the q-th largest eigenvector (q < k; columns k..15 zero),
// theta[q] its Rayleigh quotient.  The matrix is always reduced as 64 x 64:
// rows and columns >= n become a decoupled diagonal block at a value below
// every eigenvalue (-(max row sum) - 1), so the top k are those of H and every
// loop has a compile-time length.  The matrix lives in registers, thread (r,
// q) holding row r, columns q + 4u.  flag |= 16 when a value is not finite or
// a cluster's vectors are dependent.
__global__ void __launch_bounds__(SE_T) k_small_syev(const double* __restrict__ H, int n, int ldh, int k,
                                                    double* __restrict__ Y, double* __restrict__ theta,
                                                    u32* __restrict__ flag)
{
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double(*Vr)[SE_N] = (double(*)[SE_N])(sm + SE_LDS_V);
    double* LU = sm + SE_LDS_LU;
    double(*Yt)[SE_YS] = (double(*)[SE_YS])(sm + SE_LDS_Y);
    __shared__ double dg[SE_N], eo[SE_N], e2[SE_N], ta[SE_N], pv[SE_N], vc[SE_N], colv[SE_N], rsum[SE_N];
    __shared__ double th[SE_MAXK], blo[SE_MAXK], bhi[SE_MAXK], gsc[4];
    __shared__ int cnt[SE_T];
    __shared__ int s_bad;
    const int tid = threadIdx.x, lane = tid & 63, wv = scc_wave_id();
    const int r = tid >> 2, q = tid & 3;  // this thread: row r, columns q + 4u
    if (tid == 0) s_bad = 0;
    double a[16];
    {
        const int rc = min(r, n - 1);
        double h1[16], h2[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int cc = min(q + 4 * u, n - 1);
            h1[u] = H[(size_t)rc * ldh + cc];
            h2[u] = H[(size_t)cc * ldh + rc];
        }
        double as = 0.0;
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const bool in = r < n && q + 4 * u < n;
            a[u] = in ? 0.5 * (h1[u] + h2[u]) : 0.0;
            as += fabs(a[u]);
        }
        as += scc_xor_lane_f64<1>(as);
        as += scc_xor_lane_f64<2>(as);
        if (q == 0) rsum[r] = as;
    }
    __syncthreads();
    {
        const double pad = -se_wave_max(rsum[lane]) - 1.0;  // below every eigenvalue of H
#pragma unroll
        for (int u = 0; u < 16; ++u)
            if (r >= n && r == q + 4 * u) a[u] = pad;
    }
    if (tid == 0) g_se_stamps[0] = __builtin_amdgcn_s_memtime();
    // ---- tridiagonalisation (LAPACK dsytd2 order), column i: its owners write
    // it to LDS, wave 0 forms the reflector, p = tau A22 v (4 threads per row),
    // w = p - (tau/2)(p.v) v, A22 -= v w^T + w v^T in registers
#pragma unroll
    for (int i = 0; i < SE_N - 2; ++i) {
        constexpr int dummy = 0;
        (void)dummy;
        const int ui = i >> 2, qi = i & 3;
        if (q == qi) {
            if (r > i) colv[r] = a[ui];
            if (r == i) dg[i] = a[ui];
        }
        __syncthreads();
        if (wv == 0) {
            const int rr = i + 1 + lane;
            const double x = colv[min(rr, SE_N - 1)];
            const double alpha = colv[i + 1];
            const double sq = se_wave_sum((rr >= i + 2 && rr < SE_N) ? x * x : 0.0);
            double beta = alpha, t = 0.0, scal = 0.0;
            if (sq > 0.0) {
                beta = -copysign(sqrt(alpha * alpha + sq), alpha);
                t = (beta - alpha) / beta;
                scal = 1.0 / (alpha - beta);
            }
            if (rr < SE_N) {
                const double v = (rr == i + 1) ? 1.0 : x * scal;
                vc[rr] = v;
                Vr[i][rr] = v;
            }
            if (lane == 0) {
                eo[i] = beta;
                ta[i] = t;
            }
        }
        __syncthreads();
        const double t = ta[i];
        double vv[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const double v = vc[q + 4 * u];
            vv[u] = (q + 4 * u > i) ? v : 0.0;
        }
        double part = 0.0;
#pragma unroll
        for (int u = 0; u < 16; ++u) part = fma(a[u], vv[u], part);
        part += scc_xor_lane_f64<1>(part);
        part += scc_xor_lane_f64<2>(part);
        if (q == 0 && r > i) pv[r] = t * part;
        __syncthreads();
        const int rr = i + 1 + lane;
        const double K = -0.5 * t * se_wave_sum(rr < SE_N ? pv[min(rr, SE_N - 1)] * vc[min(rr, SE_N - 1)] : 0.0);
        const double vr = (r > i) ? vc[r] : 0.0;
        const double wr = (r > i) ? fma(K, vr, pv[r]) : 0.0;
        double pw[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) pw[u] = pv[q + 4 * u];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const double wc = (q + 4 * u > i) ? fma(K, vv[u], pw[u]) : 0.0;
            a[u] = fma(-vr, wc, fma(-wr, vv[u], a[u]));
        }
    }
    if (q == 2 && r == SE_N - 2) dg[SE_N - 2] = a[15];
    if (q == 2 && r == SE_N - 1) eo[SE_N - 2] = a[15];
    if (q == 3 && r == SE_N - 1) dg[SE_N - 1] = a[15];
    if (tid == 0) {
        eo[SE_N - 1] = 0.0;
        ta[SE_N - 2] = 0.0;
        ta[SE_N - 1] = 0.0;
    }
    __syncthreads();
    if (tid == 0) g_se_stamps[1] = __builtin_amdgcn_s_memtime();
    // ---- Gershgorin bounds, pivmin (LAPACK dstebz)
    if (wv == 0) {
        const int i = lane;
        const double ei = eo[i], dgi = dg[i];
        e2[i] = ei * ei;
        const double rad = (i > 0 ? fabs(eo[max(i - 1, 0)]) : 0.0) + fabs(ei);
        const double gl = se_wave_min(dgi - rad);
        const double gu = se_wave_max(dgi + rad);
        const double em = se_wave_max(ei * ei);
        if (lane == 0) {
            gsc[0] = gl;
            gsc[1] = gu;
            gsc[2] = em;
        }
    }
    __syncthreads();
    if (tid == 0) g_se_stamps[2] = __builtin_amdgcn_s_memtime();
    const double tnorm = fmax(fabs(gsc[0]), fabs(gsc[1]));
    const double pivmin = fmax(2.2250738585072014e-308 * fmax(1.0, gsc[2]), 1e-300);
    const double glo = gsc[0] - 2.0 * tnorm * kSeEps * SE_N - 1e-300;
    const double ghi = gsc[1] + 2.0 * tnorm * kSeEps * SE_N + 1e-300;
    // ---- eigenvalues: one shared round of 256 points, then 16 points per
    // wanted eigenvalue per round until the bracket is below
    // max(1e-12 |lambda|, 2 eps ||T||) (inverse iteration's need; the value
    // returned is the Rayleigh quotient)
    {
        const double x = glo + (ghi - glo) * (double)(tid + 1) / (double)(SE_T + 1);
        cnt[tid] = se_count64(dg, e2, x, pivmin);
    }
    __syncthreads();
    const int qg = tid >> 4, jg = tid & 15;
    const int idx = SE_N - 1 - qg;  // ascending index of the qg-th largest (the pad block is lowest)
    const bool want = qg < k;
    if (want && jg == 0) {
        int lo = 0, hi = SE_T;  // first point with cnt > idx (cnt is nondecreasing in the point)
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
        const double lo = want ? blo[qg] : 0.0, hi = want ? bhi[qg] : 0.0;
        if (!done) {
            const double x = lo + (hi - lo) * (double)(jg + 1) / 17.0;
            const int c = se_count64(dg, e2, x, pivmin);
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
    if (tid == 0) g_se_stamps[3] = __builtin_amdgcn_s_memtime();
    // ---- inverse iteration: eigenpair q on lane q of wave 0 (LU with partial
    // pivoting of T - lambda I, two solves from a pseudo-random start)
    if (wv == 0 && lane < k) {
        const int qq = lane;
        const double lam = 0.5 * (blo[qq] + bhi[qq]);
        double* fdr = LU + (size_t)qq * SE_LUS;  // 1 / U diagonal
        double* fu = fdr + SE_N;
        double* fu2 = fu + SE_N;
        double* fl = fu2 + SE_N;
        double* fp = fl + SE_N;
        double* y = Yt[qq];
        const double tiny = kSeEps * tnorm + 1e-300;
        double dcur = dg[0] - lam, ucur = eo[0];
#pragma unroll
        for (int i = 0; i < SE_N - 1; ++i) {
            const double li = eo[i], dn = dg[i + 1] - lam, un = (i < SE_N - 2) ? eo[i + 1] : 0.0;
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
        fdr[SE_N - 1] = 1.0 / dcur;
        fu[SE_N - 1] = 0.0;
        fu2[SE_N - 1] = 0.0;
        // the iterate in LDS (this lane's row of Yt); fixed-length unrolled loops
        // let the compiler issue the loads ahead of each dependent chain
#pragma unroll
        for (int i = 0; i < SE_N; ++i) {
            unsigned h = (unsigned)i * 2654435761u ^ ((unsigned)qq * 40503u + 12345u);
            h ^= h >> 13;
            h *= 0x5bd1e995u;
            h ^= h >> 15;
            y[i] = 0.5 + (double)(h & 0xffff) / 65536.0;
        }
        for (int iter = 0; iter < 2; ++iter) {
            double bi = y[0];  // y <- L^-1 P y
#pragma unroll
            for (int i = 0; i < SE_N - 1; ++i) {
                const bool piv = fp[i] != 0.0;
                const double bn = y[i + 1];
                const double xa = piv ? bn : bi, xb = piv ? bi : bn;
                y[i] = xa;
                bi = fma(-fl[i], xa, xb);
            }
            y[SE_N - 1] = bi;
            double z1 = 0.0, z2 = 0.0;  // y <- U^-1 y from the bottom
#pragma unroll
            for (int i = SE_N - 1; i >= 0; --i) {
                const double z0 = fma(-fu[i], z2, fma(-fu2[i], z1, y[i])) * fdr[i];
                y[i] = z0;
                z1 = z2;
                z2 = z0;
            }
            double mx = 0.0, sacc = 0.0;
#pragma unroll
            for (int i = 0; i < SE_N; ++i) mx = fmax(mx, fabs(y[i]));
            const double sc = (mx > 0.0 && mx < INFINITY) ? 1.0 / mx : 1.0;
#pragma unroll
            for (int i = 0; i < SE_N; ++i) sacc = fma(y[i] * sc, y[i] * sc, sacc);
            const double inv = sc / sqrt(sacc);
#pragma unroll
            for (int i = 0; i < SE_N; ++i) y[i] *= inv;
        }
    }
    __syncthreads();
    if (tid == 0) g_se_stamps[4] = __builtin_amdgcn_s_memtime();
    // ---- Gram-Schmidt inside clusters (|lambda_p - lambda_q| <= 1e-3 ||T||,
    // LAPACK dstein), in order, then the Rayleigh quotients y^T T y (wave 0,
    // lane = entry)
    if (wv == 0) {
        const int i = lane;
        const double di = dg[i], ei = eo[i], em = eo[max(i - 1, 0)];
        for (int qq = 0; qq < k; ++qq) {
            double yq = Yt[qq][i];
            const double lq = 0.5 * (blo[qq] + bhi[qq]);
            bool touched = false;
            for (int p = 0; p < qq; ++p) {
                const double lp = 0.5 * (blo[p] + bhi[p]);
                if (fabs(lp - lq) > 1e-3 * tnorm) continue;
                const double yp = Yt[p][i];
                const double d = se_wave_sum(yp * yq);
                yq = fma(-d, yp, yq);
                touched = true;
            }
            if (touched) {
                const double s2 = se_wave_sum(yq * yq);
                if (!(s2 > 1e-6)) s_bad = 1;  // the cluster's vectors were (nearly) dependent
                yq *= 1.0 / sqrt(s2);
                Yt[qq][i] = yq;
            }
            const double yu = Yt[qq][min(i + 1, SE_N - 1)], yd = Yt[qq][max(i - 1, 0)];
            const double tv = yq * di + (i + 1 < SE_N ? ei * yu : 0.0) + (i > 0 ? em * yd : 0.0);
            const double rq = se_wave_sum(yq * tv);
            if (lane == 0) th[qq] = rq;
        }
    }
    __syncthreads();
    if (tid == 0) g_se_stamps[5] = __builtin_amdgcn_s_memtime();
    // ---- back-transformation y <- H_0 ... H_{61} y: group qg (16 lanes) holds
    // eigenvector qg, entries r = jg + 16 u in registers
    double yv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) yv[u] = want ? Yt[qg][jg + 16 * u] : 0.0;
#pragma unroll
    for (int i = SE_N - 3; i >= 0; --i) {
        double vv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int rr = jg + 16 * u;
            const double v = Vr[i][rr];
            vv[u] = (rr > i) ? v : 0.0;
        }
        const double ti = ta[i];
        double d = 0.0;
#pragma unroll
        for (int u = 0; u < 4; ++u) d = fma(vv[u], yv[u], d);
        d += scc_xor_lane_f64<1>(d);
        d += scc_xor_lane_f64<2>(d);
        d += scc_xor_lane_f64<4>(d);
        d += scc_xor_lane_f64<8>(d);
        const double td = ti * d;
#pragma unroll
        for (int u = 0; u < 4; ++u) yv[u] = fma(-td, vv[u], yv[u]);
    }
    bool bad = false;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int rr = jg + 16 * u;
        if (rr < n) Y[(size_t)rr * 16 + qg] = want ? yv[u] : 0.0;
        bad |= !(fabs(yv[u]) < INFINITY);
    }
    if (want && jg == 0) {
        theta[qg] = th[qg];
        bad |= !(fabs(th[qg]) < INFINITY);
    }
    if ((bad || (tid == 0 && s_bad)) && flag) atomicOr(flag, 16u);
    if (tid == 0) g_se_stamps[6] = __builtin_amdgcn_s_memtime();
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
// T = R^{-1} with G + shift I = R^T R (R upper), shift = shift_rel * tr(G), by
// TWO waves working concurrently (P <= 64):
//   wave 0  the Cholesky G = L L^T, right-looking, lane i = row i in registers:
//           step k takes the pivot by readlane, rsq + one Newton step, scales
//           column k, writes it to LDS (by column and by row), publishes k + 1
//           in an LDS word, and updates its trailing columns from broadcast
//           reads of column k (16 at a time, the next chunk loading under the
//           current chunk's FMAs);
//   wave 1  W = L^{-1} column by column, lane j = column j, row i as soon as
//           wave 0 has published step i: w_i = (delta_ij - sum_{m<i} L_im w_m) / L_ii
//           (row i of L read as broadcasts); then T = W^T.
// Each wave issues ~P^2/2 FMAs; they overlap instead of running back to back.
// flag |= 1 when a pivot is not positive (rank deficient beyond the shift).
#define CI_LRS 65  // row-major copy of L: padded stride (lanes on distinct banks)
template <int P>
__device__ __forceinline__ void fsi_chol_wave(const double* __restrict__ G, double shift_rel,
                                                         u32* __restrict__ flag, double (*Lc)[P], double* Lr,
                                                         double* Ri, int* s_step)
{
    static_assert(P <= 64 && P % 16 == 0, "one lane per row, 16-column chunks");
    const int lane = threadIdx.x & 63;
    const int ic = min(lane, P - 1);
    {
        double a[P];
        const double gii = G[(size_t)ic * P + ic];
        const double tr = se_wave_sum(lane < P ? gii : 0.0);
        const double shift = shift_rel * tr;
#pragma clang loop unroll(full)
        for (int j = 0; j < P; ++j) {  // row ic of G (k_fsi_gram's output is exactly symmetric)
            const double g = G[(size_t)ic * P + j];
            a[j] = (lane < P) ? g + (j == lane ? shift : 0.0) : 0.0;
        }
        bool bad = !(tr >= 0.0) || !(tr < INFINITY);
#pragma clang loop unroll(full)
        for (int k = 0; k < P; ++k) {
            __builtin_amdgcn_sched_barrier(0);
            const double d = se_readlane(a[k], k);
            bad |= !(d > 0.0);
            const double dd = d > 0.0 ? d : 1.0;
            double g = __builtin_amdgcn_rsq(dd);
            g = g * fma(-0.5 * dd * g, g, 1.5);  // Newton step on 1/sqrt
            const double lkk = dd * g;
            const double lik = (lane > k) ? a[k] * g : (lane == k ? lkk : 0.0);
            a[k] = lik;
            if (lane < P) Lc[k][lane] = lik;
            if (lane == 0) Ri[k] = g;
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the column is in LDS
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0) __hip_atomic_store(s_step, k + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            // trailing update a_j -= L_ik L_jk, j > k, in 16-column chunks
#pragma clang loop unroll(full)
            for (int j0 = (k + 1) & ~15; j0 < P; j0 += 16) {
                double l16[16];
#pragma clang loop unroll(full)
                for (int u = 0; u < 16; ++u) l16[u] = Lc[k][j0 + u];
#pragma clang loop unroll(full)
                for (int u = 0; u < 16; ++u)
                    if (j0 + u > k) a[j0 + u] = fma(-lik, l16[u], a[j0 + u]);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if (bad && lane == 0 && flag) atomicOr(flag, 1u);
    }
}

// wave 1: column j = lane of W = L^{-1} kept in LDS (Wt[j][*], padded rows);
// w_i = (delta_ij - sum_{m<i} L_im w_m) / L_ii as soon as wave 0 published
// step i.  (w in registers next to the loaded row of L needs ~256 VGPRs and
// spills once wave 0's path shares the kernel; in LDS the wave streams two
// reads per FMA and overlaps wave 0's factorisation.)
template <int P>
__device__ __forceinline__ void fsi_inv_wave(double* __restrict__ T, const double* Lr, const double* Ri,
                                             const int* s_step, double* Wt)
{
    const int lane = threadIdx.x & 63;
    const int j = lane;
    double* wj = Wt + (size_t)min(j, P - 1) * CI_LRS;
    for (int i = 0; i < P; ++i) {
        if (lane == 0)
            while (__hip_atomic_load((int*)s_step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) <= i)
                __builtin_amdgcn_s_sleep(1);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const double* li = Lr + (size_t)i * CI_LRS;
        double s0 = (i == j) ? 1.0 : 0.0, s1 = 0.0;
        int m = j;  // w_m = 0 for m < j
        for (; m + 1 < i; m += 2) {
            s0 = fma(-li[m], wj[m], s0);
            s1 = fma(-li[m + 1], wj[m + 1], s1);
        }
        if (m < i) s0 = fma(-li[m], wj[m], s0);
        const double wi = (i >= j) ? (s0 + s1) * Ri[i] : 0.0;
        if (j < P) wj[i] = wi;
    }
    __builtin_amdgcn_wave_barrier();
    // T = W^T: row j of T is column j of W (zero left of the diagonal)
    if (j < P)
        for (int i = 0; i < P; ++i) T[(size_t)j * P + i] = (i >= j) ? wj[i] : 0.0;
}

template <int P>
__device__ __forceinline__ void fsi_cholinv_2w(const double* __restrict__ G, double shift_rel, double* __restrict__ T,
                                               u32* __restrict__ flag, double (*Lc)[P], double* Lr, double* Ri,
                                               int* s_step, double* Wt)
{
    const int wv = scc_wave_id();  // wave-uniform: the two paths are separate code, not one masked stream
    if (wv == 0)
        fsi_chol_wave<P>(G, shift_rel, flag, Lc, Lr, Ri, s_step);
    else if (wv == 1)
        fsi_inv_wave<P>(T, Lr, Ri, s_step, Wt);
}

// One wave: the Cholesky above (registers, lane = row), then W = L^{-1}
// column by column (lane j = column j in registers, row i of L read as
// broadcasts 16 at a time) and T = W^T.  (Two waves overlapping the two halves
// made the compiler spill ~7 KB per lane; here the allocator keeps every value
// in VGPRs/AGPRs.)
__global__ void __launch_bounds__(64) k_fsi_cholinv64(const double* __restrict__ G, double shift_rel,
                                                      double* __restrict__ T, u32* __restrict__ flag)
{
    __shared__ double Lc[64][64];
    __shared__ double Lr[64 * CI_LRS];
    __shared__ double Ri[64];
    __shared__ int s_step;
    fsi_chol_wave<64>(G, shift_rel, flag, Lc, Lr, Ri, &s_step);
    __syncthreads();
    const int j = threadIdx.x;
    double w[64];
#pragma clang loop unroll(full)
    for (int i = 0; i < 64; ++i) {
        __builtin_amdgcn_sched_barrier(0);
        double s = (i == j) ? 1.0 : 0.0;
#pragma clang loop unroll(full)
        for (int m0 = 0; m0 < i; m0 += 16) {
            double l16[16];
#pragma clang loop unroll(full)
            for (int u = 0; u < 16; ++u) l16[u] = (m0 + u < i) ? Lc[m0 + u][i] : 0.0;
#pragma clang loop unroll(full)
            for (int u = 0; u < 16; ++u)
                if (m0 + u < i) s = fma(-l16[u], w[m0 + u], s);
            __builtin_amdgcn_sched_barrier(0);
        }
        w[i] = (i >= j) ? s * Ri[i] : 0.0;
    }
#pragma clang loop unroll(full)
    for (int i = 0; i < 64; ++i) T[j * 64 + i] = w[i];
}

// T = R^{-1} = (L^{-1})^T for G + shift I = L L^T, one 256-thread workgroup
__global__ void __launch_bounds__(256) k_fsi_cholinv_blk(const double* __restrict__ G, double shift_rel,
                                                        double* __restrict__ T, u32* __restrict__ flag)
{
    __shared__ double A[64 * CB_S];
    __shared__ double X[64 * CB_S];
    __shared__ double Ri[64];
    __shared__ double s_tr;
    __shared__ int s_bad;
    const int tid = threadIdx.x;
    if (tid < 64) {
        const double tr = se_wave_sum(G[tid * 64 + tid]);
        if (tid == 0) {
            s_tr = tr;
            s_bad = !(tr >= 0.0) || !(tr < INFINITY);
        }
    }
    __syncthreads();
    const double shift = shift_rel * s_tr;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
        const int e = tid + 256 * u, i = e >> 6, j = e & 63;
        A[i * CB_S + j] = G[e] + (i == j ? shift : 0.0);
    }
    __syncthreads();
    fsi_cholinv_blk(A, X, Ri, &s_bad);
    // T[i][j] = X[j][i]
#pragma unroll
    for (int u = 0; u < 16; ++u) {
        const int e = tid + 256 * u, i = e >> 6, j = e & 63;
        T[e] = X[j * CB_S + i];
    }
    if (tid == 0 && s_bad && flag) atomicOr(flag, 1u);
}

static int cholinv_variant()
{
    const char* e = getenv("SCC_FSI_CHOL");  // 0: the one-wave kernel
    return (e && *e) ? atoi(e) : 1;
}

extern "C" hipError_t scc_launch_fsi_cholinv(const double* G, int P, double shift_rel, double* T, u32* flag,
                                             hipStream_t st)
{
    if (P != 64) return hipErrorInvalidValue;
    if (cholinv_variant())
        hipLaunchKernelGGL(k_fsi_cholinv_blk, dim3(1), dim3(256), 0, st, G, shift_rel, T, flag);
    else
        hipLaunchKernelGGL(k_fsi_cholinv64, dim3(1), dim3(64), 0, st, G, shift_rel, T, flag);
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

extern "C" SCC_API int scc_diag_small_syev_stamps(unsigned long long* out)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_se_stamps), sizeof(u64) * 8) == hipSuccess ? 0 : 1;
}
