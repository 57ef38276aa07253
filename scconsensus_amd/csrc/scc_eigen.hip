// scc_eigen.hip — top-k eigenpairs of the |U| x |U| fp64 Gram matrix.
//
// Dense symmetric eigensolver for the PCA step of stage 3 (reference:
// irlba::prcomp_irlba, R/reclusterDEConsensusFast.R:398).  The spectrum of
// the centred union-gene Gram is a few cluster "spikes" over a noise bulk, so
// the 15th/16th eigenvalues are routinely within 1e-3 relative of each other
// (SURVEY D5): Krylov/subspace iterations need hundreds of steps there, while
// a direct method is exact to fp64 backward error.  One workgroup (16 waves):
//   1. Householder tridiagonalisation, LAPACK dsytd2 order.  One fused sweep
//      per step: the rank-2 update of step k and the symv of step k+1 share a
//      pass over the trailing block (3 rows in flight per wave); the trailing
//      block moves from L2 into LDS once it fits.  5 barriers per step.
//   2. the k largest eigenvalues of T by multisection (64 Sturm counts per
//      wave per round), T resident in LDS
//   3. eigenvectors of T by inverse iteration (dgttrf/dgttrs LU with partial
//      pivoting, factors in LDS), re-orthogonalised inside eigenvalue clusters
//      (|dl| <= 1e-3 ||T||, as LAPACK dstein)
//   4. back-transformation by the stored reflectors, vectors in LDS
// Output Z[u*16 + q] = q-th largest eigenvector (q < k), zero padded to 16.
// Every LDS array has a global fall-back in `scratch` for very large |U|.
#include "scc_common.hpp"

#define EIG_T 1024
#define EIG_W (EIG_T / 64)
#ifndef EIG_RU
#define EIG_RU 3  // rows in flight per wave in the fused sweep (4 spills at 128 VGPRs)
#endif
#define EIG_LDS_BYTES (156 * 1024)
#define EIG_LDS_DBL (EIG_LDS_BYTES / 8)

__device__ inline double wave_sum_d(double v)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    return v;
}

__device__ inline double block_sum(double v, double* red)
{
    const int lane = threadIdx.x & 63, w = scc_wave_id();
    v = wave_sum_d(v);
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    double s = 0.0;
    for (int i = 0; i < EIG_W; ++i) s += red[i];  // fixed order: deterministic
    return s;
}

// number of eigenvalues of T (d, e^2) strictly below x (Sturm sequence)
__device__ inline int sturm_count(const double* d, const double* e2, int n, double x, double pivmin)
{
    int c = 0;
    double q = d[0] - x;
    if (fabs(q) < pivmin) q = -pivmin;
    c += (q < 0.0);
    for (int i = 1; i < n; ++i) {
        q = d[i] - x - e2[i - 1] / q;
        if (fabs(q) < pivmin) q = -pivmin;
        c += (q < 0.0);
    }
    return c;
}

// Fused sweep of step k: rows i = 1..m-1 of the trailing block T (local
// (i,j) at T[(off+i)*ld + off+j]) get the rank-2 update of step k, and the
// same sweep forms p' = tau' T' v' for step k+1 (written to pn) plus each
// wave's partial of p'.v' (pdot[wave]).  Output rows go to O (ldo, offo).
template <class TP, class OP>
__device__ __forceinline__ void fused_pass(TP T, int ld, int off, OP O, int ldo, int offo, int m, const double* v,
                                           const double* w, const double* vn, double taun, double* pn, double* pdot)
{
    const int lane = threadIdx.x & 63, wv = scc_wave_id();
    double dacc = 0.0;
    for (int i0 = 1 + wv; i0 < m; i0 += EIG_RU * EIG_W) {
        int r[EIG_RU];
        bool ok[EIG_RU];
        double vi[EIG_RU], wi[EIG_RU], s[EIG_RU];
#pragma unroll
        for (int u = 0; u < EIG_RU; ++u) {
            r[u] = i0 + u * EIG_W;
            ok[u] = r[u] < m;
            vi[u] = ok[u] ? v[r[u]] : 0.0;
            wi[u] = ok[u] ? w[r[u]] : 0.0;
            s[u] = 0.0;
        }
        for (int j = 1 + lane; j < m; j += 64) {
            const double vj = v[j], wj = w[j], vnj = vn[j - 1];
            double x[EIG_RU];
#pragma unroll
            for (int u = 0; u < EIG_RU; ++u) x[u] = ok[u] ? T[(size_t)(off + r[u]) * ld + off + j] : 0.0;
#pragma unroll
            for (int u = 0; u < EIG_RU; ++u) {
                if (ok[u]) {
                    const double y = x[u] - vi[u] * wj - wi[u] * vj;
                    O[(size_t)(offo + r[u] - 1) * ldo + offo - 1 + j] = y;
                    s[u] += y * vnj;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < EIG_RU; ++u) {
            const double su = wave_sum_d(s[u]) * taun;
            if (ok[u] && lane == 0) {
                pn[r[u] - 1] = su;
                dacc += su * vn[r[u] - 1];
            }
        }
    }
    if (lane == 0) pdot[wv] = dacc;
}

#define ESTAMP(ph)                                                                  \
    do {                                                                            \
        if (stamps && threadIdx.x == 0) stamps[ph] = __builtin_amdgcn_s_memtime(); \
    } while (0)

// A: n x n symmetric (full), row-major, leading dimension lda; destroyed (the
// reflectors are left in its rows: A[k][k+1] = 1, A[k][k+2..] = v tail).
// scratch doubles: 104 n.  Z: n x 16 out.  W: k out (descending).
__global__ void __launch_bounds__(EIG_T) k_syevx_topk(double* A, int n, int lda, int k, double* scratch, double* Z,
                                                      double* W, u64* stamps)
{
    extern __shared__ __attribute__((aligned(16))) double sm[];
    __shared__ double sh[8];
    ESTAMP(0);
    const int tid = threadIdx.x, lane = tid & 63, wv = scc_wave_id();
    double* red = sm;        // 16
    double* pdot = sm + 16;  // 16
    double* d = scratch;     // n
    double* e = d + n;       // n
    double* tau = e + n;     // n
    double* gbuf = tau + n;  // global fall-back space (99 n)
    // ---------------------------------------------------------------- 1. tridiagonalise
    const bool vec_lds = (32 + 4 * (size_t)n) <= EIG_LDS_DBL;
    double* vbuf0 = vec_lds ? sm + 32 : gbuf;
    double* vbuf1 = vbuf0 + n;
    double* wbuf = vbuf1 + n;
    double* pbuf = wbuf + n;
    int mlds = 0;
    if (vec_lds) {
        mlds = (int)sqrt((double)(EIG_LDS_DBL - 32 - 4 * (size_t)n));
        if (mlds > n) mlds = n;
    }
    double* Tl = sm + 32 + 4 * (size_t)n;
    if (n <= 2) {
        if (tid == 0) {
            d[0] = A[0];
            e[0] = (n == 2) ? A[1] : 0.0;
            tau[0] = 0.0;
            if (n == 2) {
                d[1] = A[(size_t)lda + 1];
                e[1] = 0.0;
                tau[1] = 0.0;
            }
        }
    } else {
        {  // reflector 0 from row 0, then p = tau A22 v
            const int m = n - 1;
            double part = 0.0;
            for (int j = 2 + tid; j < n; j += EIG_T) part += A[j] * A[j];
            const double xn2 = block_sum(part, red);
            const double alpha = A[1];
            double t = 0.0, beta = alpha, scal = 0.0;
            if (xn2 > 0.0) {
                beta = -copysign(sqrt(alpha * alpha + xn2), alpha);
                t = (beta - alpha) / beta;
                scal = 1.0 / (alpha - beta);
            }
            for (int j = tid; j < m; j += EIG_T) vbuf0[j] = (j == 0) ? 1.0 : A[1 + j] * scal;
            __syncthreads();
            for (int j = tid; j < m; j += EIG_T) A[1 + j] = vbuf0[j];
            if (tid == 0) {
                d[0] = A[0];
                e[0] = beta;
                tau[0] = t;
                sh[0] = t;
            }
            double dacc = 0.0;
            for (int i = wv; i < m; i += EIG_W) {
                const double* ri = A + (size_t)(1 + i) * lda + 1;
                double s = 0.0;
                for (int j = lane; j < m; j += 64) s += ri[j] * vbuf0[j];
                s = wave_sum_d(s) * t;
                if (lane == 0) {
                    pbuf[i] = s;
                    dacc += s * vbuf0[i];
                }
            }
            if (lane == 0) pdot[wv] = dacc;
            __syncthreads();
        }
        bool in_lds = false;
        int lds_base = 0, lds_ld = 0;
        int cur = 0;
        for (int kk = 0; kk <= n - 3; ++kk) {
            const int m = n - kk - 1;  // trailing block A22 = rows/cols kk+1 .. n-1
            double* v = cur ? vbuf1 : vbuf0;
            double* vn = cur ? vbuf0 : vbuf1;
            const double t = sh[0];
            double dot = 0.0;
            for (int i = 0; i < EIG_W; ++i) dot += pdot[i];
            const double a2 = -0.5 * t * dot;
            for (int i = tid; i < m; i += EIG_T) wbuf[i] = (t != 0.0) ? pbuf[i] + a2 * v[i] : 0.0;
            __syncthreads();
            const double* row0;
            int ld0;
            if (in_lds) {
                const int o = kk + 1 - lds_base;
                ld0 = lds_ld;
                row0 = Tl + (size_t)o * ld0 + o;
            } else {
                ld0 = lda;
                row0 = A + (size_t)(kk + 1) * ld0 + kk + 1;
            }
            const double v0 = v[0], w0 = wbuf[0];
            if (kk == n - 3) {  // 2 x 2 remainder
                if (tid == 0) {
                    d[n - 2] = row0[0] - 2.0 * v0 * w0;
                    e[n - 2] = row0[1] - v0 * wbuf[1] - w0 * v[1];
                    d[n - 1] = row0[ld0 + 1] - 2.0 * v[1] * wbuf[1];
                    e[n - 1] = 0.0;
                    tau[n - 2] = 0.0;
                    tau[n - 1] = 0.0;
                }
                break;
            }
            double part = 0.0;
            for (int j = 2 + tid; j < m; j += EIG_T) {
                const double x = row0[j] - v0 * wbuf[j] - w0 * v[j];
                part += x * x;
            }
            const double xn2 = block_sum(part, red);
            const double alpha = row0[1] - v0 * wbuf[1] - w0 * v[1];
            double tn = 0.0, beta = alpha, scal = 0.0;
            if (xn2 > 0.0) {
                beta = -copysign(sqrt(alpha * alpha + xn2), alpha);
                tn = (beta - alpha) / beta;
                scal = 1.0 / (alpha - beta);
            }
            for (int j = 1 + tid; j < m; j += EIG_T) {
                const double x = row0[j] - v0 * wbuf[j] - w0 * v[j];
                vn[j - 1] = (j == 1) ? 1.0 : x * scal;
            }
            if (tid == 0) {
                d[kk + 1] = row0[0] - 2.0 * v0 * w0;
                e[kk + 1] = beta;
                tau[kk + 1] = tn;
                sh[0] = tn;
            }
            __syncthreads();
            double* refl = A + (size_t)(kk + 1) * lda + kk + 2;
            for (int j = tid; j < m - 1; j += EIG_T) refl[j] = vn[j];
            const int mn = m - 1;
            if (!in_lds && mn <= mlds) {
                fused_pass(A, lda, kk + 1, Tl, mn, 0, m, v, wbuf, vn, tn, pbuf, pdot);
                in_lds = true;
                lds_base = kk + 2;
                lds_ld = mn;
            } else if (in_lds) {
                const int o = kk + 1 - lds_base;
                fused_pass(Tl, lds_ld, o, Tl, lds_ld, o + 1, m, v, wbuf, vn, tn, pbuf, pdot);
            } else {
                fused_pass(A, lda, kk + 1, A, lda, kk + 2, m, v, wbuf, vn, tn, pbuf, pdot);
            }
            __syncthreads();
            cur ^= 1;
        }
    }
    __syncthreads();
    ESTAMP(1);
    // ---------------------------------------------------------------- 2. eigenvalues
    // T into LDS (d, e, e^2), then the eigenvector block Zl (n x 16) and LU slots
    const bool t_lds = (32 + 19 * (size_t)n) <= EIG_LDS_DBL;
    double* dl = t_lds ? sm + 32 : gbuf;
    double* el = dl + n;
    double* e2l = el + n;
    double* Zl = e2l + n;  // n x 16
    for (int i = tid; i < n; i += EIG_T) {
        dl[i] = d[i];
        el[i] = e[i];
        e2l[i] = e[i] * e[i];
    }
    for (int i = tid; i < 16 * n; i += EIG_T) Zl[i] = 0.0;
    __syncthreads();
    if (tid == 0) {  // Gershgorin bounds, pivmin as LAPACK dstebz
        double gl = dl[0], gu = dl[0], emax2 = 0.0;
        for (int i = 0; i < n; ++i) {
            const double r = (i > 0 ? fabs(el[i - 1]) : 0.0) + (i < n - 1 ? fabs(el[i]) : 0.0);
            gl = fmin(gl, dl[i] - r);
            gu = fmax(gu, dl[i] + r);
            if (i < n - 1) emax2 = fmax(emax2, e2l[i]);
        }
        const double tnorm = fmax(fabs(gl), fabs(gu));
        const double eps = 2.220446049250313e-16;
        sh[0] = gl - 2.0 * tnorm * eps * n - 1e-300;
        sh[1] = gu + 2.0 * tnorm * eps * n + 1e-300;
        sh[2] = fmax(2.2250738585072014e-308 * fmax(1.0, emax2), 1e-300);
        sh[3] = tnorm;
    }
    __syncthreads();
    const double pivmin = sh[2], tnorm = sh[3];
    for (int q = wv; q < k; q += EIG_W) {
        const int target = n - 1 - q;  // ascending index of the q-th largest
        double lo = sh[0], hi = sh[1];
        for (int it = 0; it < 40; ++it) {
            const double x = lo + (hi - lo) * (double)(lane + 1) / 65.0;
            const int c = sturm_count(dl, e2l, n, x, pivmin);
            const unsigned long long above = __ballot(c > target);  // lambda_target < x
            const int first = above ? __builtin_ctzll(above) : 64;
            const double nlo = (first == 0) ? lo : lo + (hi - lo) * (double)first / 65.0;
            const double nhi = (first == 64) ? hi : lo + (hi - lo) * (double)(first + 1) / 65.0;
            if (nlo == lo && nhi == hi) break;
            lo = nlo;
            hi = nhi;
            if (hi - lo <= 2.0 * 2.220446049250313e-16 * fmax(fabs(lo), fabs(hi)) + pivmin) break;
        }
        if (lane == 0) W[q] = 0.5 * (lo + hi);
    }
    __syncthreads();
    ESTAMP(2);
    // ---------------------------------------------------------------- 3. inverse iteration
    // Waves factor T - lambda_q I into their LU slot and solve in place on
    // column q of Zl; between solves wave 0 re-orthogonalises each vector
    // against the earlier members of its eigenvalue cluster and normalises.
    {
        const double eps = 2.220446049250313e-16;
        const double tiny = eps * tnorm + 1e-300;
        const size_t slot = 5 * (size_t)n;
        double* slots = nullptr;
        int nslots = 0;
        if (t_lds) {
            const size_t used = 32 + 19 * (size_t)n;
            nslots = (int)((EIG_LDS_DBL - used) / slot);
            slots = sm + used;
        }
        if (nslots < 1) {  // global fall-back (very large |U|)
            slots = gbuf + 19 * (size_t)n;
            nslots = EIG_W;
        }
        if (nslots > EIG_W) nslots = EIG_W;
        for (int q0 = 0; q0 < k; q0 += nslots) {
            const int q = q0 + wv;
            const bool act = (wv < nslots) && (q < k);
            double* dd = slots + (size_t)wv * slot;
            double* du = dd + n;
            double* du2 = du + n;
            double* dlw = du2 + n;
            double* piv = dlw + n;
            if (act) {
                const double lam = W[q];
                if (lane == 0) {
                    for (int i = 0; i < n; ++i) {
                        dd[i] = dl[i] - lam;
                        du[i] = (i < n - 1) ? el[i] : 0.0;
                        dlw[i] = (i < n - 1) ? el[i] : 0.0;
                        du2[i] = 0.0;
                        piv[i] = 0.0;
                    }
                    for (int i = 0; i < n - 1; ++i) {
                        if (fabs(dd[i]) >= fabs(dlw[i])) {
                            if (dd[i] == 0.0) dd[i] = tiny;
                            const double f = dlw[i] / dd[i];
                            dlw[i] = f;
                            dd[i + 1] -= f * du[i];
                        } else {
                            const double f = dd[i] / dlw[i];
                            dd[i] = dlw[i];
                            dlw[i] = f;
                            const double tt = du[i];
                            du[i] = dd[i + 1];
                            dd[i + 1] = tt - f * dd[i + 1];
                            if (i < n - 2) {
                                du2[i] = du[i + 1];
                                du[i + 1] = -f * du[i + 1];
                            }
                            piv[i] = 1.0;
                        }
                    }
                    if (dd[n - 1] == 0.0) dd[n - 1] = tiny;
                }
                for (int i = lane; i < n; i += 64) {  // deterministic pseudo-random start
                    unsigned h = (unsigned)i * 2654435761u ^ ((unsigned)q * 40503u + 12345u);
                    h ^= h >> 13;
                    h *= 0x5bd1e995u;
                    h ^= h >> 15;
                    Zl[(size_t)i * 16 + q] = 0.5 + (double)(h & 0xffff) / 65536.0;
                }
            }
            __syncthreads();
            for (int iter = 0; iter < 3; ++iter) {
                if (act && lane == 0) {
                    double* b = Zl + q;  // stride 16
                    for (int i = 0; i < n - 1; ++i) {
                        if (piv[i] == 0.0) {
                            b[(size_t)(i + 1) * 16] -= dlw[i] * b[(size_t)i * 16];
                        } else {
                            const double tt = b[(size_t)i * 16];
                            b[(size_t)i * 16] = b[(size_t)(i + 1) * 16];
                            b[(size_t)(i + 1) * 16] = tt - dlw[i] * b[(size_t)i * 16];
                        }
                    }
                    b[(size_t)(n - 1) * 16] /= dd[n - 1];
                    if (n >= 2)
                        b[(size_t)(n - 2) * 16] =
                            (b[(size_t)(n - 2) * 16] - du[n - 2] * b[(size_t)(n - 1) * 16]) / dd[n - 2];
                    for (int i = n - 3; i >= 0; --i)
                        b[(size_t)i * 16] = (b[(size_t)i * 16] - du[i] * b[(size_t)(i + 1) * 16] -
                                             du2[i] * b[(size_t)(i + 2) * 16]) /
                                            dd[i];
                }
                __syncthreads();
                if (wv == 0) {
                    const int qe = min(k, q0 + nslots);
                    for (int qq = q0; qq < qe; ++qq) {
                        for (int rr = qq - 1; rr >= 0 && fabs(W[rr] - W[rr + 1]) <= 1e-3 * tnorm; --rr) {
                            double s = 0.0;
                            for (int i = lane; i < n; i += 64) s += Zl[(size_t)i * 16 + rr] * Zl[(size_t)i * 16 + qq];
                            s = wave_sum_d(s);
                            for (int i = lane; i < n; i += 64) Zl[(size_t)i * 16 + qq] -= s * Zl[(size_t)i * 16 + rr];
                        }
                        double s = 0.0;
                        for (int i = lane; i < n; i += 64) s += Zl[(size_t)i * 16 + qq] * Zl[(size_t)i * 16 + qq];
                        s = wave_sum_d(s);
                        const double inv = 1.0 / sqrt(s);
                        for (int i = lane; i < n; i += 64) Zl[(size_t)i * 16 + qq] *= inv;
                    }
                }
                __syncthreads();
            }
        }
    }
    ESTAMP(3);
    // ---------------------------------------------------------------- 4. back-transform
    // eigenvector of A = H_0 H_1 ... H_{n-3} y, applied from the last reflector;
    // one wave per vector, vectors in LDS, reflectors read from A's rows.
    for (int q = wv; q < k; q += EIG_W) {
        for (int kk = n - 3; kk >= 0; --kk) {
            const double t = tau[kk];
            if (t == 0.0) continue;
            const double* v = A + (size_t)kk * lda + kk + 1;  // v[0] = 1
            double* zc = Zl + (size_t)(kk + 1) * 16 + q;
            const int m = n - kk - 1;
            double vr[8];
            double s = 0.0;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int j = lane + 64 * u;
                vr[u] = (j < m) ? v[j] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int j = lane + 64 * u;
                if (j < m) s += vr[u] * zc[(size_t)j * 16];
            }
            for (int j = lane + 512; j < m; j += 64) s += v[j] * zc[(size_t)j * 16];
            s = wave_sum_d(s) * t;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int j = lane + 64 * u;
                if (j < m) zc[(size_t)j * 16] -= s * vr[u];
            }
            for (int j = lane + 512; j < m; j += 64) zc[(size_t)j * 16] -= s * v[j];
        }
        // deterministic sign: largest-magnitude component positive
        double best = 0.0;
        int bi = 0;
        for (int i = lane; i < n; i += 64) {
            const double a = fabs(Zl[(size_t)i * 16 + q]);
            if (a > best) {
                best = a;
                bi = i;
            }
        }
        for (int m2 = 32; m2 >= 1; m2 >>= 1) {
            const double ob = __shfl_xor(best, m2, 64);
            const int oi = __shfl_xor(bi, m2, 64);
            if (ob > best || (ob == best && oi < bi)) {
                best = ob;
                bi = oi;
            }
        }
        const double sgn = (Zl[(size_t)bi * 16 + q] < 0.0) ? -1.0 : 1.0;
        for (int i = lane; i < n; i += 64) Zl[(size_t)i * 16 + q] *= sgn;
    }
    __syncthreads();
    for (int i = tid; i < n * 16; i += EIG_T) Z[i] = ((i & 15) < k) ? Zl[i] : 0.0;
    ESTAMP(4);
}

extern "C" hipError_t scc_launch_syevx_topk(double* A, int n, int lda, int k, double* scratch, double* Z, double* W,
                                            u64* stamps, hipStream_t st)
{
    hipFuncSetAttribute((const void*)k_syevx_topk, hipFuncAttributeMaxDynamicSharedMemorySize, EIG_LDS_BYTES);
    hipLaunchKernelGGL(k_syevx_topk, dim3(1), dim3(EIG_T), EIG_LDS_BYTES, st, A, n, lda, k, scratch, Z, W, stamps);
    return hipGetLastError();
}
