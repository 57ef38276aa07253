// scc_eigen.hip — top-k eigenpairs of the |U| x |U| fp64 Gram matrix.
//
// Dense symmetric eigensolver for the PCA step of stage 3 (reference:
// irlba::prcomp_irlba, R/reclusterDEConsensusFast.R:398).  The spectrum of
// the centred union-gene Gram is a few cluster "spikes" over a noise bulk, so
// the 15th/16th eigenvalues are routinely within 1e-3 relative of each other
// (SURVEY D5): iterative Krylov/subspace solvers need hundreds of steps there,
// while a direct method is exact to fp64 backward error.  One workgroup:
//   1. Householder tridiagonalisation (LAPACK dsytd2 order, lower form read
//      through the symmetric rows; trailing matrix resident in L2)
//   2. the k largest eigenvalues of T by multisection (64 Sturm counts per
//      wave per round)
//   3. eigenvectors of T by inverse iteration (dgttrf/dgttrs-style LU with
//      partial pivoting), re-orthogonalised inside eigenvalue clusters
//      (|dl| <= 1e-3 ||T||, as LAPACK dstein)
//   4. back-transformation by the stored reflectors
// Output Z[u*16 + q] = q-th largest eigenvector (q < k), zero padded to 16.
#include "scc_common.hpp"

#define EIG_T 1024
#define EIG_W (EIG_T / 64)

__device__ inline double block_sum(double v, double* red)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    double s = 0.0;
    for (int i = 0; i < EIG_W; ++i) s += red[i];  // fixed order: deterministic
    return s;
}

__device__ inline double wave_sum_d(double v)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    return v;
}

// number of eigenvalues of T (d, e) strictly below x (Sturm sequence)
__device__ inline int sturm_count(const double* d, const double* e, int n, double x, double pivmin)
{
    int c = 0;
    double q = d[0] - x;
    if (fabs(q) < pivmin) q = -pivmin;
    c += (q < 0.0);
    for (int i = 1; i < n; ++i) {
        q = d[i] - x - e[i - 1] * e[i - 1] / q;
        if (fabs(q) < pivmin) q = -pivmin;
        c += (q < 0.0);
    }
    return c;
}

// Fused pass of step k (see k_syevx_topk): rows i = 1..m-1 of the trailing
// block T (local (i,j) at T[(off+i)*ld + off+j]) are updated by the rank-2
// term of step k, and the same sweep forms p' = tau' * T' v' for step k+1.
// Output rows go to O (ld_o, off_o) — the same storage, or LDS on the switch.
template <class TP, class OP>
__device__ __forceinline__ void fused_pass(TP T, int ld, int off, OP O, int ldo, int offo, int m, const double* v,
                                           const double* w, const double* vn, double taun, double* pn)
{
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int i = 1 + wv; i < m; i += EIG_W) {
        const size_t ri = (size_t)(off + i) * ld + off;
        const size_t ro = (size_t)(offo + i - 1) * ldo + offo - 1;
        const double vi = v[i], wi = w[i];
        double s = 0.0;
        for (int j = 1 + lane; j < m; j += 64) {
            const double r = T[ri + j] - vi * w[j] - wi * v[j];
            O[ro + j] = r;
            s += r * vn[j - 1];
        }
        s = wave_sum_d(s);
        if (lane == 0) pn[i - 1] = taun * s;
    }
}

// A: n x n symmetric (full), row-major, leading dimension lda; destroyed
// (the reflectors are left in its rows).  scratch doubles: 84 n.
// Z: n x 16 out.  W: k out (descending).  Dynamic LDS: 3 n + 16 doubles plus
// an mlds x mlds tail block.
#define ESTAMP(ph)                                                          \
    do {                                                                    \
        if (stamps && threadIdx.x == 0) stamps[ph] = __builtin_amdgcn_s_memtime(); \
    } while (0)

__global__ void __launch_bounds__(EIG_T) k_syevx_topk(double* A, int n, int lda, int k, double* scratch, double* Z,
                                                      double* W, int mlds, u64* stamps)
{
    ESTAMP(0);
    extern __shared__ __attribute__((aligned(16))) double sm[];
    __shared__ double sh[8];
    double* red = sm;                 // EIG_W
    double* vb = sm + 16;             // n   current reflector v (v[0] = 1)
    double* wb = vb + n;              // n   w = p - tau/2 (p.v) v
    double* pb = wb + n;              // n   p = tau A22 v
    double* Tl = pb + n;              // mlds * mlds (LDS-resident tail)
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    double* d = scratch;          // n
    double* e = d + n;            // n
    double* tau = e + n;          // n
    double* p = tau + n;          // n (unused scratch)
    double* lu = p + n;           // 5n per eigenvector (<= 16): LU factors of T - lambda I
    (void)p;
    // ---------------------------------------------------------------- 1. tridiagonalise
    // LAPACK dsytd2 (lower) order.  Reflector k is kept in row k of A
    // (A[k][k+1] = 1, A[k][k+2..] = v tail) for the back-transformation.
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
        // reflector 0 from row 0
        {
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
            for (int j = tid; j < m; j += EIG_T) vb[j] = (j == 0) ? 1.0 : A[1 + j] * scal;
            __syncthreads();
            for (int j = tid; j < m; j += EIG_T) A[1 + j] = vb[j];
            if (tid == 0) {
                d[0] = A[0];
                e[0] = beta;
                tau[0] = t;
                sh[0] = t;
            }
            __syncthreads();
            // p = tau A22 v
            const double tt = sh[0];
            for (int i = wv; i < m; i += EIG_W) {
                const double* ri = A + (size_t)(1 + i) * lda + 1;
                double s = 0.0;
                for (int j = lane; j < m; j += 64) s += ri[j] * vb[j];
                s = wave_sum_d(s);
                if (lane == 0) pb[i] = tt * s;
            }
            __syncthreads();
        }
        bool in_lds = false;
        int lds_base = 0, lds_ld = 0;  // step index at the switch, LDS leading dimension
        for (int kk = 0; kk <= n - 3; ++kk) {
            const int m = n - kk - 1;  // trailing block A22 = rows/cols kk+1 .. n-1
            const double t = sh[0];
            // w = p - tau/2 (p.v) v
            double pv = 0.0;
            for (int i = tid; i < m; i += EIG_T) pv += pb[i] * vb[i];
            const double dot = block_sum(pv, red);
            const double a2 = -0.5 * t * dot;
            for (int i = tid; i < m; i += EIG_T) wb[i] = (t != 0.0) ? pb[i] + a2 * vb[i] : 0.0;
            __syncthreads();
            // locate row 0 of A22 (global row kk+1)
            const double* row0;
            int off0, ld0;
            if (in_lds) {
                off0 = kk + 1 - lds_base;
                ld0 = lds_ld;
                row0 = Tl + (size_t)off0 * ld0 + off0;
            } else {
                off0 = kk + 1;
                ld0 = lda;
                row0 = A + (size_t)off0 * ld0 + off0;
            }
            // updated row 0: x_j = A22[0][j] - v0 w_j - w0 v_j
            const double v0 = vb[0], w0 = wb[0];
            if (kk == n - 3) {  // 2 x 2 remainder
                if (tid == 0) {
                    const double a00 = row0[0] - 2.0 * v0 * w0;
                    const double a01 = row0[1] - v0 * wb[1] - w0 * vb[1];
                    const double* row1 = row0 + ld0;
                    const double a11 = row1[1] - 2.0 * vb[1] * wb[1];
                    d[n - 2] = a00;
                    e[n - 2] = a01;
                    d[n - 1] = a11;
                    e[n - 1] = 0.0;
                    tau[n - 2] = 0.0;
                    tau[n - 1] = 0.0;
                }
                break;
            }
            double part = 0.0;
            for (int j = 2 + tid; j < m; j += EIG_T) {
                const double x = row0[j] - v0 * wb[j] - w0 * vb[j];
                part += x * x;
            }
            const double xn2 = block_sum(part, red);
            const double alpha = row0[1] - v0 * wb[1] - w0 * vb[1];
            double tn = 0.0, beta = alpha, scal = 0.0;
            if (xn2 > 0.0) {
                beta = -copysign(sqrt(alpha * alpha + xn2), alpha);
                tn = (beta - alpha) / beta;
                scal = 1.0 / (alpha - beta);
            }
            // v' (length m-1) reuses p's LDS buffer: p of step kk is consumed (w formed)
            double* vn = pb;
            for (int j = 1 + tid; j < m; j += EIG_T) {
                const double x = row0[j] - v0 * wb[j] - w0 * vb[j];
                vn[j - 1] = (j == 1) ? 1.0 : x * scal;
            }
            if (tid == 0) {
                d[kk + 1] = row0[0] - 2.0 * v0 * w0;
                e[kk + 1] = beta;
                tau[kk + 1] = tn;
            }
            __syncthreads();
            double* refl = A + (size_t)(kk + 1) * lda + kk + 2;
            for (int j = tid; j < m - 1; j += EIG_T) refl[j] = vn[j];
            // fused pass: rows 1..m-1 of A22 updated (v, w read), p' to scratch
            double* pn = lu;  // free until the inverse iteration
            const int mn = m - 1;
            if (!in_lds && mn <= mlds) {
                // switch: the updated trailing block is written to LDS
                fused_pass(A, lda, kk + 1, Tl, mn, 0, m, vb, wb, vn, tn, pn);
                in_lds = true;
                lds_base = kk + 2;
                lds_ld = mn;
            } else if (in_lds) {
                const int o = kk + 1 - lds_base;
                fused_pass(Tl, lds_ld, o, Tl, lds_ld, o + 1, m, vb, wb, vn, tn, pn);
            } else {
                fused_pass(A, lda, kk + 1, A, lda, kk + 2, m, vb, wb, vn, tn, pn);
            }
            __syncthreads();
            // next step: v <- v', p <- p'
            for (int j = tid; j < mn; j += EIG_T) {
                vb[j] = vn[j];
                pb[j] = pn[j];
            }
            if (tid == 0) sh[0] = tn;
            __syncthreads();
        }
    }
    __syncthreads();
    ESTAMP(1);
    // ---------------------------------------------------------------- 2. eigenvalues
    // Gershgorin bounds, pivmin as LAPACK dstebz
    if (tid == 0) {
        double gl = d[0], gu = d[0], emax2 = 0.0, tnorm = 0.0;
        for (int i = 0; i < n; ++i) {
            const double r = (i > 0 ? fabs(e[i - 1]) : 0.0) + (i < n - 1 ? fabs(e[i]) : 0.0);
            gl = fmin(gl, d[i] - r);
            gu = fmax(gu, d[i] + r);
            if (i < n - 1) emax2 = fmax(emax2, e[i] * e[i]);
        }
        tnorm = fmax(fabs(gl), fabs(gu));
        const double eps = 2.220446049250313e-16;
        gl -= 2.0 * tnorm * eps * n + 1e-300;
        gu += 2.0 * tnorm * eps * n + 1e-300;
        sh[0] = gl;
        sh[1] = gu;
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
            const int c = sturm_count(d, e, n, x, pivmin);
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
    // Each wave factors T - lambda_q I (dgttrf order, partial pivoting) for its
    // q and solves; between solves wave 0 re-orthogonalises cluster members
    // (|lambda_r - lambda_{r+1}| <= 1e-3 ||T||, as LAPACK dstein) and normalises.
    // y_q lives in Z[u*16 + q].
    {
        const double eps = 2.220446049250313e-16;
        const double tiny = eps * tnorm + 1e-300;
        for (int q = wv; q < k; q += EIG_W) {
            double* dd = lu + (size_t)q * 5 * n;
            double* du = dd + n;
            double* du2 = du + n;
            double* dl = du2 + n;
            double* piv = dl + n;
            const double lam = W[q];
            if (lane == 0) {
                for (int i = 0; i < n; ++i) {
                    dd[i] = d[i] - lam;
                    du[i] = (i < n - 1) ? e[i] : 0.0;
                    dl[i] = (i < n - 1) ? e[i] : 0.0;
                    du2[i] = 0.0;
                    piv[i] = 0.0;
                }
                for (int i = 0; i < n - 1; ++i) {
                    if (fabs(dd[i]) >= fabs(dl[i])) {
                        if (dd[i] == 0.0) dd[i] = tiny;
                        const double f = dl[i] / dd[i];
                        dl[i] = f;
                        dd[i + 1] -= f * du[i];
                    } else {
                        const double f = dd[i] / dl[i];
                        dd[i] = dl[i];
                        dl[i] = f;
                        const double t = du[i];
                        du[i] = dd[i + 1];
                        dd[i + 1] = t - f * dd[i + 1];
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
                Z[(size_t)i * 16 + q] = 0.5 + (double)(h & 0xffff) / 65536.0;
            }
        }
        __threadfence_block();
        __syncthreads();
        for (int iter = 0; iter < 3; ++iter) {
            for (int q = wv; q < k; q += EIG_W) {
                if (lane == 0) {
                    const double* dd = lu + (size_t)q * 5 * n;
                    const double* du = dd + n;
                    const double* du2 = du + n;
                    const double* dl = du2 + n;
                    const double* piv = dl + n;
                    double* b = Z + q;  // stride 16
                    for (int i = 0; i < n - 1; ++i) {
                        if (piv[i] == 0.0) {
                            b[(size_t)(i + 1) * 16] -= dl[i] * b[(size_t)i * 16];
                        } else {
                            const double t = b[(size_t)i * 16];
                            b[(size_t)i * 16] = b[(size_t)(i + 1) * 16];
                            b[(size_t)(i + 1) * 16] = t - dl[i] * b[(size_t)i * 16];
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
            }
            __threadfence_block();
            __syncthreads();
            if (wv == 0) {
                for (int q = 0; q < k; ++q) {
                    for (int r = q - 1; r >= 0 && fabs(W[r] - W[r + 1]) <= 1e-3 * tnorm; --r) {
                        double s = 0.0;
                        for (int i = lane; i < n; i += 64) s += Z[(size_t)i * 16 + r] * Z[(size_t)i * 16 + q];
                        s = wave_sum_d(s);
                        for (int i = lane; i < n; i += 64) Z[(size_t)i * 16 + q] -= s * Z[(size_t)i * 16 + r];
                    }
                    double s = 0.0;
                    for (int i = lane; i < n; i += 64) s += Z[(size_t)i * 16 + q] * Z[(size_t)i * 16 + q];
                    s = wave_sum_d(s);
                    const double inv = 1.0 / sqrt(s);
                    for (int i = lane; i < n; i += 64) Z[(size_t)i * 16 + q] *= inv;
                }
            }
            __threadfence_block();
            __syncthreads();
        }
    }
    ESTAMP(3);
    // ---------------------------------------------------------------- 4. back-transform
    // eigenvector of A = H_0 H_1 ... H_{n-3} y; apply from the last reflector.
    // One wave per vector q.
    for (int q = wv; q < k; q += EIG_W) {
        for (int kk = n - 3; kk >= 0; --kk) {
            const double t = tau[kk];
            if (t == 0.0) continue;
            const double* v = A + (size_t)kk * lda + kk + 1;  // v[0] = 1
            const int m = n - kk - 1;
            double s = 0.0;
            for (int j = lane; j < m; j += 64) s += v[j] * Z[(size_t)(kk + 1 + j) * 16 + q];
            s = wave_sum_d(s) * t;
            for (int j = lane; j < m; j += 64) Z[(size_t)(kk + 1 + j) * 16 + q] -= s * v[j];
        }
        // deterministic sign: largest-magnitude component positive
        double best = 0.0;
        int bi = 0;
        for (int i = lane; i < n; i += 64) {
            const double a = fabs(Z[(size_t)i * 16 + q]);
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
        const double sgn = (Z[(size_t)bi * 16 + q] < 0.0) ? -1.0 : 1.0;
        for (int i = lane; i < n; i += 64) Z[(size_t)i * 16 + q] *= sgn;
    }
    __syncthreads();
    for (int i = tid; i < n * 16; i += EIG_T)
        if ((i & 15) >= k) Z[i] = 0.0;
    ESTAMP(4);
}

extern "C" hipError_t scc_launch_syevx_topk(double* A, int n, int lda, int k, double* scratch, double* Z, double* W,
                                            u64* stamps, hipStream_t st)
{
    // LDS: red(16) + v, w, p (3n) + the largest square tail that fits in 156 KiB
    const size_t budget = 156 * 1024;
    const size_t fixed = sizeof(double) * (16 + 3 * (size_t)n);
    if (fixed > budget) return hipErrorInvalidValue;
    int mlds = (int)floor(sqrt((double)(budget - fixed) / sizeof(double)));
    if (mlds > n) mlds = n;
    const size_t lds = fixed + sizeof(double) * (size_t)mlds * mlds;
    hipFuncSetAttribute((const void*)k_syevx_topk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k_syevx_topk, dim3(1), dim3(EIG_T), lds, st, A, n, lda, k, scratch, Z, W, mlds, stamps);
    return hipGetLastError();
}
