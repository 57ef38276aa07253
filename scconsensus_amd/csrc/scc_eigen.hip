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

// A: n x n symmetric (full), row-major, leading dimension lda; destroyed.
// scratch doubles: 4*n + 80*n.  Z: n x 16 out.  W: k out (descending).
__global__ void __launch_bounds__(EIG_T) k_syevx_topk(double* A, int n, int lda, int k, double* scratch, double* Z,
                                                      double* W)
{
    __shared__ double red[EIG_W];
    __shared__ double sh[8];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    double* d = scratch;          // n
    double* e = d + n;            // n
    double* tau = e + n;          // n
    double* p = tau + n;          // n (symv result / w)
    double* lu = p + n;           // 5n per eigenvector (<= 16): LU factors of T - lambda I
    // ---------------------------------------------------------------- 1. tridiagonalise
    for (int kk = 0; kk < n - 2; ++kk) {
        double* rowk = A + (size_t)kk * lda;
        const int m = n - kk - 1;          // length of x = A[kk][kk+1 .. n-1]
        double part = 0.0;
        for (int i = 1 + tid; i < m; i += EIG_T) {
            const double xv = rowk[kk + 1 + i];
            part += xv * xv;
        }
        const double xnorm2 = block_sum(part, red);
        const double alpha = rowk[kk + 1];
        double taui = 0.0, beta = alpha, scal = 0.0;
        if (xnorm2 > 0.0) {
            beta = -copysign(sqrt(alpha * alpha + xnorm2), alpha);
            taui = (beta - alpha) / beta;
            scal = 1.0 / (alpha - beta);
        }
        // v stored in place: rowk[kk+1] = 1 (implicit), rowk[kk+1+i] *= scal
        __syncthreads();
        for (int i = 1 + tid; i < m; i += EIG_T) rowk[kk + 1 + i] *= scal;
        if (tid == 0) {
            d[kk] = rowk[kk];
            e[kk] = beta;
            tau[kk] = taui;
            rowk[kk + 1] = 1.0;
        }
        __syncthreads();
        if (taui != 0.0) {
            // p = taui * A22 v  (A22 = A[kk+1.., kk+1..]); one wave per row
            const double* v = rowk + kk + 1;
            for (int i = wv; i < m; i += EIG_W) {
                const double* ri = A + (size_t)(kk + 1 + i) * lda + kk + 1;
                double s = 0.0;
                for (int j = lane; j < m; j += 64) s += ri[j] * v[j];
                s = wave_sum_d(s);
                if (lane == 0) p[i] = taui * s;
            }
            __syncthreads();
            double pv = 0.0;
            for (int i = tid; i < m; i += EIG_T) pv += p[i] * v[i];
            const double dot = block_sum(pv, red);
            const double alpha2 = -0.5 * taui * dot;
            for (int i = tid; i < m; i += EIG_T) p[i] += alpha2 * v[i];
            __syncthreads();
            // A22 -= v w^T + w v^T (full square, rows stay symmetric)
            for (int i = wv; i < m; i += EIG_W) {
                double* ri = A + (size_t)(kk + 1 + i) * lda + kk + 1;
                const double vi = v[i], wi = p[i];
                for (int j = lane; j < m; j += 64) ri[j] -= vi * p[j] + wi * v[j];
            }
            __syncthreads();
        }
        // the reflector lives in rowk[kk+1..]; keep the beta in e[kk]
    }
    if (tid == 0) {
        if (n >= 2) {
            d[n - 2] = A[(size_t)(n - 2) * lda + n - 2];
            e[n - 2] = A[(size_t)(n - 2) * lda + n - 1];
            tau[n - 2] = 0.0;
        }
        d[n - 1] = A[(size_t)(n - 1) * lda + n - 1];
        e[n - 1] = 0.0;
        tau[n - 1] = 0.0;
    }
    __syncthreads();
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
        for (int iter = 0; iter < 4; ++iter) {
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
}

extern "C" hipError_t scc_launch_syevx_topk(double* A, int n, int lda, int k, double* scratch, double* Z, double* W,
                                            hipStream_t st)
{
    hipLaunchKernelGGL(k_syevx_topk, dim3(1), dim3(EIG_T), 0, st, A, n, lda, k, scratch, Z, W);
    return hipGetLastError();
}
