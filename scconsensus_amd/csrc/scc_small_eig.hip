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
#include <cstdio>
#include <mutex>

// phase stamps of the last k_small_syev (s_memtime at the start of each phase;
// diagnostic, read by scc_diag_small_syev_stamps)
__device__ u64 g_se_stamps[8];

extern "C" size_t scc_small_syev_lds_bytes() { return sizeof(double) * SE_LDS_TOTAL; }

__global__ void __launch_bounds__(SE_T) k_small_syev(const double* __restrict__ H, int n, int ldh, int k,
                                                    double* __restrict__ Y, double* __restrict__ theta,
                                                    u32* __restrict__ flag)
{
    extern __shared__ __attribute__((aligned(16))) double sm[];
    se_syev<false>([=](int i, int j) { return H[(size_t)i * ldh + j]; }, n, k, Y, theta, flag, sm, g_se_stamps);
}

// the dynamic-LDS attribute, set once per process before any launch or capture
extern "C" void scc_small_syev_prepare()
{
    static std::once_flag once;
    std::call_once(once, [] {
        (void)scc_set_lds((const void*)k_small_syev, (int)scc_small_syev_lds_bytes());
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
__device__ u64 g_cb_stamps[32];  // diagnostic: k_fsi_cholinv_blk phase stamps (SCC_FSI_CHOL_STAMPS=1)
__global__ void __launch_bounds__(256) k_fsi_cholinv_blk(const double* __restrict__ G, double shift_rel,
                                                        double* __restrict__ T, u32* __restrict__ flag,
                                                        u64* __restrict__ st)
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
    fsi_cholinv_blk(A, X, Ri, &s_bad, st);
    if (st && threadIdx.x == 0) st[31] = __builtin_amdgcn_s_memtime();
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
    if (cholinv_variant()) {
        u64* stp = nullptr;
        const char* e = getenv("SCC_FSI_CHOL_STAMPS");
        if (e && *e == '1') {
            void* sp = nullptr;
            if (hipGetSymbolAddress(&sp, HIP_SYMBOL(g_cb_stamps)) == hipSuccess) stp = (u64*)sp;
        }
        hipLaunchKernelGGL(k_fsi_cholinv_blk, dim3(1), dim3(256), 0, st, G, shift_rel, T, flag, stp);
    }
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
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    const char* e = getenv("SCC_FSI_CHOL_STAMPS");
    if (e && *e == '1') {
        u64 h[32];
        if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_cb_stamps), sizeof(h)) == hipSuccess) {
            fprintf(stderr, "[scc chol stamps] cycles from start:");
            for (int i = 1; i < 14; ++i) fprintf(stderr, " %llu", (unsigned long long)(h[i] - h[0]));
            fprintf(stderr, " end %llu\n", (unsigned long long)(h[31] - h[0]));
        }
    }
    return 0;
}

extern "C" SCC_API int scc_diag_small_syev_stamps(unsigned long long* out)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_se_stamps), sizeof(u64) * 8) == hipSuccess ? 0 : 1;
}
