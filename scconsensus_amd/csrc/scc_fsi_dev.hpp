// scc_fsi_dev.hpp — device helpers shared by the filtered subspace iteration's
// kernels (scc_small_eig.hip: the launch-per-step path; scc_subspace.hip: the
// persistent engine): the wave readlane / sum of fp64 values and the blocked
// 64 x 64 Cholesky + inverse on one workgroup.
#pragma once
#include "scc_common.hpp"

typedef double d4 __attribute__((ext_vector_type(4)));  // one fp64 MFMA 16x16x4 accumulator

// hand-off accessors (MI355X_MICROARCH.md valid form row 1): every handed-off
// double is stored and loaded sc1 (8-byte agent-scope relaxed atomics)
__device__ __forceinline__ double fx_ld(const double* p)
{
    return __longlong_as_double(
        (long long)__hip_atomic_load((const u64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void fx_st(double* p, double v)
{
    __hip_atomic_store((u64*)p, (u64)__double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// sum over t < count of p[t * stride] in t order; the loads (sc1: a round trip
// to memory each) are issued 8 at a time, with no branch between them
__device__ __forceinline__ double fx_sum(const double* p, size_t stride, int count)
{
    double s = 0.0;
    for (int t0 = 0; t0 < count; t0 += 8) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = fx_ld(p + (size_t)min(t0 + u, count - 1) * stride);
#pragma unroll
        for (int u = 0; u < 8; ++u) s = (t0 + u < count) ? s + v[u] : s;
    }
    return s;
}


__device__ inline double se_wave_sum(double v)
{
    v += scc_xor_lane_f64<32>(v);
    v += scc_xor_lane_f64<16>(v);
    v += scc_xor_lane_f64<8>(v);
    v += scc_xor_lane_f64<4>(v);
    v += scc_xor_lane_f64<2>(v);
    return v + scc_xor_lane_f64<1>(v);
}
// uniform value of lane l (compile-time or wave-uniform) of a lane-varying double
__device__ __forceinline__ double se_readlane(double x, int l)
{
    const u64 b = (u64)__double_as_longlong(x);
    const u32 lo = (u32)__builtin_amdgcn_readlane((int)(u32)b, l);
    const u32 hi = (u32)__builtin_amdgcn_readlane((int)(u32)(b >> 32), l);
    return __longlong_as_double((long long)(((u64)hi << 32) | lo));
}

// ---------------------------------------------------------------------------
// Blocked Cholesky + inverse of a 64 x 64 SPD matrix by one 256-thread
// workgroup, in LDS (row stride CB_S): the one-wave kernel (k_fsi_cholinv64) spends
// its time on a 64-step chain whose every step waits for a full-width update; here
// the chain is four 16-column panels and everything else is fp64 MFMA.
//   panel K (wave 0, lane = row 16K + lane, the panel's 16 columns in
//     registers): 16 steps of pivot readlane, rsq + Newton, column scale, and
//     the update of the panel's later columns from readlane broadcasts of the
//     diagonal rows' multipliers; L overwrites A in place.
//   trailing update A_IJ -= L_IK L_JK^T (K < J <= I), 4 MFMA 16x16x4 per block,
//     blocks dealt over the 4 waves.
//   inverse X = L^{-1}: the diagonal blocks by forward substitution (wave I for
//     block I, lane = column, 1 / L_ii from the panel's rsq), then the block
//     levels X_IJ = -X_II (sum_{J <= M < I} L_IM X_MJ) on MFMA.
// *bad |= 1 when a pivot is not positive.  A holds L afterwards (lower), X = L^{-1}.
#define CB_S 66  // LDS row stride (doubles)
__device__ __forceinline__ d4 cb_mfma(double a, double b, d4 c)
{
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// acc += sign * P(16x16 block at (pi, pj) of A-array Pa) * Qt, where the B operand
// is Q^T of the block (qi, qj) of Qa when qtrans, else the block itself
template <bool QT>
__device__ __forceinline__ d4 cb_block_mm(const double* Pa, int pi, int pj, const double* Qa, int qi, int qj,
                                          double sgn, d4 acc)
{
    const int lane = threadIdx.x & 63, i = lane & 15, kk = lane >> 4;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const double a = Pa[(16 * pi + i) * CB_S + 16 * pj + 4 * s + kk];
        // B[k][j]: QT: Q^T[k][j] = Q[16 qi + j][16 qj + k];  else Q[16 qi + k][16 qj + j]
        const double b = QT ? Qa[(16 * qi + i) * CB_S + 16 * qj + 4 * s + kk] : Qa[(16 * qi + 4 * s + kk) * CB_S + 16 * qj + i];
        acc = cb_mfma(sgn * a, b, acc);
    }
    return acc;
}

__device__ __forceinline__ void cb_store(double* Pa, int bi, int bj, d4 acc)
{
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int r = 0; r < 4; ++r) Pa[(16 * bi + (lane >> 4) + 4 * r) * CB_S + 16 * bj + (lane & 15)] = acc[r];
}
__device__ __forceinline__ d4 cb_load(const double* Pa, int bi, int bj)
{
    const int lane = threadIdx.x & 63;
    d4 acc;
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] = Pa[(16 * bi + (lane >> 4) + 4 * r) * CB_S + 16 * bj + (lane & 15)];
    return acc;
}

// A: [64][CB_S] SPD on entry (lower part read; its upper blocks (0, 1..3) are the
// level scratch); X: [64][CB_S] out; Ri: [64] scratch.  Every thread of the
// 256-thread workgroup calls it.
// every lane gets the value of lane 16 r + C (r: its own 16-lane row): DPP
// row_newbcast, one VALU move per 32 bits, no SGPR round trip
template <int C>
__device__ __forceinline__ double cb_bcast_c(double x)
{
    return __builtin_amdgcn_mov_dpp(x, 0x150 | C, 0xf, 0xf, true);  // one v_mov_b64_dpp
}
__device__ __forceinline__ double cb_bcast(double x, int c)  // c: a constant after unrolling
{
    switch (c) {
    case 0: return cb_bcast_c<0>(x);
    case 1: return cb_bcast_c<1>(x);
    case 2: return cb_bcast_c<2>(x);
    case 3: return cb_bcast_c<3>(x);
    case 4: return cb_bcast_c<4>(x);
    case 5: return cb_bcast_c<5>(x);
    case 6: return cb_bcast_c<6>(x);
    case 7: return cb_bcast_c<7>(x);
    case 8: return cb_bcast_c<8>(x);
    case 9: return cb_bcast_c<9>(x);
    case 10: return cb_bcast_c<10>(x);
    case 11: return cb_bcast_c<11>(x);
    case 12: return cb_bcast_c<12>(x);
    case 13: return cb_bcast_c<13>(x);
    case 14: return cb_bcast_c<14>(x);
    default: return cb_bcast_c<15>(x);
    }
}

// X_KK = L_KK^{-1} of diagonal block K (in A) into X, by one wave: lane l
// holds row i = l & 15 of L_KK; lane j = l & 15 forms column j of the inverse,
// w_r = (delta_rj - sum_{m<r} L_rm w_m) / L_rr, L_rm broadcast within 16 lanes
__device__ __forceinline__ void cb_diag_inverse(const double* A, double* X, const double* Ri, int K)
{
    const int lane = threadIdx.x & 63, i = lane & 15, j = i;
    double a[16], gk[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) {
        a[c] = A[(16 * K + i) * CB_S + 16 * K + c];
        gk[c] = Ri[16 * K + c];
    }
    double w[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        double sacc = (r == j) ? 1.0 : 0.0;
#pragma unroll
        for (int m = 0; m < r; ++m) sacc = fma(-cb_bcast(a[m], r), w[m], sacc);
        w[r] = (r >= j) ? sacc * gk[r] : 0.0;
    }
    if (lane < 16) {
#pragma unroll
        for (int r = 0; r < 16; ++r) X[(16 * K + r) * CB_S + 16 * K + j] = w[r];
    }
}

__device__ inline void fsi_cholinv_blk(double* A, double* X, double* Ri, int* s_bad, u64* st = nullptr)
{
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    int ns = 0;
    auto stamp = [&]() {
        if (st && tid == 0) st[ns] = __builtin_amdgcn_s_memtime();
        ++ns;
    };
    stamp();
#pragma unroll
    for (int K = 0; K < 4; ++K) {
        // (a) wave 0: block column K in one 16-step chain.  Lane l: c = l & 15,
        // r = l >> 4; every 16-lane row keeps a copy of diagonal row 16K + c (so
        // the multipliers L[16K + c][k] are a row_newbcast away in every row),
        // and rows r >= 1 also carry panel row 16(K + r) + c below the block
        if (wv == 0) {
            const int c = lane & 15, r = lane >> 4;
            const int brow = 16 * (K + r) + c;
            const bool below = r >= 1 && K + r < 4;
            double d[16], bl[16], gk[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                d[q] = A[(16 * K + c) * CB_S + 16 * K + q];
                bl[q] = A[min(brow, 63) * CB_S + 16 * K + q];
            }
            bool bad = false;
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const double pv = cb_bcast(d[k], k);
                bad |= !(pv > 0.0);
                const double dd = pv > 0.0 ? pv : 1.0;
                double g = __builtin_amdgcn_rsq(dd);
                g = g * fma(-0.5 * dd * g, g, 1.5);
                gk[k] = g;
                const double ld = (c > k) ? d[k] * g : (c == k ? dd * g : 0.0);
                const double lb = bl[k] * g;
                d[k] = ld;
                bl[k] = lb;
#pragma unroll
                for (int q = k + 1; q < 16; ++q) {
                    const double m = cb_bcast(ld, q);  // L[16K + q][k]
                    d[q] = fma(-ld, m, d[q]);
                    bl[q] = fma(-lb, m, bl[q]);
                }
            }
            if (lane < 16) {
#pragma unroll
                for (int q = 0; q < 16; ++q) A[(16 * K + c) * CB_S + 16 * K + q] = (c >= q) ? d[q] : 0.0;
            }
            if (below) {
#pragma unroll
                for (int q = 0; q < 16; ++q) A[brow * CB_S + 16 * K + q] = bl[q];
            }
            if (lane == 0) {
#pragma unroll
                for (int k = 0; k < 16; ++k) Ri[16 * K + k] = gk[k];
            }
            if (bad && lane == 0) *s_bad = 1;
        }
        __syncthreads();
        stamp();
        // (b) wave 1: the inverse of the diagonal block (needed by the levels only);
        // wave 0: the next block column's trailing update (look-ahead: it goes
        // straight on to factor it); waves 2, 3: the other trailing blocks
        if (wv == 1) cb_diag_inverse(A, X, Ri, K);
        int b = 0;
#pragma unroll
        for (int J = K + 1; J < 4; ++J)
#pragma unroll
            for (int I = J; I < 4; ++I) {
                bool mine;
                if (J == K + 1) {
                    mine = wv == 0;
                } else {
                    mine = (b & 1) + 2 == wv;
                    ++b;
                }
                if (!mine) continue;
                d4 acc = cb_load(A, I, J);
                acc = cb_block_mm<true>(A, I, K, A, J, K, -1.0, acc);
                cb_store(A, I, J, acc);
            }
    }
    __syncthreads();
    stamp();
    // the zero blocks above the diagonal of X
    if (lane < 16) {
#pragma unroll
        for (int J = 0; J < 4; ++J)
            if (J > wv) {
#pragma unroll
                for (int r = 0; r < 16; ++r) X[(16 * wv + r) * CB_S + 16 * J + lane] = 0.0;
            }
    }
    __syncthreads();
    // levels d = I - J = 1, 2, 3: S = sum_{J <= M < I} L_IM X_MJ (wave w: block J = w),
    // then X_IJ = -X_II S
#pragma unroll
    for (int d = 1; d < 4; ++d) {
        const int J = wv, I = J + d;
        double* Sw = A + 16 * (wv + 1);  // upper block (0, wv + 1): free once L is formed
        if (I < 4) {
            d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int M = J; M < I; ++M) acc = cb_block_mm<false>(A, I, M, X, M, J, 1.0, acc);
            cb_store(Sw, 0, 0, acc);
        }
        __syncthreads();
        if (I < 4) {
            d4 x = {0.0, 0.0, 0.0, 0.0};
            x = cb_block_mm<false>(X, I, I, Sw, 0, 0, -1.0, x);
            cb_store(X, I, J, x);
        }
        __syncthreads();
    }
}


// ---------------------------------------------------------------------------
// top-k eigenpairs of a symmetric matrix of order <= 64 on one workgroup
// (k_small_syev; the persistent engine's Rayleigh-Ritz step)
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

// dynamic LDS of k_small_syev (doubles)
#define SE_LUS (5 * SE_N + 2)                   // per-eigenpair LU stride (padded: lanes on distinct banks)
#define SE_YS (SE_N + 2)                        // tridiagonal eigenvector stride (padded likewise)
#define SE_LDS_V 0                              // [64][64] reflector i in row i
#define SE_LDS_LU (SE_LDS_V + SE_N * SE_N)      // [16][SE_LUS] LU factors per eigenpair
#define SE_LDS_Y (SE_LDS_LU + SE_MAXK * SE_LUS) // [16][SE_YS] tridiagonal eigenvectors
#define SE_LDS_VEC (SE_LDS_Y + SE_MAXK * SE_YS)   // [8][64] d, e, e^2, tau, p, v, column, row sums
#define SE_LDS_SML (SE_LDS_VEC + 8 * SE_N)        // [3][16] theta, brackets; [4] Gershgorin
#define SE_LDS_CNT (SE_LDS_SML + 3 * SE_MAXK + 4) // [256] int counts (+ the bad flag)
#define SE_LDS_TOTAL (SE_LDS_CNT + (SE_T + 2) / 2)

// H: n x n (ldh, n <= 64), symmetrised on load; k <= min(16, n) wanted.
// Y[r * 16 + q]: the q-th largest eigenvector (q < k; columns k..15 zero),
// theta[q] its Rayleigh quotient.  The matrix is always reduced as 64 x 64:
// rows and columns >= n become a decoupled diagonal block at a value below
// every eigenvalue (-(max row sum) - 1), so the top k are those of H and every
// loop has a compile-time length.  The matrix lives in registers, thread (r,
// q) holding row r, columns q + 4u.  flag |= 16 when a value is not finite or
// a cluster's vectors are dependent.
// One 256-thread workgroup; hload(i, j) = H[i][j]; sm: SE_LDS_TOTAL doubles of
// LDS; SC1: Y and theta are handed off to other workgroups (sc1 stores);
// stamps: phase s_memtime stamps (nullptr: none).
template <bool SC1, class HL>
__device__ __attribute__((always_inline)) void se_syev(HL hload, int n, int k, double* __restrict__ Y, double* __restrict__ theta,
                        u32* __restrict__ flag, double* sm, u64* stamps)
{
    double(*Vr)[SE_N] = (double(*)[SE_N])(sm + SE_LDS_V);
    double* LU = sm + SE_LDS_LU;
    double(*Yt)[SE_YS] = (double(*)[SE_YS])(sm + SE_LDS_Y);
    double* dg = sm + SE_LDS_VEC;
    double* eo = dg + SE_N;
    double* e2 = eo + SE_N;
    double* ta = e2 + SE_N;
    double* pv = ta + SE_N;
    double* vc = pv + SE_N;
    double* colv = vc + SE_N;
    double* rsum = colv + SE_N;
    double* th = sm + SE_LDS_SML;
    double* blo = th + SE_MAXK;
    double* bhi = blo + SE_MAXK;
    double* gsc = bhi + SE_MAXK;
    int* cnt = (int*)(sm + SE_LDS_CNT);
    int& s_bad = cnt[SE_T];
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
            h1[u] = hload(rc, cc);
            h2[u] = hload(cc, rc);
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
    if (tid == 0 && stamps) stamps[0] = __builtin_amdgcn_s_memtime();
    // ---- tridiagonalisation (LAPACK dsytd2 order) by ONE wave, lane r holding
    // row r of the matrix in registers: no workgroup barrier per column (the
    // 4-thread-per-row version spent ~1.1 us a column on three of them).
    // Column i: reflector from the lanes below the diagonal (one wave sum),
    // v to LDS and back as broadcasts, p = tau A v (4 partial sums), w, and the
    // rank-2 update of the trailing columns.  The matrix is staged through the
    // LU region (row stride 65: a lane per row without bank conflicts).
    {
        double* Ms = LU;  // [64][65], dead until the inverse iteration
#pragma unroll
        for (int u = 0; u < 16; ++u) Ms[r * 65 + q + 4 * u] = a[u];
    }
    __syncthreads();
    if (wv == 0) {
        const double* Ms = LU;
        double am[SE_N];
#pragma unroll
        for (int j = 0; j < SE_N; ++j) am[j] = Ms[lane * 65 + j];
        double* wbuf = pv;  // w of the current column
#pragma unroll
        for (int i = 0; i < SE_N - 2; ++i) {
            const double dii = se_readlane(am[i], i);  // (not "lane == i ? am[i]": that becomes am[lane])
            if (lane == 0) dg[i] = dii;
            const double x = (lane > i) ? am[i] : 0.0;
            const double alpha = se_readlane(am[i], i + 1);
            const double sq = se_wave_sum((lane > i + 1) ? x * x : 0.0);
            double beta = alpha, t = 0.0, scal = 0.0;
            if (sq > 0.0) {
                beta = -copysign(sqrt(alpha * alpha + sq), alpha);
                t = (beta - alpha) / beta;
                scal = 1.0 / (alpha - beta);
            }
            const double v = (lane == i + 1) ? 1.0 : ((lane > i + 1) ? x * scal : 0.0);
            Vr[i][lane] = v;
            if (lane == 0) {
                eo[i] = beta;
                ta[i] = t;
            }
            // p = tau A v over the trailing columns (v_j broadcast from LDS)
            double p4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int j = i + 1; j < SE_N; ++j) p4[(j - i - 1) & 3] = fma(am[j], Vr[i][j], p4[(j - i - 1) & 3]);
            const double p = t * ((p4[0] + p4[1]) + (p4[2] + p4[3]));
            const double K = -0.5 * t * se_wave_sum((lane > i) ? p * v : 0.0);
            const double w = (lane > i) ? fma(K, v, p) : 0.0;
            wbuf[lane] = w;
            // A22 -= v w^T + w v^T (rows <= i have v = w = 0: unchanged)
#pragma unroll
            for (int j = i + 1; j < SE_N; ++j) am[j] = fma(-v, wbuf[j], fma(-w, Vr[i][j], am[j]));
        }
        const double d62 = se_readlane(am[SE_N - 2], SE_N - 2), e62 = se_readlane(am[SE_N - 2], SE_N - 1);
        const double d63 = se_readlane(am[SE_N - 1], SE_N - 1);
        if (lane == 0) {
            dg[SE_N - 2] = d62;
            eo[SE_N - 2] = e62;
            dg[SE_N - 1] = d63;
            eo[SE_N - 1] = 0.0;
            ta[SE_N - 2] = 0.0;
            ta[SE_N - 1] = 0.0;
        }
    }
    __syncthreads();
    if (tid == 0 && stamps) stamps[1] = __builtin_amdgcn_s_memtime();
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
    if (tid == 0 && stamps) stamps[2] = __builtin_amdgcn_s_memtime();
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
    if (tid == 0 && stamps) stamps[3] = __builtin_amdgcn_s_memtime();
    // ---- inverse iteration: eigenpair q on lane q of wave 0 (LU with partial
    // pivoting of T - lambda I, two solves from a pseudo-random start)
    if (wv == 0 && lane < k) {
        const int qq = lane;
        const double lam = 0.5 * (blo[qq] + bhi[qq]);
        double* fdr = LU + (size_t)qq * SE_LUS;  // 1 / U diagonal
        double* fu = fdr + SE_N;
        double* fu2 = fu + SE_N;
        double* fl = fu2 + SE_N;
        double* y = Yt[qq];
        const double tiny = kSeEps * tnorm + 1e-300;
        // (LDS operands staged in registers 8 steps at a time: a load behind a
        // store of the same array would otherwise wait at every step)
        double dcur = dg[0] - lam, ucur = eo[0];
        u64 pmask = 0;
#pragma unroll
        for (int i0 = 0; i0 < SE_N - 1; i0 += 8) {
            double ev[9], dv[8];
#pragma unroll
            for (int u = 0; u < 9; ++u) ev[u] = eo[min(i0 + u, SE_N - 1)];
#pragma unroll
            for (int u = 0; u < 8; ++u) dv[u] = dg[min(i0 + u + 1, SE_N - 1)];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int i = i0 + u;
                if (i >= SE_N - 1) break;  // compile-time
                const double li = ev[u], dn = dv[u] - lam, un = (i < SE_N - 2) ? ev[u + 1] : 0.0;
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
                pmask |= (u64)(piv ? 1 : 0) << i;
                dcur = fma(-f, ua, ub);
                ucur = piv ? -f * un : un;
            }
        }
        if (dcur == 0.0) dcur = tiny;
        fdr[SE_N - 1] = 1.0 / dcur;
        fu[SE_N - 1] = 0.0;
        fu2[SE_N - 1] = 0.0;
        // the iterate in LDS (this lane's row of Yt)
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
            for (int i0 = 0; i0 < SE_N - 1; i0 += 8) {
                double yv[8], lv[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    yv[u] = y[min(i0 + u + 1, SE_N - 1)];
                    lv[u] = fl[min(i0 + u, SE_N - 2)];
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int i = i0 + u;
                    if (i >= SE_N - 1) break;
                    const bool piv = (pmask >> i) & 1;
                    const double bn = yv[u];
                    const double xa = piv ? bn : bi, xb = piv ? bi : bn;
                    yv[u] = xa;  // (the new y[i])
                    bi = fma(-lv[u], xa, xb);
                }
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (i0 + u < SE_N - 1) y[i0 + u] = yv[u];
            }
            y[SE_N - 1] = bi;
            double z1 = 0.0, z2 = 0.0;  // y <- U^-1 y from the bottom
#pragma unroll
            for (int i1 = SE_N - 1; i1 >= 0; i1 -= 8) {
                double yv[8], a1[8], a2[8], dr[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int i = i1 - u;
                    yv[u] = y[i];
                    a1[u] = fu[i];
                    a2[u] = fu2[i];
                    dr[u] = fdr[i];
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const double z0 = fma(-a1[u], z2, fma(-a2[u], z1, yv[u])) * dr[u];
                    yv[u] = z0;
                    z1 = z2;
                    z2 = z0;
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) y[i1 - u] = yv[u];
            }
            double mx = 0.0, sacc = 0.0;
#pragma unroll
            for (int i = 0; i < SE_N; ++i) mx = fmax(mx, fabs(y[i]));
            const double sc = (mx > 0.0 && mx < INFINITY) ? 1.0 / mx : 1.0;
#pragma unroll
            for (int i = 0; i < SE_N; ++i) sacc = fma(y[i] * sc, y[i] * sc, sacc);
            const double inv = sc / sqrt(sacc);
#pragma unroll
            for (int i0 = 0; i0 < SE_N; i0 += 16) {
                double yv[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) yv[u] = y[i0 + u];
#pragma unroll
                for (int u = 0; u < 16; ++u) y[i0 + u] = yv[u] * inv;
            }
        }
    }
    __syncthreads();
    if (tid == 0 && stamps) stamps[4] = __builtin_amdgcn_s_memtime();
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
    if (tid == 0 && stamps) stamps[5] = __builtin_amdgcn_s_memtime();
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
        if (rr < n) {
            if (SC1)
                fx_st(Y + (size_t)rr * 16 + qg, want ? yv[u] : 0.0);
            else
                Y[(size_t)rr * 16 + qg] = want ? yv[u] : 0.0;
        }
        bad |= !(fabs(yv[u]) < INFINITY);
    }
    if (want && jg == 0) {
        if (SC1)
            fx_st(theta + qg, th[qg]);
        else
            theta[qg] = th[qg];
        bad |= !(fabs(th[qg]) < INFINITY);
    }
    if ((bad || (tid == 0 && s_bad)) && flag) atomicOr(flag, 16u);
    if (tid == 0 && stamps) stamps[6] = __builtin_amdgcn_s_memtime();
}

