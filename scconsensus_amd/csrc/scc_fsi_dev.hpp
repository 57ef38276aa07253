// scc_fsi_dev.hpp — device helpers shared by the filtered subspace iteration's
// kernels (scc_small_eig.hip: the launch-per-step path; scc_subspace.hip: the
// persistent engine): the wave readlane / sum of fp64 values and the blocked
// 64 x 64 Cholesky + inverse on one workgroup.
#pragma once
#include "scc_common.hpp"

typedef double d4 __attribute__((ext_vector_type(4)));  // one fp64 MFMA 16x16x4 accumulator

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
__device__ inline void fsi_cholinv_blk(double* A, double* X, double* Ri, int* s_bad)
{
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
#pragma unroll
    for (int K = 0; K < 4; ++K) {
        if (wv == 0) {
            const int row = 16 * K + lane, rc = min(row, 63);
            double a[16];
#pragma unroll
            for (int c = 0; c < 16; ++c) a[c] = A[rc * CB_S + 16 * K + c];
            bool bad = false;
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const double d = se_readlane(a[k], k);
                bad |= !(d > 0.0);
                const double dd = d > 0.0 ? d : 1.0;
                double g = __builtin_amdgcn_rsq(dd);
                g = g * fma(-0.5 * dd * g, g, 1.5);
                const double l = (lane > k) ? a[k] * g : (lane == k ? dd * g : 0.0);
                a[k] = l;
                if (lane == 0) Ri[16 * K + k] = g;
#pragma unroll
                for (int c = k + 1; c < 16; ++c) a[c] = fma(-l, se_readlane(l, c), a[c]);
            }
            if (row < 64) {
#pragma unroll
                for (int c = 0; c < 16; ++c) A[row * CB_S + 16 * K + c] = (lane >= c) ? a[c] : 0.0;
            }
            if (bad && lane == 0) *s_bad = 1;
        }
        __syncthreads();
        // trailing blocks (I, J), K < J <= I <= 3, dealt over the waves
        int b = 0;
#pragma unroll
        for (int J = K + 1; J < 4; ++J)
#pragma unroll
            for (int I = J; I < 4; ++I, ++b) {
                if ((b & 3) != wv) continue;
                d4 acc = cb_load(A, I, J);
                acc = cb_block_mm<true>(A, I, K, A, J, K, -1.0, acc);
                cb_store(A, I, J, acc);
            }
        __syncthreads();
    }
    // diagonal blocks of X = L^{-1}: wave I, lane j = column j of block I
    {
        const int I = wv, j = lane & 15;
        double w[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            double s = (i == j) ? 1.0 : 0.0;
#pragma unroll
            for (int m = 0; m < i; ++m) s = fma(-A[(16 * I + i) * CB_S + 16 * I + m], w[m], s);
            w[i] = (i >= j) ? s * Ri[16 * I + i] : 0.0;
        }
        if (lane < 16) {
#pragma unroll
            for (int i = 0; i < 16; ++i) X[(16 * I + i) * CB_S + 16 * I + j] = w[i];
        }
#pragma unroll
        for (int J = 0; J < 4; ++J)  // the zero blocks above the diagonal
            if (J > I && lane < 16) {
#pragma unroll
                for (int i = 0; i < 16; ++i) X[(16 * I + i) * CB_S + 16 * J + j] = 0.0;
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

