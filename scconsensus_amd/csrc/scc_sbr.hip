// scc_sbr.hip — two-stage reduction of the PCA Gram to tridiagonal form.
//
// The PCA step of stage 3 (irlba::prcomp_irlba, R/reclusterDEConsensusFast.R:398;
// R/reclusterDEConsensus.R:234) needs the exact top-15 eigenpairs of the
// |U| x |U| centred Gram (its 15th/16th eigenvalues are routinely
// within 1e-3, so a direct method).  The one-stage Householder reduction
// (scc_eigen.hip, k_tridiag) needs one cross-workgroup hand-off per column.
// This file is the alternative by successive band reduction (opt-in, see
// scc_sbr_band for why it is not the default):
//
//   stage 1 (dense -> band of width B): per panel of B columns, three launches
//     k_sbr_panel   one workgroup: Householder QR of the panel below the band.
//                   One pass over the rows per column gives the column's norm,
//                   the dots that update the columns right of it AND the dots
//                   with the reflectors left of it (V^T V for dlarft), so a
//                   column costs two barriers; then T (dlarft) and VT = V T
//     k_sbr_y       Y = A22 VT (tiles of 32 rows) and per-tile partials of
//                   M = VT^T Y
//     k_sbr_update  A22 <- A22 - V W^T - W V^T, W = Y - V M / 2 (64 x 64 tiles)
//   stage 2 (band -> tridiagonal): k_sbr_chase, one workgroup, the band in LDS;
//     wave w chases the bulges of sweeps j = w, w + 16, ...; a sweep waits on
//     its predecessor only where their blocks overlap.  A task reads its three
//     blocks at once, keeps every operand of the reflector's application in
//     registers (reductions over rows / columns by DPP inside a lane group)
//     and hands off through LDS only (no fence on the global reflector stores).
//   back-transformation: k_sbr_back, one workgroup per eigenvector: the bulge
//     reflectors (a sweep's blocks are disjoint: one lane group each, sweeps in
//     reverse order, reflectors prefetched PF sweeps ahead), then the panels'
//     compact-WY blocks I - V T V^T in reverse (one row per thread, the next
//     panel's rows prefetched).
//
// numpy model of every step: tests/sbr_model.py.  Deterministic: fixed
// reduction orders, no floating-point atomics.
#include "scc_common.hpp"
#include <algorithm>

#define SBR_T 1024
#define SBR_W (SBR_T / 64)

// sum over the lanes of a group of G consecutive lanes (G | 64), DPP /
// permlane butterflies: every lane of the group ends with the same value.
// Whole wave only (every lane active).
template <int G>
__device__ inline double group_sum(double v)
{
    if constexpr (G >= 64) v += scc_xor_lane_f64<32>(v);
    if constexpr (G >= 32) v += scc_xor_lane_f64<16>(v);
    if constexpr (G >= 16) v += scc_xor_lane_f64<8>(v);
    if constexpr (G >= 8) v += scc_xor_lane_f64<4>(v);
    if constexpr (G >= 4) v += scc_xor_lane_f64<2>(v);
    if constexpr (G >= 2) v += scc_xor_lane_f64<1>(v);
    return v;
}

// sum over the lanes l, l + S, l + 2S, ... (S | 64)
template <int S>
__device__ inline double strided_sum(double v)
{
    if constexpr (S <= 1) v += scc_xor_lane_f64<1>(v);
    if constexpr (S <= 2) v += scc_xor_lane_f64<2>(v);
    if constexpr (S <= 4) v += scc_xor_lane_f64<4>(v);
    if constexpr (S <= 8) v += scc_xor_lane_f64<8>(v);
    if constexpr (S <= 16) v += scc_xor_lane_f64<16>(v);
    if constexpr (S <= 32) v += scc_xor_lane_f64<32>(v);
    return v;
}

__device__ inline double lane0_d(double v)
{
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readfirstlane((int)(unsigned)b), hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__device__ inline double shfl_d(double v, int src)
{
    const long long b = __double_as_longlong(v);
    const int lo = __shfl((int)(unsigned)b, src, 64), hi = __shfl((int)(b >> 32), src, 64);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// LDS requests of one wave execute in issue order, so handing LDS data to
// another wave needs only this wave's LDS traffic drained -- a generic fence
// would also wait for the reflectors' global stores.
__device__ inline void lds_drain() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// ===================================================================== stage 1
// Panel k: columns [c0, c0 + B), rows r0 = c0 + B .. n - 1 of the working
// matrix Wk (full symmetric storage, row-major, lda).  Writes R (the band) and
// zeros below it into the panel, V (m x B, unit lower trapezoidal, explicit
// zeros / ones) to Vg, T (B x B upper) to Tg and VT = V T to VT.  The panel is
// factored in place with its reflector columns left unscaled (v_c[r] =
// P[r][c] * scal_c below the diagonal), so no pass rewrites a column.
template <int B>
__global__ void __launch_bounds__(SBR_T) k_sbr_panel(double* __restrict__ Wk, int lda, int n, int c0,
                                                     double* __restrict__ Vg, double* __restrict__ Tg,
                                                     double* __restrict__ VT, u64* __restrict__ stamps)
{
    const bool stmp = stamps && threadIdx.x == 0;  // diagnostic: phase cycles of this panel
    u64 ts0 = stmp ? clock64() : 0, ts1 = 0, ts2 = 0, ts3 = 0;
    extern __shared__ __attribute__((aligned(16))) double sm[];
    constexpr int PLD = B + 1, WPC = SBR_W / B, RPS = SBR_T / B;  // waves per column, rows per thread sweep
    const int r0 = c0 + B, m = n - r0, nr = min(m, B);
    const int tid = threadIdx.x, lane = tid & 63, w = scc_wave_id();
    double* P = sm;                       // [m][PLD]
    double* Dp = P + (size_t)m * PLD;     // [WPC][B] partial column dots
    double* rowt = Dp + WPC * B;          // [B] row t before its update
    double* taus = rowt + B;              // [B]
    double* scals = taus + B;             // [B]
    double* betas = scals + B;            // [B]
    double* VV = betas + B;               // [B][B] v_c . v_t (c < t)
    double* Ts = VV + B * B;              // [B][B]
    const int tc = tid % B, tr = tid / B;  // this thread's column / first row in the row sweeps
    for (int i = tr; i < m; i += RPS) P[i * PLD + tc] = Wk[(size_t)(r0 + i) * lda + c0 + tc];
    __syncthreads();
    if (stmp) ts1 = clock64();
    const int col = w % B, part = w / B;
    for (int t = 0; t < nr; ++t) {
        // (i) D_c = sum_{r > t} P[r][t] P[r][c] for every column c: the norm
        //     (c = t), the update of the columns right of t and v_c . v_t (c < t)
        double s = 0.0;
        for (int r = t + 1 + lane + 64 * part; r < m; r += 64 * WPC) s += P[r * PLD + t] * P[r * PLD + col];
        s = group_sum<64>(s);
        if (lane == 0) Dp[part * B + col] = s;
        if (tid < B) rowt[tid] = P[t * PLD + tid];
        __syncthreads();
        // (ii) the reflector of column t (dlarfg) and its application to columns > t
        double sum = 0.0;
#pragma unroll
        for (int q = 0; q < WPC; ++q) sum += Dp[q * B + t];
        const double alpha = rowt[t];
        double beta = alpha, tau = 0.0, scal = 0.0;
        if (sum > 0.0) {
            beta = -copysign(sqrt(alpha * alpha + sum), alpha);
            tau = (beta - alpha) / beta;
            scal = 1.0 / (alpha - beta);
        }
        double dc = 0.0;
#pragma unroll
        for (int q = 0; q < WPC; ++q) dc += Dp[q * B + tc];
        if (tc > t && tau != 0.0) {
            const double wc = rowt[tc] + scal * dc;  // (v_t^T P)[c]
            for (int r = t + tr; r < m; r += RPS) {
                const double vr = (r == t) ? 1.0 : P[r * PLD + t] * scal;
                P[r * PLD + tc] -= tau * vr * wc;
            }
        }
        if (tc < t && tr == 0) VV[tc * B + t] = scals[tc] * (rowt[tc] + scal * dc);  // v_c . v_t
        if (tid == 0) {
            taus[t] = tau;
            scals[t] = scal;
            betas[t] = beta;
        }
        __syncthreads();
    }
    for (int t2 = nr + tid; t2 < B; t2 += SBR_T) taus[t2] = 0.0;  // m < B: no reflector
    __syncthreads();
    if (stmp) ts2 = clock64();
    // T (dlarft forward columnwise), one column per step in wave 0 (LDS
    // requests of one wave are ordered: column i sees columns < i)
    if (w == 0) {
        for (int i = 0; i < B; ++i) {
            const double ti = taus[i];
            if (lane < i) {
                double s = 0.0;
                for (int q = lane; q < i; ++q) s += Ts[lane * B + q] * VV[q * B + i];
                Ts[lane * B + i] = -ti * s;
            } else if (lane < B) {
                Ts[lane * B + i] = (lane == i) ? ti : 0.0;
            }
        }
    }
    __syncthreads();
    if (stmp) ts3 = clock64();
    for (int e = tid; e < B * B; e += SBR_T) Tg[e] = Ts[e];
    // one row per thread: V, VT = V T and the band (R above the diagonal, beta
    // on it, exact zeros below)
    for (int i = tid; i < m; i += SBR_T) {
        double acc[B];
#pragma unroll
        for (int c = 0; c < B; ++c) acc[c] = 0.0;
#pragma unroll 1
        for (int q = 0; q < B; ++q) {
            const double p = P[i * PLD + q];
            const double v = (q >= nr || i < q) ? 0.0 : (i == q ? 1.0 : p * scals[q]);
            Vg[(size_t)i * B + q] = v;
            Wk[(size_t)(r0 + i) * lda + c0 + q] = (i < q) ? p : (i == q ? betas[q] : 0.0);
#pragma unroll
            for (int c = 0; c < B; ++c)
                if (c >= q) acc[c] = fma(v, Ts[q * B + c], acc[c]);
        }
#pragma unroll
        for (int c = 0; c < B; ++c) VT[(size_t)i * B + c] = acc[c];
    }
    if (stmp) {
        stamps[8] = ts1 - ts0;
        stamps[9] = ts2 - ts1;
        stamps[10] = ts3 - ts2;
        stamps[11] = clock64() - ts3;
    }
}

// Y = A22 VT (A22 = Wk[r0:, r0:], m x m) for TR = 256 / B rows per workgroup
// (one output per thread), k in chunks of 64 with the next chunk's loads in
// flight during the current chunk's FMAs, and this tile's partial of
// M = VT^T Y (B x B) in Mp[blockIdx.x]
template <int B>
__global__ void __launch_bounds__(256) k_sbr_y(const double* __restrict__ Wk, int lda, int n, int r0,
                                               const double* __restrict__ VT, double* __restrict__ Y,
                                               double* __restrict__ Mp)
{
    constexpr int TR = 256 / B, KC = 64, NA = TR * KC / 256, NV = KC * B / 256;
    __shared__ double As[TR][KC + 1];
    __shared__ double Vs[KC][B + 1];
    __shared__ double Ys[TR][B + 1];
    const int m = n - r0, i0 = blockIdx.x * TR, tid = threadIdx.x;
    const int ti = tid / B, tc = tid % B;
    double ra[NA], rv[NV];
    auto fetch = [&](int k0) {
#pragma unroll
        for (int u = 0; u < NA; ++u) {
            const int e = tid + 256 * u, i = e / KC, k = e % KC;
            ra[u] = (i0 + i < m && k0 + k < m) ? Wk[(size_t)(r0 + i0 + i) * lda + r0 + k0 + k] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < NV; ++u) {
            const int e = tid + 256 * u, k = e / B, c = e % B;
            rv[u] = (k0 + k < m) ? VT[(size_t)(k0 + k) * B + c] : 0.0;
        }
    };
    fetch(0);
    double acc = 0.0;
    for (int k0 = 0; k0 < m; k0 += KC) {
#pragma unroll
        for (int u = 0; u < NA; ++u) {
            const int e = tid + 256 * u;
            As[e / KC][e % KC] = ra[u];
        }
#pragma unroll
        for (int u = 0; u < NV; ++u) {
            const int e = tid + 256 * u;
            Vs[e / B][e % B] = rv[u];
        }
        __syncthreads();
        if (k0 + KC < m) fetch(k0 + KC);
#pragma unroll 16
        for (int k = 0; k < KC; ++k) acc = fma(As[ti][k], Vs[k][tc], acc);
        __syncthreads();
    }
    Ys[ti][tc] = acc;
    if (i0 + ti < m) Y[(size_t)(i0 + ti) * B + tc] = acc;
    Vs[ti][tc] = (i0 + ti < m) ? VT[(size_t)(i0 + ti) * B + tc] : 0.0;  // this tile's VT rows (TR <= KC)
    __syncthreads();
    if (tid < B * B) {
        const int c1 = tid / B, c2 = tid % B;
        double s = 0.0;
        for (int i = 0; i < TR; ++i) s = fma(Vs[i][c1], Ys[i][c2], s);
        Mp[(size_t)blockIdx.x * B * B + tid] = s;
    }
}

// A22 <- A22 - V W^T - W V^T on a 32 x 32 tile, W = Y - V M / 2, M the sum of
// the nmp partials in tile order; each thread's four elements are loaded
// before any is computed
template <int B>
__global__ void __launch_bounds__(256) k_sbr_update(double* __restrict__ Wk, int lda, int n, int r0,
                                                    const double* __restrict__ V, const double* __restrict__ Y,
                                                    const double* __restrict__ Mp, int nmp)
{
    constexpr int TT = 32, EPT = TT * TT / 256;
    __shared__ double Ms[B][B + 1];
    __shared__ double Vi[TT][B + 1], Vj[TT][B + 1], Wi[TT][B + 1], Wj[TT][B + 1];
    const int m = n - r0, i0 = blockIdx.y * TT, j0 = blockIdx.x * TT, tid = threadIdx.x;
    double a[EPT];
#pragma unroll
    for (int u = 0; u < EPT; ++u) {
        const int e = tid + 256 * u, i = e / TT, j = e % TT;
        a[u] = (i0 + i < m && j0 + j < m) ? Wk[(size_t)(r0 + i0 + i) * lda + r0 + j0 + j] : 0.0;
    }
    if (tid < B * B) {
        double s = 0.0;
#pragma unroll 8
        for (int p = 0; p < nmp; ++p) s += Mp[(size_t)p * B * B + tid];
        Ms[tid / B][tid % B] = s;
    }
    for (int e = tid; e < TT * B; e += 256) {
        const int i = e / B, c = e % B;
        Vi[i][c] = (i0 + i < m) ? V[(size_t)(i0 + i) * B + c] : 0.0;
        Vj[i][c] = (j0 + i < m) ? V[(size_t)(j0 + i) * B + c] : 0.0;
        Wi[i][c] = (i0 + i < m) ? Y[(size_t)(i0 + i) * B + c] : 0.0;
        Wj[i][c] = (j0 + i < m) ? Y[(size_t)(j0 + i) * B + c] : 0.0;
    }
    __syncthreads();
    double wi[(TT * B + 255) / 256], wj[(TT * B + 255) / 256];
#pragma unroll
    for (int u = 0; u < (TT * B + 255) / 256; ++u) {
        const int e = tid + 256 * u, i = e / B, c = e % B;
        if (e < TT * B) {
            double si = 0.0, sj = 0.0;
#pragma unroll
            for (int q = 0; q < B; ++q) {
                si = fma(Vi[i][q], Ms[q][c], si);
                sj = fma(Vj[i][q], Ms[q][c], sj);
            }
            wi[u] = fma(-0.5, si, Wi[i][c]);
            wj[u] = fma(-0.5, sj, Wj[i][c]);
        }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < (TT * B + 255) / 256; ++u) {
        const int e = tid + 256 * u, i = e / B, c = e % B;
        if (e < TT * B) {
            Wi[i][c] = (i0 + i < m) ? wi[u] : 0.0;
            Wj[i][c] = (j0 + i < m) ? wj[u] : 0.0;
        }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < EPT; ++u) {
        const int e = tid + 256 * u, i = e / TT, j = e % TT;
        double s = 0.0;
#pragma unroll
        for (int c = 0; c < B; ++c) s = fma(Vi[i][c], Wj[j][c], fma(Wi[i][c], Vj[j][c], s));
        if (i0 + i < m && j0 + j < m) Wk[(size_t)(r0 + i0 + i) * lda + r0 + j0 + j] = a[u] - s;
    }
}

// ===================================================================== stage 2
// The lower band (2B diagonals: B of the band, B - 1 more for the bulges) in
// LDS, column-major, bd[c * 2B + (r - c)], with B zero columns past n so that
// every read of a task's (possibly clipped) blocks lands on an exact zero and
// needs no mask.  Wave w runs sweeps j = w, w + 16, ...; task s of sweep j
// reduces the rows [j + 1 + sB, j + (s + 1)B] with the reflector taken from
// column src (j, or the first column of the previous block).
//
// Hand-off (prog[j], per sweep): a task first writes its source column
// (beta, zeros) and publishes 2s + 1, then finishes and publishes 2s + 2.
// Task (j, s) touches rows / columns [j + (s - 1)B + 1, j + (s + 2)B]; of
// sweep j - 1 it overlaps task s + 1 wholly and task s + 2 in ONE entry only,
// that task's beta (its source column's top), so it starts at
// prog[j - 1] >= 2s + 5: the chain of sweep starts advances by two tasks and
// a reflector per sweep instead of four tasks.
//
// Lane (rho, g) = (lane % B, lane / B), columns kappa = g + NG k (k < CPL):
// D[rho][kappa] (diagonal block), E[rho][kappa] (block below) and the source
// block transposed, S[kappa][rho], so that every reduction is a row sum
// (in-lane over k, then strided DPP over g) except v.y and the norm (group
// sums over rho); v is loaded at both rho and kappa, y at kappa is one
// bpermute.
template <int B>
__global__ void __launch_bounds__(SBR_T) k_sbr_chase(const double* __restrict__ Wk, int lda, int n,
                                                     double* __restrict__ d, double* __restrict__ e,
                                                     double* __restrict__ refl, double* __restrict__ rtau, int smax,
                                                     u64* __restrict__ stamps)
{
    extern __shared__ __attribute__((aligned(16))) double bd[];
    constexpr int BW = 2 * B, NG = 64 / B, CPL = B / NG;
    int* prog = (int*)(bd + (size_t)(n + B) * BW);
    const int tid = threadIdx.x, lane = tid & 63, w = scc_wave_id();
    const bool stmp = stamps && tid == 0;  // diagnostic: wave 0's wait / task cycles
    u64 t_wait = 0, t_task = 0, n_task = 0;
    const u64 t_all = stmp ? clock64() : 0;
    for (int x = tid; x < (n + B) * BW; x += SBR_T) {
        const int c = x / BW, dg = x - c * BW;
        bd[x] = (dg <= B && c + dg < n) ? Wk[(size_t)(c + dg) * lda + c] : 0.0;
    }
    for (int j = tid; j < n; j += SBR_T) prog[j] = 0;
    __syncthreads();
    const int rho = lane % B, g = lane / B;
    auto ix = [](int r, int c) { return c * (BW - 1) + r; };  // c * BW + (r - c)
    // lane-constant offsets of the operands from per-task scalar bases:
    // S[kappa][rho] = bd[p0 (BW-1) + q0 + o_st], D[rho][kappa] = bd[q0 BW + o_dv],
    // E[rho][kappa] = bd[q0 (BW-1) + q1 + 1 + o_eb], x[a] = bd[src (BW-1) + q0 + a]
    int o_st[CPL], o_dv[CPL], o_eb[CPL];
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        const int kap = g + NG * k;
        o_st[k] = rho * (BW - 1) + kap;
        o_dv[k] = rho >= kap ? kap * (BW - 1) + rho : rho * (BW - 1) + kap;
        o_eb[k] = kap * (BW - 1) + rho;
    }
    for (int j = w; j <= n - 3; j += SBR_W) {
        int p0 = j + 1, p1 = min(j + B, n - 1);
        for (int s = 0;; ++s) {
            const int q0 = s ? p1 + 1 : p0, q1 = s ? min(p1 + B, n - 1) : p1, src = s ? p0 : j;
            if (q1 <= q0) break;
            const u64 tw0 = stmp ? clock64() : 0;
            if (j > 0) {
                if (lane == 0)
                    while (__hip_atomic_load(&prog[j - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < 2 * s + 5)
                        __builtin_amdgcn_s_sleep(1);
                asm volatile("" ::: "memory");
                __builtin_amdgcn_wave_barrier();
            }
            const u64 tw1 = stmp ? clock64() : 0;
            // ---- every operand of the task at once (S is read at s = 0 too,
            //      unused: no branch)
            const int b_x = src * (BW - 1) + q0, b_st = p0 * (BW - 1) + q0, b_d = q0 * BW,
                      b_e = q0 * (BW - 1) + q1 + 1;
            const double xr = bd[b_x + rho];
            double xk[CPL], st[CPL], dv[CPL], eb[CPL];
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
                xk[k] = bd[b_x + g + NG * k];
                st[k] = bd[b_st + o_st[k]];
                dv[k] = bd[b_d + o_dv[k]];
                eb[k] = bd[b_e + o_eb[k]];
            }
            // ---- the reflector (dlarfg) of x = A[q0 .. q1][src]
            const double alpha = lane0_d(xr);
            const double xn2 = group_sum<B>(rho > 0 ? xr * xr : 0.0);
            double beta = alpha, tau = 0.0, scal = 0.0;
            if (xn2 > 0.0) {
                beta = -copysign(sqrt(fma(alpha, alpha, xn2)), alpha);
                tau = (beta - alpha) / beta;
                scal = 1.0 / (alpha - beta);
            }
            const double vr = (rho == 0) ? 1.0 : xr * scal;  // v at my row (0 past the block)
            double vk[CPL];                                   // v at my columns
#pragma unroll
            for (int k = 0; k < CPL; ++k) vk[k] = (g + NG * k == 0) ? 1.0 : xk[k] * scal;
            // ---- the source column becomes (beta, 0, ..., 0): published first
            if (rho == 0)
#pragma unroll
                for (int k = 0; k < CPL; ++k) bd[b_x + g + NG * k] = (g + NG * k == 0) ? beta : 0.0;
            lds_drain();
            if (lane == 0) __hip_atomic_store(&prog[j], 2 * s + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (g == 0) refl[((size_t)j * smax + s) * B + rho] = vr;
            if (lane == 0) rtau[(size_t)j * smax + s] = tau;
            if (tau != 0.0) {
                // ---- left on the rest of the source block (s >= 1): S <- S - tau v (v^T S)
                if (s) {
                    double ws = 0.0;
#pragma unroll
                    for (int k = 0; k < CPL; ++k) ws = fma(vk[k], st[k], ws);
                    const double twl = tau * strided_sum<B>(ws);  // tau (v^T S)[rho]
                    if (rho > 0)
#pragma unroll
                        for (int k = 0; k < CPL; ++k) bd[b_st + o_st[k]] = fma(-twl, vk[k], st[k]);
                }
                // ---- two-sided on D, right on E
                double ys = 0.0, zs = 0.0;
#pragma unroll
                for (int k = 0; k < CPL; ++k) {
                    ys = fma(dv[k], vk[k], ys);
                    zs = fma(eb[k], vk[k], zs);
                }
                const double y = strided_sum<B>(ys);  // (D v)[rho]
                const double tz = tau * strided_sum<B>(zs);  // tau (E v)[rho]
                double yk[CPL];
#pragma unroll
                for (int k = 0; k < CPL; ++k) yk[k] = shfl_d(y, g + NG * k);  // (D v)[kappa] from lane kappa
                const double hc = 0.5 * tau * group_sum<B>(vr * y);          // (tau / 2) v.(D v)
                const double wr = tau * fma(-hc, vr, y);                     // w = tau (D v) - (tau^2 / 2)(v.D v) v
#pragma unroll
                for (int k = 0; k < CPL; ++k) {
                    const int kap = g + NG * k;
                    const double wk = tau * fma(-hc, vk[k], yk[k]);
                    if (rho >= kap) bd[b_d + o_dv[k]] = fma(-vr, wk, fma(-wr, vk[k], dv[k]));
                    bd[b_e + o_eb[k]] = fma(-tz, vk[k], eb[k]);
                }
            }
            lds_drain();
            if (lane == 0) __hip_atomic_store(&prog[j], 2 * s + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (stmp) {
                const u64 tw2 = clock64();
                t_wait += tw1 - tw0;
                t_task += tw2 - tw1;
                ++n_task;
            }
            p0 = q0;
            p1 = q1;
        }
        lds_drain();
        if (lane == 0) __hip_atomic_store(&prog[j], 1 << 30, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (stmp) {
        stamps[0] = t_wait;
        stamps[1] = t_task;
        stamps[7] = n_task;
        stamps[2] = clock64() - t_all;
    }
    __syncthreads();
    for (int i = tid; i < n; i += SBR_T) {
        d[i] = bd[ix(i, i)];
        e[i] = (i + 1 < n) ? bd[ix(i + 1, i)] : 0.0;
    }
}

// ===================================================================== back-transformation
// Zq [16][lda]: the k eigenvectors of the tridiagonal in, of the Gram out; one
// workgroup per vector (blockIdx.x), the vector in LDS.  x = Q1 Q2 z:
//   Q2: sweeps in reverse order, lane group s (B lanes) applies sweep j's
//       reflector s (a sweep's blocks are disjoint), one barrier per sweep;
//       each group's reflector and tau for sweep j - PF are loaded while
//       sweep j is applied;
//   Q1: panels in reverse, x -= V (T (V^T x)): thread i owns row r0 + i, its
//       row of V in registers (loaded during the previous panel), the T
//       factors in LDS.
template <int B>
__global__ void __launch_bounds__(SBR_T) k_sbr_back(double* __restrict__ Zq, int lda, int n,
                                                    const double* __restrict__ refl, const double* __restrict__ rtau,
                                                    int smax, const double* __restrict__ Vg,
                                                    const double* __restrict__ Tg, int npanel)
{
    extern __shared__ __attribute__((aligned(16))) double sm[];
    constexpr int PF = 8;
    double* z = sm;                                   // [n]
    double* Ts = z + ((n + 1) & ~1);                  // [npanel][B][B]
    double* part = Ts + (size_t)npanel * B * B;       // [SBR_W][B]
    double* tdot = part + SBR_W * B;                  // [B]
    double* t2s = tdot + B;                           // [B]
    const int q = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = scc_wave_id();
    for (int i = tid; i < n; i += SBR_T) z[i] = Zq[(size_t)q * lda + i];
    for (int x = tid; x < npanel * B * B; x += SBR_T) Ts[x] = Tg[x];
    // ---- Q2
    const int grp = tid / B, rho = tid % B;
    auto fetch = [&](int j, double& v, double& t) {
        v = 0.0;
        t = 0.0;
        if (j >= 0 && grp <= (n - 3 - j) / B) {  // sweep j has (n - 3 - j) / B + 1 blocks
            const size_t o = (size_t)j * smax + grp;
            t = rtau[o];
            v = refl[o * B + rho];
        }
    };
    double vb[PF], tb[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u) fetch(n - 3 - u, vb[u], tb[u]);
    __syncthreads();
    for (int j0 = n - 3; j0 >= 0; j0 -= PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            const int j = j0 - u;
            if (j < 0) break;
            const double v = vb[u], t = tb[u];
            fetch(j - PF, vb[u], tb[u]);
            const int r = j + 1 + grp * B + rho;
            const double zr = (r < n) ? z[r] : 0.0;
            const double dot = group_sum<B>(v * zr);
            if (r < n && t != 0.0) z[r] = zr - t * dot * v;
            __syncthreads();
        }
    }
    // ---- Q1
    double vc[B], vn[B];
    auto fetch_v = [&](int p, double* v) {
        const int m = n - (p + 1) * B;
        const double* V = Vg + (size_t)p * n * B + (size_t)tid * B;
#pragma unroll
        for (int c = 0; c < B; ++c) v[c] = (p >= 0 && tid < m) ? V[c] : 0.0;
    };
    fetch_v(npanel - 1, vc);
    for (int p = npanel - 1; p >= 0; --p) {
        const int r0 = (p + 1) * B, m = n - r0;
        fetch_v(p - 1, vn);
        const double zi = (tid < m) ? z[r0 + tid] : 0.0;
#pragma unroll
        for (int c = 0; c < B; ++c) {
            const double s = group_sum<64>(vc[c] * zi);
            if (lane == 0) part[w * B + c] = s;
        }
        __syncthreads();
        if (tid < B) {
            double s = 0.0;
            for (int x = 0; x < SBR_W; ++x) s += part[x * B + tid];
            tdot[tid] = s;
        }
        __syncthreads();
        if (tid < B) {  // t2 = T tdot (T upper triangular)
            const double* T = Ts + (size_t)p * B * B + tid * B;
            double s = 0.0;
            for (int c = tid; c < B; ++c) s += T[c] * tdot[c];
            t2s[tid] = s;
        }
        __syncthreads();
        if (tid < m) {
            double s = 0.0;
#pragma unroll
            for (int c = 0; c < B; ++c) s += vc[c] * t2s[c];
            z[r0 + tid] = zi - s;
        }
#pragma unroll
        for (int c = 0; c < B; ++c) vc[c] = vn[c];
        __syncthreads();
    }
    for (int i = tid; i < n; i += SBR_T) Zq[(size_t)q * lda + i] = z[i];
}

// ===================================================================== host
// Band width by n: 0 -> the one-stage solver.  Limits: the chase's band
// (n x 2B doubles) and the panel in LDS; one row per thread in k_sbr_back's
// Q1 and one lane group per block of a sweep in its Q2.
static int sbr_band(int n)
{
    if (n >= 48 && n <= 586) return 16;
    if (n > 586 && n <= 1026) return 8;
    return 0;
}

static size_t sbr_panel_lds(int n, int B)
{
    const int m = n - B;
    return sizeof(double) * ((size_t)m * (B + 1) + (SBR_W / B) * (size_t)B + 4 * (size_t)B + 2 * (size_t)B * B);
}

static size_t sbr_chase_lds(int n, int B) { return sizeof(double) * (size_t)(n + B) * 2 * B + sizeof(int) * (size_t)n; }

static int sbr_npanel(int n, int B)
{
    int np = 0;
    for (int c0 = 0; n - (c0 + B) >= 2; c0 += B) ++np;
    return np;
}

static size_t sbr_back_lds(int n, int B)
{
    return sizeof(double) * ((size_t)((n + 1) & ~1) + (size_t)sbr_npanel(n, B) * B * B + SBR_W * (size_t)B + 2 * B);
}

// 0: the one-stage solver handles n.  Opt-in (SCC_EIG_SBR=1): measured on
// MI355X the panel QR costs about as much per column (2.7 us, two barriers)
// as the one-stage reduction's hand-off, and the chase adds 1-5 ms, so the
// one-stage solver is faster at every n tried (323 ... 1000).
extern "C" int scc_sbr_band(int n)
{
    const char* env = getenv("SCC_EIG_SBR");
    if (!(env && *env && atoi(env) != 0)) return 0;
    const int B = sbr_band(n);
    if (!B) return 0;
    const size_t cap = 160 * 1024;
    if (sbr_panel_lds(n, B) > cap || sbr_chase_lds(n, B) > cap || sbr_back_lds(n, B) > cap) return 0;
    if (n - B > SBR_T || (n - 3) / B + 1 > SBR_T / B) return 0;
    return B;
}

struct SbrLayout {
    size_t wk, vg, tg, vt, y, mp, refl, rtau, total;
    int smax, npanel;
};

static SbrLayout sbr_layout(int n, int lda, int B)
{
    SbrLayout L;
    size_t o = 0;
    auto take = [&](size_t cnt) {
        const size_t at = o;
        o += (cnt + 31) & ~(size_t)31;
        return at;
    };
    L.npanel = sbr_npanel(n, B);
    L.smax = (n + B - 1) / B + 2;
    L.wk = take((size_t)n * lda);
    L.vg = take((size_t)std::max(L.npanel, 1) * n * B);
    L.tg = take((size_t)std::max(L.npanel, 1) * B * B);
    L.vt = take((size_t)n * B);
    L.y = take((size_t)n * B);
    L.mp = take((size_t)((n + 256 / B - 1) / (256 / B) + 1) * B * B);
    L.refl = take((size_t)n * L.smax * B);
    L.rtau = take((size_t)n * L.smax);
    L.total = o;
    return L;
}

extern "C" size_t scc_sbr_scratch_doubles(int n, int lda)
{
    const int B = scc_sbr_band(n);
    return B ? sbr_layout(n, lda, B).total : 0;
}

template <int B>
static hipError_t sbr_reduce(const double* A, int n, int lda, double* scr, double* d, double* e, u64* stamps,
                             hipStream_t st)
{
    const SbrLayout L = sbr_layout(n, lda, B);
    double* Wk = scr + L.wk;
    hipError_t err = hipMemcpy2DAsync(Wk, sizeof(double) * lda, A, sizeof(double) * lda, sizeof(double) * n, n,
                                      hipMemcpyDeviceToDevice, st);
    if (err != hipSuccess) return err;
    const size_t plds = sbr_panel_lds(n, B);
    hipFuncSetAttribute((const void*)k_sbr_panel<B>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)plds);
    for (int p = 0; p < L.npanel; ++p) {
        const int c0 = p * B, r0 = c0 + B, m = n - r0;
        double* Vg = scr + L.vg + (size_t)p * n * B;
        hipLaunchKernelGGL(k_sbr_panel<B>, dim3(1), dim3(SBR_T), plds, st, Wk, lda, n, c0, Vg,
                           scr + L.tg + (size_t)p * B * B, scr + L.vt, p == 0 ? stamps : nullptr);
        const int nty = (m + 256 / B - 1) / (256 / B);
        hipLaunchKernelGGL(k_sbr_y<B>, dim3(nty), dim3(256), 0, st, Wk, lda, n, r0, scr + L.vt, scr + L.y, scr + L.mp);
        const int ntt = (m + 31) / 32;
        hipLaunchKernelGGL(k_sbr_update<B>, dim3(ntt, ntt), dim3(256), 0, st, Wk, lda, n, r0, Vg, scr + L.y,
                           scr + L.mp, nty);
    }
    const size_t clds = sbr_chase_lds(n, B);
    hipFuncSetAttribute((const void*)k_sbr_chase<B>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)clds);
    hipLaunchKernelGGL(k_sbr_chase<B>, dim3(1), dim3(SBR_T), clds, st, Wk, lda, n, d, e, scr + L.refl, scr + L.rtau,
                       L.smax, stamps);
    return hipGetLastError();
}

// A (n x n symmetric, row-major, lda, read only) -> the tridiagonal (d, e:
// e[i] = T[i+1][i]) and, in scr, everything scc_launch_sbr_back needs.
extern "C" hipError_t scc_launch_sbr_reduce(const double* A, int n, int lda, double* scr, double* d, double* e,
                                            unsigned long long* stamps, hipStream_t st)
{
    const int B = scc_sbr_band(n);
    if (B == 16) return sbr_reduce<16>(A, n, lda, scr, d, e, stamps, st);
    if (B == 8) return sbr_reduce<8>(A, n, lda, scr, d, e, stamps, st);
    return hipErrorInvalidValue;
}

template <int B>
static hipError_t sbr_back(double* Zq, int n, int lda, int k, const double* scr, hipStream_t st)
{
    const SbrLayout L = sbr_layout(n, lda, B);
    const size_t lds = sbr_back_lds(n, B);
    hipFuncSetAttribute((const void*)k_sbr_back<B>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k_sbr_back<B>, dim3(k), dim3(SBR_T), lds, st, Zq, lda, n, scr + L.refl, scr + L.rtau, L.smax,
                       scr + L.vg, scr + L.tg, L.npanel);
    return hipGetLastError();
}

extern "C" hipError_t scc_launch_sbr_back(double* Zq, int n, int lda, int k, const double* scr, hipStream_t st)
{
    const int B = scc_sbr_band(n);
    if (B == 16) return sbr_back<16>(Zq, n, lda, k, scr, st);
    if (B == 8) return sbr_back<8>(Zq, n, lda, k, scr, st);
    return hipErrorInvalidValue;
}
