// scc_eigen.hip — top-k eigenpairs of the |U| x |U| fp64 Gram matrix.
//
// Dense symmetric eigensolver for the PCA step of stage 3 (reference:
// irlba::prcomp_irlba, R/reclusterDEConsensusFast.R:398; R/reclusterDEConsensus.R:234).
// The spectrum of the centred union-gene Gram is a few cluster "spikes" over a
// noise bulk, so the 15th/16th eigenvalues are routinely within 1e-3 relative
// of each other: Krylov/subspace iterations need hundreds of steps
// there, while a direct method is exact to fp64 backward error.
//
// Three launches:
//   1. k_tridiag  — Householder tridiagonalisation (LAPACK dsytd2, lower) on
//      `nwg` persistent workgroups.  Rows are dealt cyclically (row r lives in
//      workgroup r % nwg) and stay in that CU's LDS for the whole reduction,
//      so the matrix never goes back to L2/HBM.  One cross-workgroup hand-off
//      per column: every workgroup publishes tau*A22*v for its rows (and the
//      owner of the next column publishes that row), then all workgroups
//      redundantly and deterministically form w and the next reflector.  Every
//      handed-off double travels as two 8-byte {half, step tag} granules, each
//      written by one write-through (`sc1`) store and polled with `sc1` loads
//      (MI355X_MICROARCH.md price list: data-tagged granules), so a hand-off
//      costs one store-to-load trip and no counter or fence.
//   2. k_tri_vectors — one workgroup per wanted eigenpair: multisection on
//      Sturm counts (256 points per round), inverse iteration with the
//      partially pivoted LU of T - lambda I (LAPACK dgttrf/dgttrs order),
//      then the back-transformation by the stored reflectors.
//   3. k_eig_finish — Gram-Schmidt inside eigenvalue clusters
//      (|dl| <= 1e-3 ||T||, the LAPACK dstein criterion), normalisation and a
//      deterministic sign (largest-magnitude component positive).
// Output Z[u*16 + q] = q-th largest eigenvector (q < k), zero padded to 16;
// W[q] the q-th largest eigenvalue.
#include "scc_common.hpp"
#include "scc.h"
#include <algorithm>
#include <cstdlib>
#include <mutex>

#define TRI_T 256
#define TRI_W (TRI_T / 64)
#define VEC_T 256
#define VEC_W (VEC_T / 64)
#define BT_NB 32  // reflectors per compact-WY block of the back-transformation
#define FIN_T 1024
#define FIN_W (FIN_T / 64)
#define EIG_LDS_MAX (160 * 1024)
#define EIG_MAX_WG 256
#define EIG_SPIN_LIMIT (1u << 22)

static constexpr double kEps = 2.220446049250313e-16;

// butterfly 32, 16, ..., 1 through DPP / permlane swaps (whole wave only;
// every lane ends with the same value)
__device__ inline double wave_sum_d(double v)
{
    v += scc_xor_lane_f64<32>(v);
    v += scc_xor_lane_f64<16>(v);
    v += scc_xor_lane_f64<8>(v);
    v += scc_xor_lane_f64<4>(v);
    v += scc_xor_lane_f64<2>(v);
    return v + scc_xor_lane_f64<1>(v);
}

// write-through / L1-bypassing accessors for the cross-workgroup hand-off
__device__ inline double ld_sc1(const double* p)
{
    return __longlong_as_double(
        (long long)__hip_atomic_load((u64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ inline void st_sc1(double* p, double v)
{
    __hip_atomic_store((u64*)p, (u64)__double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// 8-byte granules {32-bit half, 32-bit tag} written by ONE sc1 store each: a
// double travels as two granules; a reader polls until both tags match
// (MI355X_MICROARCH.md price list: data-tagged granules, handoff-1to1).
template <bool LOCAL>
__device__ inline void put_g(u64* g, double x, u32 tag)
{
    const u64 b = (u64)__double_as_longlong(x);
    const u64 t = (u64)tag << 32;
    if (LOCAL) {  // one XCD: a plain 8-byte store lands in the shared L2, where the sc1 polls read
        __hip_atomic_store(g, t | (b >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_store(g + 1, t | (b & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else {
        __hip_atomic_store(g, t | (b >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(g + 1, t | (b & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
__device__ inline u64 get_g(const u64* g) { return __hip_atomic_load((u64*)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ inline double g_val(u64 hi, u64 lo) { return __longlong_as_double((long long)((hi << 32) | (lo & 0xffffffffull))); }

// deterministic block sum over W waves (every thread returns the same value)
template <int W>
__device__ inline double block_sum(double v, double* red)
{
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    v = wave_sum_d(v);
    if (lane == 0) red[wv] = v;
    __syncthreads();
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < W; ++i) s += red[i];
    __syncthreads();
    return s;
}

// ---------------------------------------------------------------------------
// 1. tridiagonalisation
struct TriArgs {
    const double* A;  // n x n symmetric, row-major, lda
    int n, lda, nwg, rows_lds;
    int xcd_local;    // 1: the participating workgroups all run on one XCD (read from
                      // HW_REG_XCC_ID at run time) and hand off through that XCD's L2
    int lds_rows_cap; // rows per workgroup the dynamic LDS holds
    u32* reg;         // [3] XCD pick (xcc + 1), registrations, check-ins (zeroed per launch)
    double* d;        // [n] diagonal of T
    double* e;        // [n] off-diagonal (e[i] = T[i+1][i])
    double* tau;      // [n]
    double* refl;     // reflector i in row i: refl[i*lda + j], j >= i+1 (refl[i][i+1] = 1)
    u64* pg;          // [2][2 lda] granules of tau*A22*v of the current column (hand-off)
    u64* rg;          // [2][2 lda] granules of row i+1 of A^(i-1) (hand-off)
    u64* dg;          // [2][2 EIG_MAX_WG] granules of each workgroup's partial p.v
    double* work;     // own rows when they do not fit LDS: [nwg][R][n]
    u32* counter;     // (unused)
    u64* stamps;      // diagnostic: WG 0 per-phase cycle sums (nullptr normally)
    u32* err;         // 1: a hand-off timed out
};

// Householder reflector from y[lo..n-1] (alpha = y[lo], x = y[lo+1..]), LAPACK
// dlarfg: v[lo] = 1, v[j] = x_j / (alpha - beta); returns beta and tau.
template <int T>
__device__ inline void house(const double* y, int lo, int n, double* v, double* red, double& beta, double& tau)
{
    const int tid = threadIdx.x;
    double part = 0.0;
    for (int j = lo + 1 + tid; j < n; j += T) part += y[j] * y[j];
    const double xn2 = block_sum<T / 64>(part, red);
    const double alpha = y[lo];
    double scal = 0.0;
    beta = alpha;
    tau = 0.0;
    if (xn2 > 0.0) {
        beta = -copysign(sqrt(alpha * alpha + xn2), alpha);
        tau = (beta - alpha) / beta;
        scal = 1.0 / (alpha - beta);
    }
    for (int j = lo + tid; j < n; j += T) v[j] = (j == lo) ? 1.0 : y[j] * scal;
}

// REG: rows in registers when they fit (wave wv holds local rows wv + TRI_W m,
// m < TRI_MR; lane holds columns lane + 64 t, t < NJ), so phase B is
// register FMAs plus one DPP reduction per row instead of LDS round trips.
#define TRI_MR 3
template <bool LOCAL, int NJ>
__global__ void __launch_bounds__(TRI_T) k_tridiag(TriArgs a)
{
    constexpr int NJA = NJ > 0 ? NJ : 1;  // register row slots per lane (NJ = 0: rows in LDS / HBM)
    extern __shared__ __attribute__((aligned(16))) double sm[];
    __shared__ int s_abort, s_rank, s_nwg;
    const int n = a.n, lda = a.lda;
    const int tid = threadIdx.x, lane = tid & 63, wv = scc_wave_id();
    int me = blockIdx.x, nwg = a.nwg;
    if (LOCAL) {
        // the first workgroup to arrive picks its XCD; up to a.nwg workgroups
        // found on that XCD take part, ranked by arrival; the others leave.
        if (tid == 0) {
            u32 x;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
            x &= 0xfu;
            const u32 old = atomicCAS(&a.reg[0], 0u, x + 1u);
            const u32 target = old ? old - 1u : x;
            int rank = -1;
            if (x == target) {
                const u32 r = atomicAdd(&a.reg[1], 1u);
                if (r < (u32)a.nwg) rank = (int)r;
            }
            const u32 seen = atomicAdd(&a.reg[2], 1u) + 1u;  // after the registration returned
            int nw = 0;
            if (rank >= 0) {
                u32 spins = 0, cur = seen;
                while (cur < gridDim.x) {
                    __builtin_amdgcn_s_sleep(2);
                    cur = __hip_atomic_load(&a.reg[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (++spins > EIG_SPIN_LIMIT) {
                        __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        rank = -1;
                        break;
                    }
                }
                const u32 reg = __hip_atomic_load(&a.reg[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                nw = (int)min(reg, (u32)a.nwg);
                if (nw > n) nw = n;
                if (rank >= nw) rank = -1;
            }
            s_rank = rank;
            s_nwg = nw;
        }
        __syncthreads();
        if (s_rank < 0) return;
        me = s_rank;
        nwg = s_nwg;
    }
    const int R = (n + nwg - 1) / nwg;
    // the first TRI_W * TRI_MR own rows live in registers (when n <= 64 NJ),
    // the others in LDS (or the HBM row store when they do not fit)
    const int nreg_max = (NJ > 0 && n <= 64 * NJA) ? TRI_W * TRI_MR : 0;
    const bool rows_lds = LOCAL ? (max(R - nreg_max, 0) <= a.lds_rows_cap) : (a.rows_lds != 0);
    double* vA = sm;           // v_i   (support i+1..n-1)
    double* vB = vA + n;       // v_{i-1}, then v_{i+1}
    double* wp = vB + n;       // w_{i-1}, then w_i
    double* y = wp + n;        // hand-off row / scratch
    double* pp = y + n;        // handed-off p of the current column
    double* red = pp + n;      // 64
    double* part = red + 64;   // EIG_MAX_WG
    double* rows = rows_lds ? (part + EIG_MAX_WG) : (a.work + (size_t)me * R * n);
    const int nown = (me < n) ? (n - me + nwg - 1) / nwg : 0;
    const int nreg = min(nown, nreg_max);
    double rr[TRI_MR][NJA];
    if (tid == 0) s_abort = 0;
    if (nreg > 0) {
#pragma unroll
        for (int m = 0; m < TRI_MR; ++m) {
            const int l = wv + TRI_W * m;
#pragma unroll
            for (int t = 0; t < NJA; ++t) {
                const int j = lane + 64 * t;
                const double x = a.A[(size_t)(me + nwg * min(l, nown - 1)) * lda + min(j, n - 1)];
                rr[m][t] = (l < nreg && j < n) ? x : 0.0;
            }
        }
    }
    for (int l = nreg; l < nown; ++l) {
        const double* src = a.A + (size_t)(me + nwg * l) * lda;
        for (int j = tid; j < n; j += TRI_T) rows[(size_t)(l - nreg) * n + j] = src[j];
    }
    for (int j = tid; j < n; j += TRI_T) y[j] = a.A[j];  // row 0
    __syncthreads();
    if (n == 1) {
        if (me == 0 && tid == 0) {
            a.d[0] = y[0];
            a.e[0] = 0.0;
            a.tau[0] = 0.0;
        }
        return;
    }
    double* vc = vA;
    double* vp = vB;
    double beta, tc;
    house<TRI_T>(y, 1, n, vc, red, beta, tc);
    if (me == 0) {
        if (tid == 0) {
            a.d[0] = y[0];
            a.e[0] = beta;
            a.tau[0] = tc;
        }
        for (int j = 1 + tid; j < n; j += TRI_T) a.refl[j] = vc[j];
    }
    double tp = 0.0;  // tau_{i-1}
    __syncthreads();
    u64 t_b = 0, t_w = 0, t_c = 0, t_r = 0, t0 = 0;
    const bool stmp = a.stamps && me == 0 && tid == 0;
    for (int i = 0; i <= n - 2; ++i) {
        const int par = i & 1;
        const u32 tag = (u32)(i + 1);
        if (stmp) t0 = __builtin_amdgcn_s_memtime();
        u64* pg = a.pg + (size_t)par * 2 * lda;
        u64* rg = a.rg + (size_t)par * 2 * lda;
        u64* dg = a.dg + (size_t)par * 2 * EIG_MAX_WG * TRI_W;
        const bool prev = (i >= 1) && (tp != 0.0);
        // ---- phase B: own rows r >= i+1: apply update i-1, p_r = tau_i A_r. v_i;
        // publish p_r (and row i+1 by its owner) as tagged granules
        double pd = 0.0;
        const int l0 = (i + 1 > me) ? (i + 1 - me + nwg - 1) / nwg : 0;
        if (nreg > 0) {
            // this lane's columns of v_i, v_{i-1}, w_{i-1} (zero outside i+1..n-1, so
            // the dead columns of a row stay untouched and add nothing)
            double vcr[NJA], vpr[NJA], wpr[NJA];
#pragma unroll
            for (int t = 0; t < NJA; ++t) {  // unconditional (clamped) loads, then masks: no branch per load
                const int j = lane + 64 * t, jc = min(j, n - 1);
                const bool live = j > i && j < n;
                const double c = vc[jc], pv = vp[jc], pw = wp[jc];
                vcr[t] = live ? c : 0.0;
                vpr[t] = (live && prev) ? pv : 0.0;
                wpr[t] = (live && prev) ? pw : 0.0;
            }
            // the (up to) 3 register rows together: their v_r / w_r read at once,
            // the rank-2 updates and dot products, then ONE transposed butterfly
            // for the 3 row sums (per row the same additions in the same order as
            // wave_sum_d: lanes l, l ^ 32, l ^ 16, ...; bit-identical)
            static_assert(TRI_MR <= 4, "phase B reduces up to 4 register rows at once");
            double sdm[4] = {0.0, 0.0, 0.0, 0.0};
            double vrm[TRI_MR], wrm[TRI_MR];
#pragma unroll
            for (int m = 0; m < TRI_MR; ++m) {
                const int l = wv + TRI_W * m;
                const int rc = min(me + nwg * l, n - 1);  // clamped, unconditional loads
                const double a = vp[rc], b = wp[rc];
                vrm[m] = prev ? a : 0.0;
                wrm[m] = prev ? b : 0.0;
            }
#pragma unroll
            for (int m = 0; m < TRI_MR; ++m) {
                const int l = wv + TRI_W * m;
                if (l >= nreg || l < l0) continue;
                const int r = me + nwg * l;
                const double vr = vrm[m], wr = wrm[m];
                double sd = 0.0;
#pragma unroll
                for (int t = 0; t < NJA; ++t) {
                    const double x = fma(-vr, wpr[t], fma(-wr, vpr[t], rr[m][t]));
                    rr[m][t] = x;
                    sd = fma(x, vcr[t], sd);
                }
                sdm[m] = sd;
                if (r == i + 1) {
#pragma unroll
                    for (int t = 0; t < NJA; ++t) {
                        const int j = lane + 64 * t;
                        if (j > i && j < n) put_g<LOCAL>(rg + 2 * j, rr[m][t], tag);
                    }
                }
            }
            {
                const bool h32 = (lane & 32) != 0, h16 = (lane & 16) != 0;
                double k0 = h32 ? sdm[2] : sdm[0], k1 = h32 ? sdm[3] : sdm[1];
                const double g0 = h32 ? sdm[0] : sdm[2], g1 = h32 ? sdm[1] : sdm[3];
                k0 += scc_xor_lane_f64<32>(g0);
                k1 += scc_xor_lane_f64<32>(g1);
                double c = h16 ? k1 : k0;
                c += scc_xor_lane_f64<16>(h16 ? k0 : k1);
                c += scc_xor_lane_f64<8>(c);
                c += scc_xor_lane_f64<4>(c);
                c += scc_xor_lane_f64<2>(c);
                c += scc_xor_lane_f64<1>(c);
                // lane 16 m holds row m's sum
                const int m = lane >> 4;
                const int l = wv + TRI_W * m;
                const int rc = min(me + nwg * l, n - 1);
                const double p = tc * c;
                const double pv = p * vc[rc];
                if ((lane & 15) == 0 && m < TRI_MR && l < nreg && l >= l0) put_g<LOCAL>(pg + 2 * rc, p, tag);
                // the wave's p.v partial in row order (lane 0 adds them as before)
#pragma unroll
                for (int mm = 0; mm < TRI_MR; ++mm) {
                    const int lm = wv + TRI_W * mm;
                    const double x = __shfl(pv, 16 * mm, 64);
                    if (lane == 0 && lm < nreg && lm >= l0) pd += x;
                }
            }
        }
        for (int l = max(l0, nreg) + wv; l < nown; l += TRI_W) {
            const int r = me + nwg * l;
            double* row = rows + (size_t)(l - nreg) * n;
            const double vr = prev ? vp[r] : 0.0, wr = prev ? wp[r] : 0.0;
            const bool pub = (r == i + 1);
            double s = 0.0;
            for (int j = i + 1 + lane; j < n; j += 64) {
                double x = row[j];
                if (prev) {
                    x = fma(-vr, wp[j], fma(-wr, vp[j], x));
                    row[j] = x;
                }
                if (pub) put_g<LOCAL>(rg + 2 * j, x, tag);
                s = fma(x, vc[j], s);
            }
            s = wave_sum_d(s);
            const double p = tc * s;
            if (lane == 0) {
                put_g<LOCAL>(pg + 2 * r, p, tag);
                pd += p * vc[r];
            }
        }
        if (lane == 0) red[32 + wv] = pd;  // (red[0..TRI_W) belongs to block_sum)
        if (stmp) t_r += __builtin_amdgcn_s_memtime() - t0;
        __syncthreads();
        if (tid == 0) {
            double s = 0.0;
            for (int q = 0; q < TRI_W; ++q) s += red[32 + q];
            put_g<LOCAL>(dg + 2 * me, s, tag);
        }
        if (stmp) {
            const u64 t1 = __builtin_amdgcn_s_memtime();
            t_b += t1 - t0;
            t0 = t1;
        }
        // ---- phase C (every workgroup, identical arithmetic): poll the granules
        // of p, row i+1 and the partials, then w_i, row i+1 of A^(i), d[i+1]
        // and reflector i+1 into the free v buffer
        {
            // every granule this thread needs is loaded at once and only the
            // missing ones are polled again: one store-to-load trip per step
            constexpr int GJ = 4;
            u32 spins = 0;
            bool bad = false;
            const bool hasd = tid < nwg;
            for (int j0 = i + 1; j0 < n || (j0 == i + 1 && hasd); j0 += GJ * TRI_T) {
                u64 g[GJ][4];
                u64 gd[2] = {0, 0};
                bool need[GJ];
#pragma unroll
                for (int u = 0; u < GJ; ++u) {
                    const int j = j0 + u * TRI_T + tid;
                    need[u] = j < n;
                    if (need[u]) {
                        g[u][0] = get_g(pg + 2 * j);
                        g[u][1] = get_g(pg + 2 * j + 1);
                        g[u][2] = get_g(rg + 2 * j);
                        g[u][3] = get_g(rg + 2 * j + 1);
                    }
                }
                const bool wantd = hasd && j0 == i + 1;
                if (wantd) {
                    gd[0] = get_g(dg + 2 * tid);
                    gd[1] = get_g(dg + 2 * tid + 1);
                }
                for (;;) {
                    bool ok = true;
#pragma unroll
                    for (int u = 0; u < GJ; ++u) {
                        if (!need[u]) continue;
                        const int j = j0 + u * TRI_T + tid;
#pragma unroll
                        for (int h = 0; h < 4; ++h) {
                            if ((u32)(g[u][h] >> 32) != tag) {
                                ok = false;
                                g[u][h] = get_g((h < 2 ? pg : rg) + 2 * j + (h & 1));
                            }
                        }
                    }
                    if (wantd) {
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            if ((u32)(gd[h] >> 32) != tag) {
                                ok = false;
                                gd[h] = get_g(dg + 2 * tid + h);
                            }
                        }
                    }
                    if (ok) break;
                    if (++spins > EIG_SPIN_LIMIT) {
                        bad = true;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
#pragma unroll
                for (int u = 0; u < GJ; ++u) {
                    if (!need[u]) continue;
                    const int j = j0 + u * TRI_T + tid;
                    pp[j] = g_val(g[u][0], g[u][1]);
                    y[j] = g_val(g[u][2], g[u][3]);
                }
                if (wantd) part[tid] = g_val(gd[0], gd[1]);
                if (bad) break;
            }
            if (bad) {
                __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                s_abort = 1;
            }
        }
        __syncthreads();
        if (s_abort) return;
        if (stmp) {
            const u64 t1 = __builtin_amdgcn_s_memtime();
            t_w += t1 - t0;
            t0 = t1;
        }
        // p.v over the handed-off p of every row, in a fixed order (a block sum
        // over j): identical in every workgroup AND independent of how many
        // workgroups joined (the per-workgroup partials part[] are not)
        double pdl = 0.0;
        for (int j = i + 1 + tid; j < n; j += TRI_T) pdl = fma(pp[j], vc[j], pdl);
        const double pdt = block_sum<TRI_W>(pdl, red);
        const double a2 = -0.5 * tc * pdt;
        const double v1 = vc[i + 1];
        const double w1 = (tc != 0.0) ? fma(a2, v1, pp[i + 1]) : 0.0;
        double xp = 0.0;
        for (int j = i + 1 + tid; j < n; j += TRI_T) {
            const double vj = vc[j];
            const double wj = (tc != 0.0) ? fma(a2, vj, pp[j]) : 0.0;
            const double yj = fma(-v1, wj, fma(-w1, vj, y[j]));
            wp[j] = wj;
            y[j] = yj;
            if (j >= i + 3) xp = fma(yj, yj, xp);
        }
        if (i + 1 <= n - 2) {
            // Householder reflector from y[i+2..] (LAPACK dlarfg)
            const double xn2 = block_sum<TRI_W>(xp, red);
            const double alpha = y[i + 2];
            double bn = alpha, tn = 0.0, scal = 0.0;
            if (xn2 > 0.0) {
                bn = -copysign(sqrt(alpha * alpha + xn2), alpha);
                tn = (bn - alpha) / bn;
                scal = 1.0 / (alpha - bn);
            }
            for (int j = i + 2 + tid; j < n; j += TRI_T) vp[j] = (j == i + 2) ? 1.0 : y[j] * scal;
            if (me == 0) {
                if (tid == 0) {
                    a.d[i + 1] = y[i + 1];
                    a.e[i + 1] = bn;
                    a.tau[i + 1] = tn;
                }
                for (int j = i + 2 + tid; j < n; j += TRI_T)
                    a.refl[(size_t)(i + 1) * lda + j] = (j == i + 2) ? 1.0 : y[j] * scal;
            }
            tp = tc;
            tc = tn;
            double* t = vc;  // v_i becomes the previous reflector
            vc = vp;
            vp = t;
        } else {
            __syncthreads();
            if (me == 0 && tid == 0) {
                a.d[n - 1] = y[n - 1];
                a.e[n - 1] = 0.0;
                a.tau[n - 1] = 0.0;
            }
        }
        __syncthreads();
        if (stmp) t_c += __builtin_amdgcn_s_memtime() - t0;
    }
    if (stmp) {
        a.stamps[0] = t_b;
        a.stamps[1] = t_w;
        a.stamps[2] = t_c;
        a.stamps[7] = t_r;
    }
}


// XCD registration shared by both tridiagonalisation kernels: the first
// workgroup to arrive picks its XCD; up to a.nwg workgroups found on that XCD
// take part, ranked by arrival; the others leave.  Returns the rank (-1: leave)
// and the number of participants.
__device__ inline void xcd_register(const TriArgs& a, int n, int* s_rank, int* s_nwg)
{
    if (threadIdx.x == 0) {
        u32 x;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
        x &= 0xfu;
        const u32 old = atomicCAS(&a.reg[0], 0u, x + 1u);
        const u32 target = old ? old - 1u : x;
        int rank = -1;
        if (x == target) {
            const u32 r = atomicAdd(&a.reg[1], 1u);
            if (r < (u32)a.nwg) rank = (int)r;
        }
        const u32 seen = atomicAdd(&a.reg[2], 1u) + 1u;  // after the registration returned
        int nw = 0;
        if (rank >= 0) {
            u32 spins = 0, cur = seen;
            while (cur < gridDim.x) {
                __builtin_amdgcn_s_sleep(2);
                cur = __hip_atomic_load(&a.reg[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (++spins > EIG_SPIN_LIMIT) {
                    __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    rank = -1;
                    break;
                }
            }
            const u32 reg = __hip_atomic_load(&a.reg[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            nw = (int)min(reg, (u32)a.nwg);
            if (rank >= nw) rank = -1;
        }
        *s_rank = rank;
        *s_nwg = nw;
    }
    __syncthreads();
}

// Work items of a follow-up kernel pinned to the XCD the tridiagonalisation ran
// on (its reflectors sit in that XCD's L2): grid = 8 x items; workgroups on
// that XCD claim items from a counter until none are left, the others leave at
// once.  The workgroup that arrives last claims items too, so every item is
// done whatever the dispatch placement, and nothing waits on another
// workgroup (no co-residency assumption).  vc: 2 zeroed counters; *role:
// thread 0's state across calls (0 on entry).  Returns the next item or -1.
__device__ inline int xcd_next(const u32* xcd_pick, u32* vc, int items, int* role)
{
    __shared__ int s_item;
    __syncthreads();  // every thread has read the previous item
    if (threadIdx.x == 0) {
        if (*role == 0) {
            u32 x;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
            x &= 0xfu;
            const u32 want = __hip_atomic_load(xcd_pick, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - 1u;
            const u32 arrived = atomicAdd(&vc[1], 1u);
            *role = (x == want || arrived == gridDim.x - 1) ? 1 : 2;
        }
        int r = -1;
        if (*role == 1) {
            const u32 t = atomicAdd(&vc[0], 1u);
            if (t < (u32)items) r = (int)t;
        }
        s_item = r;
    }
    __syncthreads();
    return s_item;
}

// Variant of xcd_next for grids that are co-resident (8 x items workgroups
// all fit on the chip at once): one item per workgroup; workgroups off the
// XCD wait until every workgroup has arrived and then take what is left.
__device__ inline int xcd_item_wait(const u32* xcd_pick, u32* vc, int items, u32* err)
{
    __shared__ int s_item;
    if (threadIdx.x == 0) {
        u32 x;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
        x &= 0xfu;
        const u32 want = __hip_atomic_load(xcd_pick, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - 1u;
        int r = -1;
        if (x == want) {
            const u32 t = atomicAdd(&vc[0], 1u);
            if (t < (u32)items) r = (int)t;
        }
        atomicAdd(&vc[1], 1u);
        if (r < 0) {
            u32 spins = 0;
            while (__hip_atomic_load(&vc[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < gridDim.x) {
                __builtin_amdgcn_s_sleep(2);
                if (++spins > EIG_SPIN_LIMIT) {
                    __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
            }
            const u32 on = min(__hip_atomic_load(&vc[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), (u32)items);
            if (on < (u32)items) {
                const u32 t = on + atomicAdd(&vc[2], 1u);
                if (t < (u32)items) r = (int)t;
            }
        }
        s_item = r;
    }
    __syncthreads();
    return s_item;
}

// ---------------------------------------------------------------------------
// 2. eigenvalue q (q-th largest) and its eigenvector, one workgroup each
struct VecArgs {
    const double* d;
    const double* e;
    const double* tau;
    const double* refl;
    int n, lda, k, lu_lds;
    double* lu;     // global LU slots [k][5n] when they do not fit LDS
    double* Zq;     // [16][lda] back-transformed vectors (unnormalised sign)
    double* W;      // [k]
    double* tnorm;  // [1]
    const double* tf;  // [ceil((n-2)/BT_NB)][BT_NB][BT_NB] compact-WY T factors
    const u32* xcd;    // the tridiagonalisation's XCD pick (x + 1), or nullptr: run anywhere
    u32* vcount;       // [3] xcd_next / xcd_item_wait counters (zeroed per launch)
    u32* err;
    int wait;          // 1: xcd_item_wait (grid co-resident), 0: xcd_next
    u64* stamps;    // diagnostic: workgroup 0's phase boundaries at [3..7] (nullptr normally)
    int bt_none;    // 1: leave the tridiagonal's eigenvector (the two-stage path back-transforms it)
    int twist;      // 1: twisted factorization for isolated eigenvalues (SCC_EIG_TWIST, default 1)
};

// numbers of eigenvalues of T (d, e^2) strictly below x[0..SP) (Sturm
// sequences, dstebz): SP independent recurrences interleaved so that each
// step's latency chain is shared by SP shifts (one pass over d, e^2)
#define VEC_SP 1
__device__ inline void sturm_counts(const double* d, const double* e2, int n, const double* x, double pivmin, int* c)
{
    double q[VEC_SP];
#pragma unroll
    for (int p = 0; p < VEC_SP; ++p) {
        q[p] = d[0] - x[p];
        q[p] = fabs(q[p]) < pivmin ? -pivmin : q[p];
        c[p] = (q[p] < 0.0);
    }
    auto step = [&](double di, double ei) {
#pragma unroll
        for (int p = 0; p < VEC_SP; ++p) {
            // e2 / q as the hardware reciprocal refined by one Newton step (a few
            // ulp from the IEEE quotient; the count is insensitive to that)
            const double r0 = __builtin_amdgcn_rcp(q[p]);
            const double r = fma(fma(-q[p], r0, 1.0), r0, r0);
            double t = fma(-ei, r, di - x[p]);
            t = fabs(t) < pivmin ? -pivmin : t;
            q[p] = t;
            c[p] += (t < 0.0);
        }
    };
    // whole blocks of 8 steps with their inputs loaded ahead of the chain (a
    // bound check per step costs a branch on the chain), then the remainder
    int i0 = 1;
    for (; i0 + 8 <= n; i0 += 8) {
        double dv[8], ev[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            dv[u] = d[i0 + u];
            ev[u] = e2[i0 + u - 1];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) step(dv[u], ev[u]);
    }
    for (; i0 < n; ++i0) step(d[i0], e2[i0 - 1]);
}

// Eigenvector of an isolated eigenvalue from the twisted factorization of
// T - lam I (Parlett & Dhillon; LAPACK dlar1v without the representation
// tree): the stationary forward (D+) and backward (D-) recurrences run on two
// lanes of one wave in lockstep, gamma_r = D+_r + D-_r - (d_r - lam) picks the
// twist index r = argmin |gamma_r| (smallest r on ties), z_r = 1 and the
// entries on either side are products of ratios formed by all threads (two
// lanes again).  The shift comes from a bisection closed to 4 eps ||T||, so
// one solve suffices (TW_PASSES = 2 adds a pass at the Rayleigh-corrected
// shift lam + gamma_r / |z|^2).  Two dependent chains of n divisions and two of n
// multiplies, where the LU and two inverse-iteration solves were five chains
// of n steps on one thread.  Used when [lam - delta, lam + delta], delta =
// 1e-7 ||T||, holds exactly one eigenvalue (so the vector's error, ~eps ||T|| /
// gap, stays below ~1e-9); returns false (block-uniform) otherwise or when the
// vector is not finite, and the caller runs inverse iteration.  y: the
// normalised vector; wk: 4 n scratch doubles.
#define TW_PASSES 1  // twisted solves (a second one after a Rayleigh correction of the shift)
__device__ __forceinline__ bool tri_twisted(const double* dl, const double* el, const double* e2l, int n, double lam, double tnorm,
                            double pivmin, double* wk, double* y, double* red, int* ired, u64* stm)
{
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    u64 c0 = stm ? clock64() : 0, c1 = 0, c2 = 0;
    double* Dp = wk;
    double* Dm = wk + n;
    double* rl = wk + 2 * (size_t)n;  // -e_i / D+_i   (z_i from z_{i+1}, i < r)
    double* rm = wk + 3 * (size_t)n;  // -e_{i-1} / D-_i (z_i from z_{i-1}, i > r)
    __shared__ int s_cnt[4];
    const double tiny = kEps * tnorm + 1e-300;
    const double del = 1e-7 * tnorm + pivmin;
    constexpr int SB = 8;
    for (int pass = 0; pass < TW_PASSES; ++pass) {
        // lanes 0..3 of wave 0 in lockstep: D+ at lam from the top (0), D- at
        // lam from the bottom (1), Sturm counts at lam - delta (2) and lam +
        // delta (3, first pass only).  The recurrence is carried in determinant
        // form, p_i = (d_i - x) p_{i-1} - e_{i-1}^2 p_{i-2}: one FMA on the
        // dependent chain, no division (lanes 0 and 1 store p_i and p_{i-1},
        // all threads form D_i = p_i / p_{i-1} afterwards; the counts are sign
        // changes), the pair rescaled by a power of two once per SB steps
        if (tid < (pass == 0 ? 4 : 2)) {
            const bool fwd = tid != 1;
            const double x = tid == 2 ? lam - del : (tid == 3 ? lam + del : lam);
            // lanes 2 and 3 store into y (overwritten later): no branch per step
            double* po = tid == 0 ? Dp : (tid == 1 ? Dm : y);  // p_i
            double* qo = tid == 0 ? rl : (tid == 1 ? rm : y);  // p_{i-1}, same scale
            double pp = 1.0;
            double pc = dl[fwd ? 0 : n - 1] - x;
            int neg = pc < 0.0;
            po[fwd ? 0 : n - 1] = pc;
            qo[fwd ? 0 : n - 1] = 1.0;
            auto step = [&](int s, double av, double ev) {
                const double pn = fma(av, pc, -ev * pp);
                neg += (pn < 0.0) != (pc < 0.0);
                const int i = fwd ? s : n - 1 - s;
                po[i] = pn;
                qo[i] = pc;
                pp = pc;
                pc = pn;
            };
            int s0 = 1;
            for (; s0 + SB <= n; s0 += SB) {  // whole blocks: no bound check inside
                double av[SB], ev[SB];
#pragma unroll
                for (int u = 0; u < SB; ++u) {  // inputs loaded ahead of the chain
                    const int s = s0 + u;
                    const int i = fwd ? s : n - 1 - s;
                    av[u] = dl[i] - x;
                    ev[u] = e2l[fwd ? s - 1 : i];
                }
#pragma unroll
                for (int u = 0; u < SB; ++u) step(s0 + u, av[u], ev[u]);
                const int ex = ilogb(pc);
                if (ex > 256 || ex < -256) {
                    pc = ldexp(pc, -ex);
                    pp = ldexp(pp, -ex);
                }
            }
            for (; s0 < n; ++s0) {
                const int i = fwd ? s0 : n - 1 - s0;
                step(s0, dl[i] - x, e2l[fwd ? s0 - 1 : i]);
            }
            if (pass == 0 && tid >= 2) s_cnt[tid] = neg;
        }
        __syncthreads();
        if (pass == 0 && stm) c1 = clock64();
        if (pass == 0 && s_cnt[3] - s_cnt[2] != 1) return false;  // not isolated (or non-finite)
        for (int i = tid; i < n; i += VEC_T) {  // D = p_i / p_{i-1}; an exact zero pivot -> tiny
            const double dp = Dp[i] / rl[i], dm = Dm[i] / rm[i];
            Dp[i] = (fabs(dp) < tiny) ? (dp < 0.0 ? -tiny : tiny) : dp;
            Dm[i] = (fabs(dm) < tiny) ? (dm < 0.0 ? -tiny : tiny) : dm;
        }
        __syncthreads();
        double best = INFINITY;
        int br = n;
        for (int r = tid; r < n; r += VEC_T) {
            const double g = fabs(Dp[r] + Dm[r] - (dl[r] - lam));
            if (g < best) {
                best = g;
                br = r;
            }
        }
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) {
            const double ob = __shfl_xor(best, m, 64);
            const int orr = __shfl_xor(br, m, 64);
            if (ob < best || (ob == best && orr < br)) {
                best = ob;
                br = orr;
            }
        }
        if (lane == 0) {
            red[wv] = best;
            ired[wv] = br;
        }
        __syncthreads();
        best = red[0];
        br = ired[0];
        for (int w = 1; w < VEC_W; ++w)
            if (red[w] < best || (red[w] == best && ired[w] < br)) {
                best = red[w];
                br = ired[w];
            }
        __syncthreads();
        if (br >= n) return false;  // every gamma NaN
        const int r = br;
        const double gam = Dp[r] + Dm[r] - (dl[r] - lam);
        for (int i = tid; i < n; i += VEC_T) {
            rl[i] = (i < n - 1) ? -el[i] / Dp[i] : 0.0;
            rm[i] = (i > 0) ? -el[i - 1] / Dm[i] : 0.0;
        }
        __syncthreads();
        if (tid < 2) {  // lane 0: z_{r-1} .. z_0, lane 1: z_{r+1} .. z_{n-1}
            const bool up = tid == 0;
            const int len = up ? r : n - 1 - r;
            double z = 1.0;
            if (up) y[r] = 1.0;
            int s0 = 1;
            for (; s0 + SB - 1 <= len; s0 += SB) {  // whole blocks: no bound check inside
                double rv[SB];
#pragma unroll
                for (int u = 0; u < SB; ++u) rv[u] = up ? rl[r - s0 - u] : rm[r + s0 + u];
#pragma unroll
                for (int u = 0; u < SB; ++u) {
                    z *= rv[u];
                    y[up ? r - s0 - u : r + s0 + u] = z;
                }
            }
            for (; s0 <= len; ++s0) {
                z *= up ? rl[r - s0] : rm[r + s0];
                y[up ? r - s0 : r + s0] = z;
            }
        }
        __syncthreads();
        double ss = 0.0;
        for (int i = tid; i < n; i += VEC_T) ss = fma(y[i], y[i], ss);
        ss = block_sum<VEC_W>(ss, red);
        if (!(ss >= 1.0) || !(ss < INFINITY)) return false;
        if (pass + 1 < TW_PASSES) {
            if (stm) c2 = clock64();
            lam += gam / ss;  // Rayleigh quotient of z
        } else {
            const double inv = 1.0 / sqrt(ss);
            for (int i = tid; i < n; i += VEC_T) y[i] *= inv;
            __syncthreads();
        }
    }
    if (stm) {
        if (!c2) c2 = c1;
        stm[8] = c1 - c0;
        stm[9] = c2 - c1;
        stm[10] = clock64() - c2;
    }
    return true;
}

__device__ __forceinline__ void tri_vector_item(const VecArgs& a, const int q)
{
    extern __shared__ __attribute__((aligned(16))) double sm[];
    __shared__ double red[16];
    __shared__ int ired[VEC_W];
    const int n = a.n, tid = threadIdx.x, lane = tid & 63, wv = scc_wave_id();
    const bool stmp = a.stamps && q == 0 && tid == 0;
    const u64 t0 = stmp ? clock64() : 0;
    double* dl = sm;
    double* el = dl + n;
    double* e2l = el + n;
    double* y = e2l + n;
    double* lu = a.lu_lds ? (y + n) : (a.lu + (size_t)q * 6 * n);
    for (int i = tid; i < n; i += VEC_T) {
        dl[i] = a.d[i];
        el[i] = a.e[i];
        e2l[i] = a.e[i] * a.e[i];
    }
    __syncthreads();
    // Gershgorin bounds and pivmin (LAPACK dstebz)
    double gl = INFINITY, gu = -INFINITY, em = 0.0;
    for (int i = tid; i < n; i += VEC_T) {
        const double r = (i > 0 ? fabs(el[i - 1]) : 0.0) + (i < n - 1 ? fabs(el[i]) : 0.0);
        gl = fmin(gl, dl[i] - r);
        gu = fmax(gu, dl[i] + r);
        if (i < n - 1) em = fmax(em, e2l[i]);
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        gl = fmin(gl, __shfl_xor(gl, m, 64));
        gu = fmax(gu, __shfl_xor(gu, m, 64));
        em = fmax(em, __shfl_xor(em, m, 64));
    }
    if (lane == 0) {
        red[wv] = gl;
        red[4 + wv] = gu;
        red[8 + wv] = em;
    }
    __syncthreads();
    gl = red[0];
    gu = red[4];
    em = red[8];
    for (int w = 1; w < VEC_W; ++w) {
        gl = fmin(gl, red[w]);
        gu = fmax(gu, red[4 + w]);
        em = fmax(em, red[8 + w]);
    }
    __syncthreads();
    const double tnorm = fmax(fabs(gl), fabs(gu));
    const double pivmin = fmax(2.2250738585072014e-308 * fmax(1.0, em), 1e-300);
    double lo = gl - 2.0 * tnorm * kEps * n - 1e-300;
    double hi = gu + 2.0 * tnorm * kEps * n + 1e-300;
    // ---- multisection: VEC_T x VEC_SP Sturm counts per round (point tid * SP + p)
    const int target = n - 1 - q;  // ascending index of the q-th largest
    constexpr int NP = VEC_T * VEC_SP;
    for (int it = 0; it < 64; ++it) {
        double x[VEC_SP];
        int c[VEC_SP];
#pragma unroll
        for (int p = 0; p < VEC_SP; ++p) x[p] = lo + (hi - lo) * (double)(tid * VEC_SP + p + 1) / (double)(NP + 1);
        sturm_counts(dl, e2l, n, x, pivmin, c);
        int fp = VEC_SP;  // my first point with lambda_target < x
#pragma unroll
        for (int p = VEC_SP - 1; p >= 0; --p)
            if (c[p] > target) fp = p;
        const unsigned long long above = __ballot(fp < VEC_SP);
        const int src = above ? __builtin_ctzll(above) : 0;
        const int fsrc = __shfl(fp, src, 64);
        if (lane == 0) ired[wv] = above ? (wv * 64 + src) * VEC_SP + fsrc : NP;
        __syncthreads();
        int first = NP;
        for (int w = 0; w < VEC_W; ++w) first = min(first, ired[w]);
        __syncthreads();
        const double nlo = (first == 0) ? lo : lo + (hi - lo) * (double)first / (double)(NP + 1);
        const double nhi = (first == NP) ? hi : lo + (hi - lo) * (double)(first + 1) / (double)(NP + 1);
        if (nlo == lo && nhi == hi) break;
        lo = nlo;
        hi = nhi;
        // 1e-11 relative (or 2 eps ||T||) is enough for inverse iteration (two
        // solves gain (shift error / gap)^2); the twisted factorization takes
        // the shift as it is, so with a.twist the bracket closes to 4 eps ||T||
        // (its vector error ~ shift error / gap)
        if (hi - lo <= (a.twist ? 4.0 * kEps * tnorm
                                : fmax(1e-11 * fmax(fabs(lo), fabs(hi)), 2.0 * kEps * tnorm)) + pivmin)
            break;
    }
    const double lam = 0.5 * (lo + hi);
    const u64 t1 = stmp ? clock64() : 0;
    if (tid == 0) {
        a.W[q] = lam;
        if (q == 0) a.tnorm[0] = tnorm;
    }
    // ---- twisted factorization for an isolated eigenvalue (tri_twisted);
    // otherwise (a cluster closer than 1e-7 ||T||, a non-finite vector) inverse
    // iteration below
    u64 t2 = 0;
    const bool twisted = a.twist && a.lu_lds && tri_twisted(dl, el, e2l, n, lam, tnorm, pivmin, y + n, y, red, ired, stmp ? a.stamps : nullptr);
    if (!twisted) {
        // ---- inverse iteration (dgttrf / dgttrs) by thread 0: the factor's
        // recurrence runs in registers (the next diagonal and super-diagonal are
        // carried, the inputs are independent loads), pivots stored as reciprocals
        double* fdr = lu;  // 1 / U diagonal
        double* fu = fdr + n;
        double* fu2 = fu + n;
        double* fl = fu2 + n;
        double* fp = fl + n;
        double* w = fp + n;  // forward-solve result
        const double tiny = kEps * tnorm + 1e-300;
        if (tid == 0) {
            // inputs of LU_B steps are loaded together ahead of the dependent chain
            constexpr int LU_B = 8;
            double dcur = dl[0] - lam, ucur = (n > 1) ? el[0] : 0.0;
            for (int i0 = 0; i0 < n - 1; i0 += LU_B) {
                double li[LU_B], dn[LU_B], un[LU_B];
    #pragma unroll
                for (int u = 0; u < LU_B; ++u) {  // clamped unconditional loads
                    const int i = i0 + u;
                    const double e0 = el[min(i, n - 1)], d1 = dl[min(i + 1, n - 1)], e1 = el[min(i + 1, n - 1)];
                    li[u] = e0;
                    dn[u] = d1 - lam;
                    un[u] = (i < n - 2) ? e1 : 0.0;
                }
    #pragma unroll
                for (int u = 0; u < LU_B; ++u) {  // branch-free step: one division on the chain
                    const int i = i0 + u;
                    if (i >= n - 1) break;
                    const bool piv = fabs(dcur) < fabs(li[u]);  // LAPACK dgttrf: swap rows i, i+1
                    const double dc = (!piv && dcur == 0.0) ? tiny : dcur;
                    const double den = piv ? li[u] : dc;
                    // (piv ? dc : l) / den as a refined hardware reciprocal (a few ulp)
                    const double r0 = __builtin_amdgcn_rcp(den);
                    const double f = (piv ? dc : li[u]) * fma(fma(-den, r0, 1.0), r0, r0);
                    fl[i] = f;
                    fdr[i] = den;  // the pivot; its reciprocal is taken below, off the chain
                    // operands selected first, one FMA each on the chain (no branch)
                    const double ua = piv ? dn[u] : ucur, ub = piv ? ucur : dn[u];
                    fu[i] = ua;
                    fu2[i] = piv ? un[u] : 0.0;  // zero at i = n - 2
                    fp[i] = piv ? 1.0 : 0.0;
                    dcur = fma(-f, ua, ub);
                    ucur = piv ? -f * un[u] : un[u];
                }
            }
            if (dcur == 0.0) dcur = tiny;
            fdr[n - 1] = dcur;
            fu[n - 1] = 0.0;
            fu2[n - 1] = 0.0;
        }
        __syncthreads();
        for (int i = tid; i < n; i += VEC_T) fdr[i] = 1.0 / fdr[i];
        t2 = stmp ? clock64() : 0;
        for (int i = tid; i < n; i += VEC_T) {  // deterministic pseudo-random start
            unsigned h = (unsigned)i * 2654435761u ^ ((unsigned)q * 40503u + 12345u);
            h ^= h >> 13;
            h *= 0x5bd1e995u;
            h ^= h >> 15;
            y[i] = 0.5 + (double)(h & 0xffff) / 65536.0;
        }
        __syncthreads();
        for (int iter = 0; iter < 2; ++iter) {
            if (tid == 0) {
                constexpr int SB = 8;  // inputs of SB steps loaded ahead of the dependent chain
                double bi = y[0];
                for (int i0 = 0; i0 < n - 1; i0 += SB) {  // w = L^-1 P y
                    double bn[SB], f[SB], pv[SB];
    #pragma unroll
                    for (int u = 0; u < SB; ++u) {
                        const int i = min(i0 + u, n - 2);
                        bn[u] = y[i + 1];
                        f[u] = fl[i];
                        pv[u] = fp[i];
                    }
    #pragma unroll
                    for (int u = 0; u < SB; ++u) {
                        if (i0 + u >= n - 1) break;
                        // operands selected first, one FMA on the chain (no branch)
                        const bool piv = pv[u] != 0.0;
                        const double xa = piv ? bn[u] : bi, xb = piv ? bi : bn[u];
                        w[i0 + u] = xa;
                        bi = fma(-f[u], xa, xb);
                    }
                }
                w[n - 1] = bi;
                double z1 = 0.0, z2 = 0.0;  // y = U^-1 w, from the bottom
                for (int i1 = n - 1; i1 >= 0; i1 -= SB) {
                    double wv8[SB], u1[SB], u2[SB], r[SB];
    #pragma unroll
                    for (int u = 0; u < SB; ++u) {
                        const int i = max(i1 - u, 0);
                        wv8[u] = w[i];
                        u1[u] = fu[i];
                        u2[u] = fu2[i];
                        r[u] = fdr[i];
                    }
    #pragma unroll
                    for (int u = 0; u < SB; ++u) {
                        const int i = i1 - u;
                        if (i < 0) break;
                        const double z0 = fma(-u1[u], z2, fma(-u2[u], z1, wv8[u])) * r[u];  // z2 = y[i+1], z1 = y[i+2]
                        y[i] = z0;
                        z1 = z2;
                        z2 = z0;
                    }
                }
            }
            __syncthreads();
            // scale by the largest magnitude first (a solve can grow y by 1/pivot ~ 1e300)
            double mx = 0.0;
            for (int i = tid; i < n; i += VEC_T) mx = fmax(mx, fabs(y[i]));
    #pragma unroll
            for (int m = 32; m >= 1; m >>= 1) mx = fmax(mx, __shfl_xor(mx, m, 64));
            if (lane == 0) red[8 + wv] = mx;
            __syncthreads();
            mx = red[8];
            for (int w2 = 1; w2 < VEC_W; ++w2) mx = fmax(mx, red[8 + w2]);
            const double sc = (mx > 0.0 && mx < INFINITY) ? 1.0 / mx : 1.0;
            double s = 0.0;
            for (int i = tid; i < n; i += VEC_T) {
                const double v = y[i] * sc;
                s += v * v;
            }
            s = block_sum<VEC_W>(s, red);
            const double inv = sc / sqrt(s);
            for (int i = tid; i < n; i += VEC_T) y[i] *= inv;
            __syncthreads();
        }
    }
    if (twisted) t2 = stmp ? clock64() : 0;
    // ---- back-transformation z = H_0 H_1 ... H_{n-3} y in blocks of BT_NB
    // reflectors, last block first: block b is I - V T V^T (compact WY, T from
    // k_refl_T), three barrier-separated steps per block
    const u64 t3 = stmp ? clock64() : 0;
    __shared__ double bw[BT_NB], bt[BT_NB];
    const int nr = a.bt_none ? 0 : n - 2;
    for (int b = (nr > 0 ? (nr + BT_NB - 1) / BT_NB : 0) - 1; b >= 0; --b) {
        const int kb = b * BT_NB, nb = min(BT_NB, nr - kb);
        {  // bw = V^T y: wave wv takes i = wv + VEC_W t, all its loads in flight together
            constexpr int NT = BT_NB / VEC_W;
            double acc[NT];
#pragma unroll
            for (int t = 0; t < NT; ++t) acc[t] = 0.0;
            for (int j = kb + 1 + lane; j < n; j += 64) {
                const double yj = y[j];
#pragma unroll
                for (int t = 0; t < NT; ++t) {
                    const int i = wv + VEC_W * t;  // v_i is zero at rows <= kb + i
                    const double v = a.refl[(size_t)(kb + min(i, nb - 1)) * a.lda + j];  // unconditional load
                    acc[t] += (i < nb && j > kb + i) ? v * yj : 0.0;
                }
            }
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const double sd = wave_sum_d(acc[t]);
                if (lane == 0 && wv + VEC_W * t < nb) bw[wv + VEC_W * t] = sd;
            }
        }
        __syncthreads();
        if (tid < nb) {  // bt = T bw (upper triangular)
            const double* T = a.tf + ((size_t)b * BT_NB + tid) * BT_NB;
            double sd = 0.0;
            for (int m = tid; m < nb; ++m) sd += T[m] * bw[m];
            bt[tid] = sd;
        }
        __syncthreads();
        for (int j = kb + 1 + tid; j < n; j += VEC_T) {  // y -= V bt
            const int im = min(nb, j - kb);
            double sd = 0.0;
#pragma unroll 8
            for (int i = 0; i < im; ++i) sd += a.refl[(size_t)(kb + i) * a.lda + j] * bt[i];
            y[j] -= sd;
        }
        __syncthreads();
    }
    for (int i = tid; i < n; i += VEC_T) a.Zq[(size_t)q * a.lda + i] = y[i];
    if (stmp) {
        a.stamps[3] = t1 - t0;
        a.stamps[4] = t2 - t1;
        a.stamps[5] = t3 - t2;
        a.stamps[6] = clock64() - t3;
    }
}

__global__ void __launch_bounds__(VEC_T) k_tri_vectors(VecArgs a)
{
    if (!a.xcd) {
        tri_vector_item(a, (int)blockIdx.x);
        return;
    }
    if (a.wait) {
        const int q = xcd_item_wait(a.xcd, a.vcount, a.k, a.err);
        if (q >= 0) tri_vector_item(a, q);
        return;
    }
    int role = 0;
    for (int q; (q = xcd_next(a.xcd, a.vcount, a.k, &role)) >= 0;) tri_vector_item(a, q);
}

// T[0:i, i] = -tau_i T[0:i, 0:i] G[i, 0:i], T[i][i] = tau_i (G[i][j] = v_i .
// v_j for j < i).  Row r of T only depends on row r (T[r][i] = -tau_i sum_{r <=
// m < i} T[r][m] G[i][m]), so thread r < 32 keeps its row in registers and
// runs all columns without a barrier; G is read as LDS broadcasts.
__device__ __forceinline__ void refl_T_recur(const double (*G)[BT_NB + 1], const double* __restrict__ tau, int kb,
                                             int nb, double* __restrict__ tf, int b)
{
    const int r = threadIdx.x;
    if (r >= BT_NB) return;
    double t[BT_NB];
#pragma unroll
    for (int i = 0; i < BT_NB; ++i) {
        const double ti = i < nb ? tau[kb + min(i, nb - 1)] : 0.0;
        double sacc = 0.0;
#pragma unroll
        for (int m = 0; m < i; ++m) sacc = fma(m >= r ? t[m] : 0.0, G[i][m], sacc);
        t[i] = (i < nb) ? ((r < i) ? -ti * sacc : (r == i ? ti : 0.0)) : 0.0;
    }
#pragma unroll
    for (int i = 0; i < BT_NB; ++i) tf[(size_t)b * BT_NB * BT_NB + r * BT_NB + i] = t[i];
}

// T factors of the compact WY form of the reflectors, one workgroup per block
// of BT_NB (LAPACK dlarft, forward / columnwise): T[i][i] = tau_i,
// T[0:i, i] = -tau_i T[0:i, 0:i] (V[:, 0:i]^T v_i).
__device__ __forceinline__ void refl_T_item(const double* __restrict__ refl, const double* __restrict__ tau, int n,
                                            int lda, double* __restrict__ tf, const int b)
{
    __shared__ double G[BT_NB][BT_NB + 1];
    const int kb = b * BT_NB, nb = min(BT_NB, n - 2 - kb), tid = threadIdx.x;
    // G[i][j] = v_i . v_j for j < i (both nonzero from row kb + i + 1): wave wv
    // takes rows i = wv and wv + 16, every j < i in registers
    const int lane = tid & 63, wv = scc_wave_id();
    for (int i = wv; i < BT_NB; i += 16) {
        double acc[BT_NB];
#pragma unroll
        for (int j = 0; j < BT_NB; ++j) acc[j] = 0.0;
        if (i < nb) {
            const double* vi = refl + (size_t)(kb + i) * lda;
            for (int r = kb + i + 1 + lane; r < n; r += 64) {
                const double x = vi[r];
#pragma unroll
                for (int j = 0; j < BT_NB; ++j) {
                    const double y = refl[(size_t)(kb + min(j, nb - 1)) * lda + r];  // unconditional load
                    acc[j] += (j < i) ? x * y : 0.0;
                }
            }
        }
#pragma unroll
        for (int j = 0; j < BT_NB; ++j) {
            const double sj = wave_sum_d(acc[j]);
            if (lane == 0) G[i][j] = sj;
        }
    }
    __syncthreads();
    refl_T_recur(G, tau, kb, nb, tf, b);
}

// k_refl_T with the block's 32 reflector rows staged in LDS (32 n doubles,
// coalesced), then G[i][j] = v_i . v_j by thread (i, j) from LDS: one pass over
// the reflectors instead of 32 strided loads per row step and 32 wave sums per
// row.  Grid: one workgroup per block.
__global__ void __launch_bounds__(1024) k_refl_T_lds(const double* __restrict__ refl, const double* __restrict__ tau,
                                                     int n, int lda, double* __restrict__ tf)
{
    extern __shared__ __attribute__((aligned(16))) double Vs[];  // [BT_NB][n]
    __shared__ double G[BT_NB][BT_NB + 1];
    const int b = blockIdx.x, kb = b * BT_NB, nb = min(BT_NB, n - 2 - kb), tid = threadIdx.x;
    const int lane = tid & 63, wv = scc_wave_id();
    // v_i: rows > kb + i (zero elsewhere and past nb); clamped unconditional
    // loads, all of a lane's in flight before the first store
    constexpr int SR = 8;  // row steps per batch
    for (int i = wv; i < BT_NB; i += 16) {
        const double* src = refl + (size_t)(kb + min(i, nb - 1)) * lda;
        for (int r0 = lane; r0 < n; r0 += 64 * SR) {
            double v[SR];
#pragma unroll
            for (int u = 0; u < SR; ++u) v[u] = src[min(r0 + 64 * u, n - 1)];
#pragma unroll
            for (int u = 0; u < SR; ++u) {
                const int r = r0 + 64 * u;
                if (r < n) Vs[(size_t)i * n + r] = (i < nb && r > kb + i) ? v[u] : 0.0;
            }
        }
    }
    __syncthreads();
    if (wv < 4) {  // G = V V^T on fp64 MFMA: wave w the 16 x 16 tile (16 (w >> 1), 16 (w & 1))
        const int i0 = 16 * (wv >> 1), j0 = 16 * (wv & 1), kr = lane >> 4, cc = lane & 15;
        const double* va = Vs + (size_t)(i0 + cc) * n;
        const double* vb = Vs + (size_t)(j0 + cc) * n;
        typedef double d4v __attribute__((ext_vector_type(4)));
        d4v acc = {0.0, 0.0, 0.0, 0.0};
        for (int k0 = kb & ~3; k0 < n; k0 += 4) {  // rows <= kb are zero in every v of the block
            const int r = min(k0 + kr, n - 1);
            const bool ok = k0 + kr < n;
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(ok ? va[r] : 0.0, ok ? vb[r] : 0.0, acc, 0, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) G[i0 + kr + 4 * q][j0 + cc] = acc[q];
    }
    __syncthreads();
    refl_T_recur(G, tau, kb, nb, tf, b);
}

__global__ void __launch_bounds__(1024) k_refl_T(const double* __restrict__ refl, const double* __restrict__ tau, int n,
                                                 int lda, double* __restrict__ tf, const u32* xcd, u32* vcount)
{
    if (!xcd) {
        refl_T_item(refl, tau, n, lda, tf, (int)blockIdx.x);
        return;
    }
    const int nblk = (n - 2 + BT_NB - 1) / BT_NB;
    int role = 0;
    for (int b; (b = xcd_next(xcd, vcount, nblk, &role)) >= 0;) refl_T_item(refl, tau, n, lda, tf, b);
}

// ---------------------------------------------------------------------------
// 3. cluster re-orthogonalisation, normalisation, sign, transposed store
__global__ void __launch_bounds__(FIN_T) k_eig_finish(double* Zq, int n, int lda, int k, const double* W,
                                                     const double* tnorm_p, double* Z)
{
    __shared__ double red[FIN_W];
    __shared__ int ired[FIN_W];
    __shared__ double sbest[FIN_W];
    const int tid = threadIdx.x, lane = tid & 63, wv = scc_wave_id();
    const double tnorm = tnorm_p[0];
    for (int qq = 0; qq < k; ++qq) {  // vectors live in global memory (one workgroup)
        double* z = Zq + (size_t)qq * lda;
        for (int rr = qq - 1; rr >= 0 && fabs(W[rr] - W[rr + 1]) <= 1e-3 * tnorm; --rr) {
            const double* zr = Zq + (size_t)rr * lda;
            double s = 0.0;
            for (int i = tid; i < n; i += FIN_T) s += zr[i] * z[i];
            s = block_sum<FIN_W>(s, red);
            for (int i = tid; i < n; i += FIN_T) z[i] -= s * zr[i];
            __syncthreads();
        }
        double s = 0.0;
        for (int i = tid; i < n; i += FIN_T) s += z[i] * z[i];
        s = block_sum<FIN_W>(s, red);
        const double inv = 1.0 / sqrt(s);
        // deterministic sign: largest-magnitude component positive (lowest index on ties)
        double best = -1.0;
        int bi = 0;
        for (int i = tid; i < n; i += FIN_T) {
            const double v = fabs(z[i]);
            if (v > best) {
                best = v;
                bi = i;
            }
        }
        for (int m = 32; m >= 1; m >>= 1) {
            const double ob = __shfl_xor(best, m, 64);
            const int oi = __shfl_xor(bi, m, 64);
            if (ob > best || (ob == best && oi < bi)) {
                best = ob;
                bi = oi;
            }
        }
        if (lane == 0) {
            sbest[wv] = best;
            ired[wv] = bi;
        }
        __syncthreads();
        best = sbest[0];
        bi = ired[0];
        for (int w = 1; w < FIN_W; ++w)
            if (sbest[w] > best || (sbest[w] == best && ired[w] < bi)) {
                best = sbest[w];
                bi = ired[w];
            }
        const double sg = (z[bi] < 0.0) ? -inv : inv;
        __syncthreads();
        for (int i = tid; i < n; i += FIN_T) z[i] *= sg;
        __syncthreads();
    }
    for (int i = tid; i < n * 16; i += FIN_T) {
        const int u = i >> 4, q = i & 15;
        Z[i] = (q < k) ? Zq[(size_t)q * lda + u] : 0.0;
    }
}

// Back-transformation of all k eigenvectors at once, one workgroup: the
// vectors and one block of BT_NB reflectors at a time in LDS (the block is
// read from global memory once, with every load in flight, instead of once
// per eigenpair workgroup behind dependent waits), then per block
// W = V^T Y, W <- T W, Y <- Y - V W (compact WY, last block first).  Used when
// (k + BT_NB) n doubles fit the LDS; k_tri_vectors then leaves its vector
// untransformed (bt_none).
#define TB_T 1024
__global__ void __launch_bounds__(TB_T) k_tri_back(double* __restrict__ Zq, int n, int lda, int k,
                                                   const double* __restrict__ refl, const double* __restrict__ tf,
                                                   u64* __restrict__ stamps)
{
    const bool stmp = stamps && threadIdx.x == 0;  // diagnostic: per-phase cycles
    u64 ph[5] = {0, 0, 0, 0, 0}, tq = stmp ? clock64() : 0;
    auto mark = [&](int i) {
        if (stmp) {
            const u64 t = clock64();
            ph[i] += t - tq;
            tq = t;
        }
    };
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double* Y = sm;                          // [k][n]
    double* Vs = Y + (size_t)k * n;          // [BT_NB][n]: v_i at rows kb+1 .. n-1 (zero at rows <= kb+i)
    __shared__ double W[BT_NB][16], W2[BT_NB][16], Ts[BT_NB][BT_NB];  // Ts: zero below the diagonal and past nb
    __shared__ double Wp[4][BT_NB][16];  // per-wave partials of V^T Y
    const int tid = threadIdx.x, lane = tid & 63, wv = scc_wave_id();
    for (int x0 = 0; x0 < k * n; x0 += 8 * TB_T) {
        double yv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int x = min(x0 + u * TB_T + tid, k * n - 1);
            yv[u] = Zq[(size_t)(x / n) * lda + x % n];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int x = x0 + u * TB_T + tid;
            if (x < k * n) Y[x] = yv[u];
        }
    }
    const int nr = n - 2;
    mark(4);
    // block b's reflectors and T factor are loaded into registers while block
    // b + 1 is applied (SB clamped unconditional loads per thread, in flight
    // across the block's compute), then stored to LDS at the top of block b
    constexpr int SB = 12;
    double vv[SB], tv = 0.0;
    auto fetch = [&](int b) {
        const int kb = b * BT_NB, nb = min(BT_NB, nr - kb), m0 = kb + 1, m = n - m0;
#pragma unroll
        for (int u = 0; u < SB; ++u) {
            const int x = min(u * TB_T + tid, BT_NB * m - 1);
            const int i = x / m, j = m0 + x % m;
            vv[u] = refl[(size_t)(kb + min(i, nb - 1)) * lda + j];
        }
        tv = tf[(size_t)b * BT_NB * BT_NB + min(tid, BT_NB * BT_NB - 1)];
    };
    const int nblk = nr > 0 ? (nr + BT_NB - 1) / BT_NB : 0;
    if (nblk > 0) fetch(nblk - 1);
    for (int b = nblk - 1; b >= 0; --b) {
        const int kb = b * BT_NB, nb = min(BT_NB, nr - kb), m0 = kb + 1, m = n - m0;
        __syncthreads();  // the previous block's Y update is complete before Vs is reused
        mark(3);
#pragma unroll
        for (int u = 0; u < SB; ++u) {
            const int x = u * TB_T + tid;
            if (x < BT_NB * m) {
                const int i = x / m, j = m0 + x % m;
                Vs[x] = (i < nb && j > kb + i) ? vv[u] : 0.0;
            }
        }
        if (tid < BT_NB * BT_NB) Ts[tid / BT_NB][tid % BT_NB] = tv;
        __syncthreads();
        if (b > 0) fetch(b - 1);
        mark(0);
        // W = V^T Y on fp64 MFMA (16x16x4: A = V, 16 reflectors x 4 rows; B =
        // Y^T, 4 rows x 16 vectors): waves 0-3 the reflectors 0-15, waves 4-7
        // 16-31, each wave every 4th group of 4 rows; partials summed below in
        // wave order (deterministic).  Rows of Vs past nb are zero, vectors
        // past k are masked to zero.
        if (wv < 8) {
            const int tile = wv >> 2, part = wv & 3, qv = lane & 15;
            const double* va = Vs + (size_t)(tile * 16 + (lane & 15)) * m;
            const double* yb = Y + (size_t)min(qv, k - 1) * n + m0;
            typedef double d4v __attribute__((ext_vector_type(4)));
            d4v acc = {0.0, 0.0, 0.0, 0.0};
            for (int j0 = part * 4; j0 < m; j0 += 16) {
                const int j = j0 + (lane >> 4), jc = min(j, m - 1);
                const double av = va[jc], yv = yb[jc];  // unconditional (clamped) loads, then masks
                const double a = (j < m) ? av : 0.0;
                const double bq = (j < m && qv < k) ? yv : 0.0;
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bq, acc, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) Wp[part][tile * 16 + (lane >> 4) + 4 * r][lane & 15] = acc[r];
        }
        __syncthreads();
        if (tid < BT_NB * 16) {
            const int i = tid >> 4, q = tid & 15;
            W[i][q] = ((Wp[0][i][q] + Wp[1][i][q]) + Wp[2][i][q]) + Wp[3][i][q];
        }
        if (tid < BT_NB * 16) {  // W2 = T W (T upper triangular, zero past nb)
            const int i = tid >> 4, q = tid & 15;
            double s = 0.0;
#pragma unroll
            for (int c = 0; c < BT_NB; ++c) s = fma(Ts[i][c], W[c][q], s);
            W2[i][q] = s;
        }
        __syncthreads();
        mark(2);
        // Y -= V W2 on fp64 MFMA: output tile = 16 rows of Y^T x 16 vectors,
        // A[j][i] = V[i][j], B = W2 (32 x 16), K = the block's 32 reflectors
        {
            typedef double d4v __attribute__((ext_vector_type(4)));
            const int ntile = (m + 15) / 16;
            for (int t = wv; t < ntile; t += TB_T / 64) {
                d4v acc = {0.0, 0.0, 0.0, 0.0};
                const int jr = t * 16 + (lane & 15);
#pragma unroll
                for (int i0 = 0; i0 < BT_NB; i0 += 4) {
                    const int i = i0 + (lane >> 4);
                    const double av = Vs[(size_t)i * m + min(jr, m - 1)];
                    const double a = (jr < m) ? av : 0.0;
                    const double bq = W2[i][lane & 15];
                    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bq, acc, 0, 0, 0);
                }
                // D[row][col]: row = (lane >> 4) + 4 r indexes the 16 rows of the
                // A tile (rows of Y^T = positions j), col = lane & 15 the vector q
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int j = t * 16 + (lane >> 4) + 4 * r, q = lane & 15;
                    if (j < m && q < k) Y[(size_t)q * n + m0 + j] -= acc[r];
                }
            }
        }
    }
    __syncthreads();
    mark(3);
    for (int x = tid; x < k * n; x += TB_T) Zq[(size_t)(x / n) * lda + x % n] = Y[x];
    if (stmp)
        for (int i = 0; i < 5; ++i) stamps[12 + i] = ph[i];
}

// Explicit Q = H_0 H_1 ... H_{n-3} = B_0 B_1 ... B_{m-1} (B_b = I - V_b T_b
// V_b^T, the compact-WY blocks of k_refl_T), formed on the side stream while
// k_tri_vectors finds the tridiagonal's eigenvectors: the rows of Q evolve
// independently (q_r^T <- q_r^T B_b, block by block from e_r^T), so each
// workgroup owns QF_R rows in LDS and needs no other workgroup.  Per block:
// S = Q_rows V_b and Q_rows -= (S T_b) V_b^T, both on fp64 MFMA 16x16x4.
// The back-transformation is then one product Z = Q Y (k_apply_q) instead
// of the one-workgroup, block-sequential k_tri_back on the critical path.
#define QF_R 16
#define QF_T 256
#define QF_MAXC 6  // 64-column chunks of a reflector row held in registers (n <= 384)
static_assert(8 * (QF_T / 64) == BT_NB, "k_form_q stages BT_NB reflector rows, QF_VB per wave");
__global__ void __launch_bounds__(QF_T) k_form_q(const double* __restrict__ refl, const double* __restrict__ tf, int n,
                                                 int lda, double* __restrict__ Q)
{
    typedef double d4v __attribute__((ext_vector_type(4)));
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double* Qs = sm;                     // [QF_R][n]
    double* Vs = Qs + (size_t)QF_R * n;  // [BT_NB][n]: v_i over all rows (zero at rows <= kb + i)
    __shared__ double Sp[2][QF_R][BT_NB];  // K-halves of Q_rows V_b
    __shared__ double S2[QF_R][BT_NB];     // (Q_rows V_b) T_b
    __shared__ double Ts[BT_NB][BT_NB];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int r0 = blockIdx.x * QF_R;
    for (int r = wv; r < QF_R; r += QF_T / 64)
        for (int j = lane; j < n; j += 64) Qs[(size_t)r * n + j] = (r0 + r == j) ? 1.0 : 0.0;
    const int nr = n - 2, nblk = nr > 0 ? (nr + BT_NB - 1) / BT_NB : 0;
    // V_b's rows: wave w stages rows i = w + 4 u, lanes over j.  Block b + 1's
    // values are loaded into registers (clamped, unconditional) while block b
    // is applied, and stored to LDS (masked) at the top of the next iteration,
    // so the reflector fetch latency is paid once instead of once per block
    constexpr int QF_VB = 8;
    double pf[QF_MAXC][QF_VB];
    auto fetch = [&](int b) {
        const int kb = b * BT_NB, nb = min(BT_NB, nr - kb);
#pragma unroll
        for (int c = 0; c < QF_MAXC; ++c) {
            const int jc = min(c * 64 + lane, n - 1);
#pragma unroll
            for (int u = 0; u < QF_VB; ++u)
                pf[c][u] = refl[(size_t)(kb + min(wv + (QF_T / 64) * u, nb - 1)) * lda + jc];
        }
    };
    if (nblk > 0) fetch(0);
    for (int b = 0; b < nblk; ++b) {
        const int kb = b * BT_NB, nb = min(BT_NB, nr - kb), m0 = kb + 1;
        __syncthreads();  // the previous block's update of Qs is complete before Vs is reused
#pragma unroll
        for (int c = 0; c < QF_MAXC; ++c) {
            const int j = c * 64 + lane;
#pragma unroll
            for (int u = 0; u < QF_VB; ++u) {
                const int i = wv + (QF_T / 64) * u;
                if (j < n) Vs[(size_t)i * n + j] = (i < nb && j > kb + i) ? pf[c][u] : 0.0;
            }
        }
        for (int x = tid; x < BT_NB * BT_NB; x += QF_T) (&Ts[0][0])[x] = tf[(size_t)b * BT_NB * BT_NB + x];
        __syncthreads();
        if (b + 1 < nblk) fetch(b + 1);
        {  // S = Q_rows V_b^T-side: 16 rows x 32 reflectors, K = the rows j >= m0; wave
            // w: reflector tile w & 1, K half w >> 1
            const int tile = wv & 1, half = wv >> 1;
            const double* qa = Qs + (size_t)(lane & 15) * n;
            const double* vb = Vs + (size_t)(tile * 16 + (lane & 15)) * n;
            d4v acc = {0.0, 0.0, 0.0, 0.0};
            for (int j0 = m0 + 4 * half; j0 < n; j0 += 8) {
                const int j = j0 + (lane >> 4), jc = min(j, n - 1);
                const double a = qa[jc], bq = vb[jc];
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(j < n ? a : 0.0, j < n ? bq : 0.0, acc, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) Sp[half][(lane >> 4) + 4 * r][tile * 16 + (lane & 15)] = acc[r];
        }
        __syncthreads();
        for (int x = tid; x < QF_R * BT_NB; x += QF_T) {  // S2 = S T (T upper triangular, zero past nb)
            const int r = x / BT_NB, i = x % BT_NB;
            double sacc = 0.0;
#pragma unroll 8
            for (int c = 0; c < BT_NB; ++c) sacc = fma(Sp[0][r][c] + Sp[1][r][c], Ts[c][i], sacc);
            S2[r][i] = sacc;
        }
        __syncthreads();
        // Q_rows[:, j] -= S2 V_b[:, j] for j >= m0: 16 x 16 tiles over j, K = 32 reflectors
        for (int t = wv; t * 16 < n - m0; t += QF_T / 64) {
            const int jb = m0 + t * 16;
            d4v acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int i0 = 0; i0 < BT_NB; i0 += 4) {
                const int i = i0 + (lane >> 4), j = jb + (lane & 15);
                const double a = S2[lane & 15][i];  // A[row r][k i]
                const double bv = Vs[(size_t)i * n + min(j, n - 1)];
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, j < n ? bv : 0.0, acc, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = (lane >> 4) + 4 * r, j = jb + (lane & 15);
                if (j < n) Qs[(size_t)row * n + j] -= acc[r];
            }
        }
    }
    __syncthreads();
    for (int r = wv; r < QF_R; r += QF_T / 64)
        if (r0 + r < n)
            for (int j = lane; j < n; j += 64) Q[(size_t)(r0 + r) * lda + j] = Qs[(size_t)r * n + j];
}

// Z = Q Y: the back-transformed eigenvectors, Zt[q][r] = sum_j Q[r][j] Y[q][j]
// (Y = the tridiagonal's eigenvectors, [16][lda]); one 16-row tile of Z^T per
// workgroup (one wave), K = n in steps of 4
__global__ void __launch_bounds__(64) k_apply_q(const double* __restrict__ Q, const double* __restrict__ Y, int n,
                                                int lda, int k, double* __restrict__ Zt)
{
    typedef double d4v __attribute__((ext_vector_type(4)));
    const int lane = threadIdx.x, r0 = blockIdx.x * 16;
    const int r = min(r0 + (lane & 15), n - 1), q = lane & 15;
    d4v acc = {0.0, 0.0, 0.0, 0.0};
    const double* qrow = Q + (size_t)r * lda;
    const double* ycol = Y + (size_t)min(q, k - 1) * lda;
    for (int j0 = 0; j0 < n; j0 += 32) {  // 8 MFMA steps, their 16 loads in flight together
        double a[8], bq[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int jc = min(j0 + 4 * u + (lane >> 4), n - 1);
            a[u] = qrow[jc];
            bq[u] = ycol[jc];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int j = j0 + 4 * u + (lane >> 4);
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(j < n ? a[u] : 0.0, (j < n && q < k) ? bq[u] : 0.0, acc, 0,
                                                       0, 0);
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int rr = r0 + (lane >> 4) + 4 * i;
        if (rr < n && q < k) Zt[(size_t)q * lda + rr] = acc[i];
    }
}

static size_t form_q_lds(int n) { return sizeof(double) * (size_t)(QF_R + BT_NB) * n; }

// dynamic LDS of k_tri_back (its static arrays take 32 KB more)
static size_t tri_back_lds(int n, int k) { return sizeof(double) * ((size_t)k + BT_NB) * n; }

// Same result with the k vectors in LDS (k n doubles <= 160 KB): vectors
// with no cluster predecessor ("heads", almost all of them) are normalised
// and signed in parallel, one wave each, with no workgroup barrier; the rest
// follow in order with block-wide Gram-Schmidt against their predecessors.
// Reduction orders are fixed (bitwise deterministic).
__device__ inline void fin_wave_finalize(double* z, int n, int lane)
{
    double ss = 0.0, best = -1.0;
    int bi = 0;
    for (int i = lane; i < n; i += 64) {
        const double v = z[i];
        ss = fma(v, v, ss);
        if (fabs(v) > best) {
            best = fabs(v);
            bi = i;
        }
    }
    ss = wave_sum_d(ss);
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const double ob = __shfl_xor(best, m, 64);
        const int oi = __shfl_xor(bi, m, 64);
        if (ob > best || (ob == best && oi < bi)) {
            best = ob;
            bi = oi;
        }
    }
    const double inv = 1.0 / sqrt(ss);
    const double sg = (z[bi] < 0.0) ? -inv : inv;
    for (int i = lane; i < n; i += 64) z[i] *= sg;
}

__global__ void __launch_bounds__(FIN_T) k_eig_finish_lds(const double* Zq, int n, int lda, int k, const double* W,
                                                         const double* tnorm_p, double* Z)
{
    extern __shared__ __attribute__((aligned(16))) double zl[];  // [k][n]
    __shared__ double red[FIN_W];
    const int tid = threadIdx.x, lane = tid & 63, wv = scc_wave_id();
    const double tnorm = tnorm_p[0];
    for (int x = tid; x < k * n; x += FIN_T) zl[x] = Zq[(size_t)(x / n) * lda + x % n];
    __syncthreads();
    auto head = [&](int q) { return q == 0 || !(fabs(W[q - 1] - W[q]) <= 1e-3 * tnorm); };
    if (wv < k && head(wv)) fin_wave_finalize(zl + (size_t)wv * n, n, lane);
    __syncthreads();
    for (int q = 1; q < k; ++q) {
        if (head(q)) continue;
        double* z = zl + (size_t)q * n;
        for (int rr = q - 1; rr >= 0 && fabs(W[rr] - W[rr + 1]) <= 1e-3 * tnorm; --rr) {
            const double* zr = zl + (size_t)rr * n;
            double s = 0.0;
            for (int i = tid; i < n; i += FIN_T) s += zr[i] * z[i];
            s = block_sum<FIN_W>(s, red);
            for (int i = tid; i < n; i += FIN_T) z[i] -= s * zr[i];
            __syncthreads();
        }
        if (wv == 0) fin_wave_finalize(z, n, lane);
        __syncthreads();
    }
    for (int i = tid; i < n * 16; i += FIN_T) {
        const int u = i >> 4, q = i & 15;
        Z[i] = (q < k) ? zl[(size_t)q * n + u] : 0.0;
    }
}

static void launch_eig_finish(double* Zq, int n, int lda, int k, const double* W, const double* tnorm, double* Z,
                              hipStream_t st)
{
    const size_t lds = sizeof(double) * (size_t)k * n;
    if (lds <= 150 * 1024) {
        scc_set_lds((const void*)k_eig_finish_lds, (int)lds);
        hipLaunchKernelGGL(k_eig_finish_lds, dim3(1), dim3(FIN_T), lds, st, Zq, n, lda, k, W, tnorm, Z);
    } else {
        hipLaunchKernelGGL(k_eig_finish, dim3(1), dim3(FIN_T), 0, st, Zq, n, lda, k, W, tnorm, Z);
    }
}

// ---------------------------------------------------------------------------
// host side
static int eig_local_env()
{
    const char* env = getenv("SCC_EIG_XCD");
    return (env && *env) ? atoi(env) : -1;
}

struct EigLayout {
    size_t d, e, tau, tnorm, flags, pg, rg, dg, zq, zt, refl, tf, lu, work, q, total;
};

static EigLayout eig_layout(int n, int lda, int k, int nwg, bool rows_lds, bool lu_lds)
{
    EigLayout L;
    size_t o = 0;
    auto take = [&](size_t cnt) {
        const size_t at = o;
        o += (cnt + 31) & ~(size_t)31;  // 256-B aligned pieces
        return at;
    };
    L.d = take(n);
    L.e = take(n);
    L.tau = take(n);
    L.tnorm = take(1);
    L.flags = take(8);  // counter, err, XCD registration [3], follow-up counters [6] (u32 in doubles' space)
    L.pg = take(4 * (size_t)lda);  // u64 granules occupy doubles' space
    L.rg = take(4 * (size_t)lda);
    L.dg = take(4 * EIG_MAX_WG * TRI_W);  // one partial per wave agent
    L.zq = take(16 * (size_t)lda);
    L.zt = take(16 * (size_t)lda);
    L.refl = take((size_t)n * lda);
    L.tf = take((size_t)((n + BT_NB) / BT_NB) * BT_NB * BT_NB);
    L.lu = lu_lds ? o : take((size_t)16 * 6 * n);
    const int R = (n + nwg - 1) / nwg;
    // XCD-local mode: fewer workgroups may register than planned -> room for all rows
    L.work = take(((size_t)n + 4 * 64) * n);  // row store of the HBM fall-backs (any participant count)
    L.q = take((size_t)n * lda);              // explicit Q of the reflectors (k_form_q)
    L.total = o;
    (void)k;
    return L;
}

static size_t tri_lds_bytes(int n, int R, bool rows_lds)
{
    return sizeof(double) * (5 * (size_t)n + 64 + EIG_MAX_WG + (rows_lds ? (size_t)R * n : 0));
}

// register row slots (64 columns each) of k_tridiag for this n, 0: rows in LDS / HBM only
static int tri_nj(int n) { return n <= 384 ? 6 : (n <= 512 ? 8 : (n <= 896 ? 14 : 0)); }
// own rows per workgroup k_tridiag keeps in registers
static int tri_reg_rows(int n) { return tri_nj(n) ? TRI_W * TRI_MR : 0; }

static int eig_nwg(int n)
{
    const int cus = scc_device_cus(64);
    const char* env = getenv("SCC_EIG_NWG");
    int nwg = (env && *env) ? atoi(env) : (n + 9) / 10;
    nwg = nwg < 8 ? 8 : nwg;
    if (nwg > cus) nwg = cus;
    if (nwg > EIG_MAX_WG) nwg = EIG_MAX_WG;
    if (nwg > n) nwg = n;
    if (nwg < 1) nwg = 1;
    return nwg;
}

// One XCD (32 CUs, hand-offs through its L2) while the rows fit those CUs'
// LDS; beyond that the rows spread over more XCDs and stay in LDS, which
// measured faster than one XCD with rows in HBM (n = 845: 7.1 vs 13.0 ms;
// n = 1000: 9.3 vs 21.3 ms).  SCC_EIG_XCD=0/1 forces either.
static bool eig_local(int n)
{
    const int env = eig_local_env();
    if (env >= 0) return env != 0;
    int nwg = eig_nwg(n);
    if (nwg > 32) nwg = 32;
    return tri_lds_bytes(n, std::max((n + nwg - 1) / nwg - tri_reg_rows(n), 0), true) <= EIG_LDS_MAX;
}

static void eig_plan(int n, int& nwg, bool& rows_lds, bool& lu_lds)
{
    nwg = eig_nwg(n);
    if (eig_local(n) && nwg > 32) nwg = 32;  // one XCD holds 32 CUs
    const int R = std::max((n + nwg - 1) / nwg - tri_reg_rows(n), 0);  // rows outside registers
    rows_lds = tri_lds_bytes(n, R, true) <= EIG_LDS_MAX;
    lu_lds = sizeof(double) * 10 * (size_t)n <= EIG_LDS_MAX;
}

// A non-blocking side stream (and fork / join events) per device for work
// that overlaps the eigensolver's main chain; created once, never destroyed
// (process lifetime, like the HIP runtime's own streams).
static void side_stream(hipStream_t* s, hipEvent_t* fork_ev, hipEvent_t* join_ev)
{
    static hipStream_t ss[64] = {};
    static hipEvent_t fe[64] = {}, je[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
        *s = nullptr;
        return;
    }
    if (!ss[dev]) {
        if (hipStreamCreateWithFlags(&ss[dev], hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&fe[dev], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&je[dev], hipEventDisableTiming) != hipSuccess) {
            ss[dev] = nullptr;
            *s = nullptr;
            return;
        }
    }
    *s = ss[dev];
    *fork_ev = fe[dev];
    *join_ev = je[dev];
}

extern "C" size_t scc_si_scratch_doubles(int n);
extern "C" int scc_si_wanted(int n);
extern "C" int scc_fsi_wanted(int n);
extern "C" size_t scc_fsi_scratch_doubles(int n);
extern "C" void scc_fsi_forget(const void* p, size_t bytes);
extern "C" hipError_t scc_eigen_fsi(const double* C, int n, int ldc, int k, double* scr, double* Z, double* Wout,
                                    int* ok, unsigned long long key, hipStream_t st);
extern "C" hipError_t scc_eigen_si(const double* C, int n, int ldc, int k, double* scr, double* Z, double* Wout,
                                   int* ok, hipStream_t st);

// which solver answered the calling thread's last scc_launch_eigen_topk:
// 0 direct, 1 subspace iteration, 2 filtered subspace iteration (a launch per
// step), 3 the same in the persistent engine, 4 the direct solver rerun
// without cooperative waits after a hand-off time-out (diagnostic)
static thread_local int g_eig_last_path = 0;
extern "C" SCC_API int scc_diag_eig_last_path() { return g_eig_last_path; }

// scratch of the direct solver alone
extern "C" size_t scc_eigen_topk_scratch_direct(int n, int lda, int k)
{
    int nwg;
    bool rl, ll;
    eig_plan(n, nwg, rl, ll);
    return eig_layout(n, lda, k, nwg, rl, ll).total;
}

// direct solver + (for large n) the subspace iteration tried first (scc_subspace.hip)
extern "C" size_t scc_eigen_scratch_doubles(int n, int lda, int k)
{
    size_t extra = 0;
    if (scc_fsi_wanted(n)) extra = scc_fsi_scratch_doubles(n);
    if (scc_si_wanted(n)) extra = std::max(extra, scc_si_scratch_doubles(n));
    return scc_eigen_topk_scratch_direct(n, lda, k) + extra;
}

// A: n x n symmetric (full), row-major, lda (read only).  scratch: see
// scc_eigen_scratch_doubles.  Z: n x 16 out, W: k out (descending).
// *err_dev (device u32 inside scratch) is set to 1 if a hand-off timed out
// even on the non-cooperative rerun.  key: the caller's identity for the
// filtered iteration's graph cache (context serial and workspace generation;
// 0: no graph).  marks (optional): 6 events recorded before/after each of the
// three launches (a null entry is skipped).
// set by eig_direct: whether its launches wait on co-resident workgroups
// (more than one tridiagonalisation workgroup, or follow-ups pinned to its XCD)
static thread_local bool t_eig_coop = true;

static hipError_t eig_direct(const double* A, int n, int lda, int k, double* scratch, double* Z, double* W,
                             hipEvent_t* marks, unsigned long long* stamps, bool safe, hipStream_t st);

extern "C" hipError_t scc_launch_eigen_topk(const double* A, int n, int lda, int k, double* scratch, double* Z,
                                            double* W, unsigned int** err_dev, int* nwg_out, hipEvent_t* marks,
                                            unsigned long long* stamps, unsigned long long key, hipStream_t st)
{
    int nwg;
    bool rows_lds, lu_lds;
    eig_plan(n, nwg, rows_lds, lu_lds);
    const EigLayout L = eig_layout(n, lda, k, nwg, rows_lds, lu_lds);
    u32* flags = (u32*)(scratch + L.flags);
    if (err_dev) *err_dev = flags + 1;
    if (nwg_out) *nwg_out = nwg;
    hipError_t e = hipMemsetAsync(flags, 0, 64, st);  // counter, err, XCD pick [3], follow-up counters [6]
    if (e != hipSuccess) return e;
    g_eig_last_path = 0;
    if (scc_fsi_wanted(n)) {
        // |U| >= 128: Chebyshev-filtered subspace iteration first (scc_subspace.hip),
        // accepted only when every test passes (else the direct solver below)
        if (marks && marks[0]) hipEventRecord(marks[0], st);
        int ok = 0;
        e = scc_eigen_fsi(A, n, lda, k, scratch + scc_eigen_topk_scratch_direct(n, lda, k), Z, W, &ok, key, st);
        if (e != hipSuccess) return e;
        if (ok) {
            g_eig_last_path = ok == 2 ? 3 : 2;  // 3: the persistent engine ran the filter loop
            if (marks)
                for (int m = 1; m < 6; ++m)
                    if (marks[m]) hipEventRecord(marks[m], st);
            return hipSuccess;
        }
        e = hipMemsetAsync(flags, 0, 64, st);
        if (e != hipSuccess) return e;
    } else if (scc_si_wanted(n)) {
        // large |U|: block subspace iteration first; accepted only when every
        // Ritz residual passes (else the direct solver below runs)
        if (marks && marks[0]) hipEventRecord(marks[0], st);
        int ok = 0;
        e = scc_eigen_si(A, n, lda, k, scratch + scc_eigen_topk_scratch_direct(n, lda, k), Z, W, &ok, st);
        if (e != hipSuccess) return e;
        if (ok) {
            g_eig_last_path = 1;
            if (marks)
                for (int m = 1; m < 6; ++m)
                    if (marks[m]) hipEventRecord(marks[m], st);
            return hipSuccess;
        }
    }
    if ((e = eig_direct(A, n, lda, k, scratch, Z, W, marks, stamps, false, st)) != hipSuccess) return e;
    // The direct solver's tridiagonalisation hands off between co-resident
    // workgroups (bounded polls).  On a shared device they may not all become
    // resident: the time-out flag is read here, and the same solve reruns on
    // ONE workgroup with no cooperative wait (slower, same algorithm).  A plan
    // of one workgroup without XCD pinning waits on nobody: no read, the call
    // stays asynchronous.
    // SCC_EIG_FORCE_TIMEOUT=1 (tests) takes the rerun as if the flag were set.
    const char* ft = getenv("SCC_EIG_FORCE_TIMEOUT");
    const bool forced = ft && atoi(ft);
    if (!t_eig_coop && !forced) return hipSuccess;
    u32 herr = 0;
    if ((e = hipMemcpyAsync(&herr, flags + 1, sizeof(u32), hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
    if (herr || forced) {
        if (getenv("SCC_EIG_SI_LOG")) fprintf(stderr, "[scc eig] direct solver hand-off timed out: one-workgroup rerun\n");
        if ((e = hipMemsetAsync(flags, 0, 64, st)) != hipSuccess) return e;
        if ((e = eig_direct(A, n, lda, k, scratch, Z, W, nullptr, nullptr, true, st)) != hipSuccess) return e;
        g_eig_last_path = 4;
    }
    return hipSuccess;
}

// The direct solver: k_tridiag, then k_tri_vectors beside the reflectors'
// T factors / explicit Q on the per-device side stream, the back-transform
// and k_eig_finish.  safe: one workgroup, rows anywhere, no XCD pinning and no
// co-resident waits (the rerun after a hand-off time-out).
static hipError_t eig_direct(const double* A, int n, int lda, int k, double* scratch, double* Z, double* W,
                             hipEvent_t* marks, unsigned long long* stamps, bool safe, hipStream_t st)
{
    // the side stream and its fork / join events are shared by every context
    // on a device: one host thread at a time enqueues this sequence on a
    // device, so another context cannot re-record fork_ev / join_ev between
    // our record and the wait on it (launches are asynchronous: the lock is
    // held while they are queued, not while they run)
    static std::mutex dev_mu[64];
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> guard(dev_mu[(dev >= 0 && dev < 64) ? dev : 0]);
    int nwg;
    bool rows_lds, lu_lds;
    eig_plan(n, nwg, rows_lds, lu_lds);
    const EigLayout L = eig_layout(n, lda, k, nwg, rows_lds, lu_lds);
    u32* flags = (u32*)(scratch + L.flags);
    hipError_t e;
    if (safe) {
        nwg = 1;
        rows_lds = tri_lds_bytes(n, std::max(n - tri_reg_rows(n), 0), true) <= EIG_LDS_MAX;
    }
    // granule tags restart at 1 every launch
    e = hipMemsetAsync(scratch + L.pg, 0, sizeof(double) * (L.zq - L.pg), st);
    if (e != hipSuccess) return e;
    TriArgs t;
    t.A = A;
    t.n = n;
    t.lda = lda;
    t.nwg = nwg;
    t.rows_lds = rows_lds ? 1 : 0;
    t.d = scratch + L.d;
    t.e = scratch + L.e;
    t.tau = scratch + L.tau;
    t.refl = scratch + L.refl;
    t.pg = (u64*)(scratch + L.pg);
    t.rg = (u64*)(scratch + L.rg);
    t.dg = (u64*)(scratch + L.dg);
    t.work = scratch + L.work;
    t.counter = flags;
    t.reg = flags + 2;
    t.xcd_local = (!safe && eig_local(n)) ? 1 : 0;
    t.stamps = stamps;
    t.err = flags + 1;
    const int R = (n + nwg - 1) / nwg;
    // at least 82 KB so that every workgroup has a CU of its own
    size_t lds = tri_lds_bytes(n, std::max(R - tri_reg_rows(n), 0), rows_lds);
    if (lds < 82 * 1024) lds = 82 * 1024;
    t.lds_rows_cap = rows_lds ? (int)((lds / sizeof(double) - (5 * (size_t)n + 64 + EIG_MAX_WG)) / n) : 0;
    t_eig_coop = nwg > 1 || t.xcd_local;
    if (marks && marks[0]) hipEventRecord(marks[0], st);
    const int cus = scc_device_cus(64);
    {
        // register rows for n <= 896 (6, 8 or 14 column slots per lane; the rest
        // of a workgroup's rows in LDS), else LDS / HBM rows
        const int nj = tri_nj(n);
        const void* fn;
        if (t.xcd_local)
            fn = nj == 6    ? (const void*)(k_tridiag<true, 6>)
                 : nj == 8  ? (const void*)(k_tridiag<true, 8>)
                 : nj == 14 ? (const void*)(k_tridiag<true, 14>)
                            : (const void*)(k_tridiag<true, 0>);
        else
            fn = nj == 6    ? (const void*)(k_tridiag<false, 6>)
                 : nj == 8  ? (const void*)(k_tridiag<false, 8>)
                 : nj == 14 ? (const void*)(k_tridiag<false, 14>)
                            : (const void*)(k_tridiag<false, 0>);
        scc_set_lds(fn, (int)lds);
        const dim3 grid(t.xcd_local ? std::min(8 * nwg, cus) : nwg);
        void* args[] = {&t};
        e = hipLaunchKernel(fn, grid, dim3(TRI_T), args, lds, st);
        if (e != hipSuccess) return e;
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (marks && marks[1]) hipEventRecord(marks[1], st);
    VecArgs v{};
    v.d = t.d;
    v.e = t.e;
    v.tau = t.tau;
    v.refl = t.refl;
    v.n = n;
    v.lda = lda;
    v.k = k;
    v.lu_lds = lu_lds ? 1 : 0;
    {
        const char* te = getenv("SCC_EIG_TWIST");  // 0: inverse iteration for every eigenpair
        v.twist = (te && *te && atoi(te) == 0) ? 0 : 1;
    }
    v.lu = scratch + L.lu;
    v.Zq = scratch + L.zq;
    v.W = W;
    v.tnorm = scratch + L.tnorm;
    v.stamps = stamps;
    v.tf = scratch + L.tf;
    // follow-up kernels on the tridiagonalisation's XCD (its reflectors are in that L2)
    // one item per workgroup with a co-resident wait when 8 x k workgroups fit
    // (measured at config B: eig_vec 0.37 ms anywhere, 0.42 claim loop, 0.32 wait)
    constexpr int pin_mode = 2;
    const bool pin = !safe && t.xcd_local != 0 && pin_mode != 0;
    v.wait = pin_mode == 2;
    v.xcd = pin && (pin_mode == 1 || 8 * k <= 256) ? t.reg : nullptr;  // wait needs co-residency
    v.vcount = flags + 5;
    v.err = flags + 1;
    const size_t vlds = sizeof(double) * (lu_lds ? 10 : 4) * (size_t)n;
    scc_set_lds((const void*)k_tri_vectors, (int)vlds);
    // Back-transformation: the explicit Q formed on a side stream beside
    // k_tri_vectors, then Z = Q Y (SCC_EIG_BT=2, the default where its LDS
    // fits); SCC_EIG_BT=1: one workgroup applying the reflector blocks to all
    // k vectors after k_tri_vectors (k_tri_back); 0: per eigenpair, inside
    // k_tri_vectors
    const char* bt_env = getenv("SCC_EIG_BT");
    const int bt_mode = (bt_env && *bt_env) ? atoi(bt_env) : 2;
    const bool back_fits = n > 2 && n - 1 <= 12 * TB_T / BT_NB && tri_back_lds(n, k) + 33 * 1024 <= EIG_LDS_MAX;
    const bool q_form = n > 2 && bt_mode == 2 && form_q_lds(n) + 24 * 1024 <= EIG_LDS_MAX &&  // + its static arrays
                        n <= 64 * QF_MAXC;
    const bool bt_one = !q_form && back_fits && bt_mode != 0;  // one fetch batch covers a block
    v.bt_none = (bt_one || q_form) ? 1 : 0;
    // k_refl_T (reflectors -> T factors) does not depend on the tridiagonal's
    // eigenpairs: it runs on a side stream beside k_tri_vectors (and k_form_q
    // after it), so k_tri_vectors needs nothing from the reflectors' XCD
    hipStream_t side = nullptr;
    hipEvent_t fork_ev = nullptr, join_ev = nullptr;
    if (bt_one || q_form) {
        v.xcd = nullptr;
        side_stream(&side, &fork_ev, &join_ev);
    }
    if (n > 2) {
        const int nblk = (n - 2 + BT_NB - 1) / BT_NB;
        hipStream_t rs = st;
        if (side) {
            hipEventRecord(fork_ev, st);
            hipStreamWaitEvent(side, fork_ev, 0);
            rs = side;
        }
        const size_t rlds = sizeof(double) * BT_NB * (size_t)n;
        if (rlds + 20 * 1024 <= EIG_LDS_MAX) {  // + the static G, T (one coalesced read: no XCD pinning)
            scc_set_lds((const void*)k_refl_T_lds, (int)rlds);
            hipLaunchKernelGGL(k_refl_T_lds, dim3(nblk), dim3(1024), rlds, rs, t.refl, t.tau, n, lda,
                               scratch + L.tf);
        } else {
            hipLaunchKernelGGL(k_refl_T, dim3(pin ? 8 * nblk : nblk), dim3(1024), 0, rs, t.refl, t.tau, n, lda,
                               scratch + L.tf, pin ? t.reg : nullptr, flags + 9);
        }
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if (q_form) {
            const size_t qlds = form_q_lds(n);
            scc_set_lds((const void*)k_form_q, (int)qlds);
            hipLaunchKernelGGL(k_form_q, dim3((n + QF_R - 1) / QF_R), dim3(QF_T), qlds, rs, t.refl, scratch + L.tf, n,
                               lda, scratch + L.q);
            if ((e = hipGetLastError()) != hipSuccess) return e;
        }
        if (side) hipEventRecord(join_ev, side);
    }
    if (marks && marks[2]) hipEventRecord(marks[2], st);
    hipLaunchKernelGGL(k_tri_vectors, dim3(v.xcd ? 8 * k : k), dim3(VEC_T), vlds, st, v);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (side && n > 2) hipStreamWaitEvent(st, join_ev, 0);
    double* zfin = v.Zq;
    if (q_form) {
        hipLaunchKernelGGL(k_apply_q, dim3((n + 15) / 16), dim3(64), 0, st, scratch + L.q, v.Zq, n, lda, k,
                           scratch + L.zt);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        zfin = scratch + L.zt;
    } else if (bt_one) {
        const size_t blds = tri_back_lds(n, k);
        scc_set_lds((const void*)k_tri_back, (int)blds);
        hipLaunchKernelGGL(k_tri_back, dim3(1), dim3(TB_T), blds, st, v.Zq, n, lda, k, v.refl, v.tf, stamps);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (marks && marks[3]) hipEventRecord(marks[3], st);
    if (marks && marks[4]) hipEventRecord(marks[4], st);
    launch_eig_finish(zfin, n, lda, k, W, v.tnorm, Z, st);
    if (marks && marks[5]) hipEventRecord(marks[5], st);
    return hipGetLastError();
}


// diagnostic (tests): top-k eigenpairs of a device matrix A (n x n, lda) into
// Z (n x 16) and W (k) through scc_launch_eigen_topk; returns 0 on success,
// *path = scc_diag_eig_last_path()
extern "C" SCC_API int scc_diag_eigen_topk(const double* A, int n, int lda, int k,
                                                                          double* Z, double* W, int* path)
{
    double* scr = nullptr;
    const size_t sz = sizeof(double) * scc_eigen_scratch_doubles(n, lda, k);
    if (hipMalloc((void**)&scr, sz) != hipSuccess) return 1;
    unsigned int* err = nullptr;
    hipError_t e = scc_launch_eigen_topk(A, n, lda, k, scr, Z, W, &err, nullptr, nullptr, nullptr, 0, nullptr);
    unsigned int h = 0;
    if (e == hipSuccess && err) e = hipMemcpy(&h, err, sizeof(h), hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (path) *path = g_eig_last_path;
    scc_fsi_forget(scr, sz);
    hipFree(scr);
    return (e == hipSuccess && h == 0) ? 0 : 1;
}
