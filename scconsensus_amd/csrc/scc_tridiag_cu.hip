// scc_tridiag_cu.hip — Householder tridiagonalisation of the |U| x |U| Gram on
// ONE compute unit (PCA step of stage 3: irlba::prcomp_irlba,
// R/reclusterDEConsensusFast.R:398; R/reclusterDEConsensus.R:234).
//
// The one-stage reduction (LAPACK dsytd2, lower) is a chain of n - 1 dependent
// symmetric matrix-vector products.  Spread over a whole XCD (k_tridiag in
// scc_eigen.hip) every column pays a cross-CU hand-off (~3 us per column at
// n = 323).  For n <= TC_NMAX the lower triangle fits ONE CU's register file
// plus its LDS, so this kernel keeps the whole matrix resident in one 512-thread
// workgroup and a column costs three workgroup barriers and ~4 fp64 FMAs per
// live element, nothing else:
//   * rows [TC_RB, n): in registers.  Wave w holds rows TC_RB + w + 8m
//     (m < TC_MR), lane l holding columns 64 s + l of every slot s up to the
//     row's diagonal (76 doubles per lane).
//   * rows [r1, min(n, TC_RB)): packed lower rows in LDS; rows [0, r1) (only
//     when they do not fit) packed in a global scratch buffer that only their
//     owning wave touches.  Memory row r belongs to wave r % 8.
// Per column i (v_i, tau_i known; the rank-2 update of step i-1 is applied
// lazily, while its elements are read for the product):
//   phase 1  every wave: a <- a - v'_r w'_c - w'_r v'_c on its live elements,
//            row sums  sum_c a v_c (8 rows reduced at once by a lane transpose)
//            and column sums  sum_r a v_r  (per-lane slot accumulators), and
//            the element of column i+1 (the next column to reduce);
//   barrier; phase 2 (thread j): y_j = row sum + the 8 waves' column sums in a
//            fixed order, p = tau y, K = p.v;  barrier; w = p - tau K / 2 v,
//            x_j = a_{j,i+1} - v_j w_{i+1} - w_j (column i+1 of A^(i)),
//            |x_{i+3..}|^2;  barrier; every thread forms the next reflector
//            (dlarfg) and reloads its register slots.
// Every reduction has a fixed order, so the result is bit-reproducible run to
// run (unlike the arrival-ordered multi-workgroup kernel).  Outputs d, e, tau
// and the reflectors in the layout k_tridiag writes, so the eigenpair kernels
// that follow are unchanged.
#include "scc_common.hpp"

#define TC_T 512
#define TC_W (TC_T / 64)
#define TC_RB 240                        // first register row
#define TC_MR 12                         // register rows per wave
#define TC_NMAX (TC_RB + TC_W * TC_MR)   // 336
#define TC_NS 6                          // 64-column slots per lane
#define TC_MS 4                          // slots of a memory row (r < TC_RB)
#define TC_LDS_BYTES (160 * 1024)

struct TriCuArgs {
    const double* A;  // n x n symmetric, row-major (lower triangle read)
    int n, lda;
    int r1;           // rows [0, r1) in grows, [r1, min(n, TC_RB)) in LDS
    double* grows;    // packed lower rows 0..r1-1 (row r at r (r + 1) / 2)
    double* d;        // [n] diagonal of T
    double* e;        // [n] off-diagonal
    double* tau;      // [n]
    double* refl;     // reflector i in row i (j >= i + 1), refl[i][i+1] = 1
    u32* reg;         // reg[0] = XCD + 1 (the eigenpair kernels pin to it)
    u64* stamps;      // diagnostic (SCC_STAMPS): wave 0's cycles per phase, else null
};

__device__ __forceinline__ double tc_sum(double v)
{
    v += scc_xor_lane_f64<32>(v);
    v += scc_xor_lane_f64<16>(v);
    v += scc_xor_lane_f64<8>(v);
    v += scc_xor_lane_f64<4>(v);
    v += scc_xor_lane_f64<2>(v);
    return v + scc_xor_lane_f64<1>(v);
}

__device__ __forceinline__ u64 tc_bits(double x) { return (u64)__double_as_longlong(x); }
__device__ __forceinline__ double tc_dbl(u32 hi, u32 lo) { return __longlong_as_double((long long)(((u64)hi << 32) | lo)); }

// value of a wave-uniform lane (SGPR broadcast, no LDS)
__device__ __forceinline__ double tc_rl(double x, int lane)
{
    const u64 b = tc_bits(x);
    const u32 lo = (u32)__builtin_amdgcn_readlane((int)(u32)b, lane);
    const u32 hi = (u32)__builtin_amdgcn_readlane((int)(u32)(b >> 32), lane);
    return tc_dbl(hi, lo);
}

// element j (wave-uniform) of a lane-slotted vector (slot j >> 6, lane j & 63):
// one readlane pair per slot, the slot picked among the scalar results (a
// select on the register array itself would become a dynamic index, i.e. a
// trip through scratch)
template <int NS>
__device__ __forceinline__ double tc_bcast(const double (&v)[TC_NS], int j)
{
    const int s = j >> 6, l = j & 63;
    u32 lo = 0, hi = 0;
#pragma unroll
    for (int t = 0; t < NS; ++t) {
        const u64 b = tc_bits(v[t]);
        const u32 tl = (u32)__builtin_amdgcn_readlane((int)(u32)b, l);
        const u32 th = (u32)__builtin_amdgcn_readlane((int)(u32)(b >> 32), l);
        lo = (s == t) ? tl : lo;
        hi = (s == t) ? th : hi;
    }
    return tc_dbl(hi, lo);
}

// a <- [a lanes 0-31, b lanes 0-31], b <- [a lanes 32-63, b lanes 32-63]
__device__ __forceinline__ void tc_swap32(double& a, double& b)
{
    const u64 x = tc_bits(a), y = tc_bits(b);
    const auto l = __builtin_amdgcn_permlane32_swap((u32)x, (u32)y, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap((u32)(x >> 32), (u32)(y >> 32), false, false);
    a = tc_dbl(h[0], l[0]);
    b = tc_dbl(h[1], l[1]);
}
// 16-lane rows: a <- [a0, b0, a2, b2], b <- [a1, b1, a3, b3]
__device__ __forceinline__ void tc_swap16(double& a, double& b)
{
    const u64 x = tc_bits(a), y = tc_bits(b);
    const auto l = __builtin_amdgcn_permlane16_swap((u32)x, (u32)y, false, false);
    const auto h = __builtin_amdgcn_permlane16_swap((u32)(x >> 32), (u32)(y >> 32), false, false);
    a = tc_dbl(h[0], l[0]);
    b = tc_dbl(h[1], l[1]);
}

// Eight wave sums at once: afterwards lane l holds the total of x[(l >> 3) & 7]
// (a transpose-reduce: 10 lane exchanges instead of 48; fixed order).
__device__ __forceinline__ double tc_sum8(double (&x)[8], int lane)
{
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        tc_swap32(x[g], x[g + 4]);
        x[g] = x[g] + x[g + 4];  // lanes 0-31: row g, 32-63: row g + 4
    }
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        tc_swap16(x[g], x[g + 2]);
        x[g] = x[g] + x[g + 2];  // row g + 2 b4 + 4 b5
    }
    const bool b3 = (lane & 8) != 0;
    const double send = b3 ? x[0] : x[1];
    double u = (b3 ? x[1] : x[0]) + scc_xor_lane_f64<8>(send);  // row b3 + 2 b4 + 4 b5
    u += scc_xor_lane_f64<4>(u);
    u += scc_xor_lane_f64<2>(u);
    return u + scc_xor_lane_f64<1>(u);
}

// Four wave sums at once: afterwards lane l holds the total of x[(l >> 4) & 3].
__device__ __forceinline__ double tc_sum4(double (&x)[4], int lane)
{
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        tc_swap32(x[g], x[g + 2]);
        x[g] = x[g] + x[g + 2];  // lanes 0-31: row g, 32-63: row g + 2
    }
    tc_swap16(x[0], x[1]);
    double u = x[0] + x[1];  // row b4 + 2 b5
    u += scc_xor_lane_f64<8>(u);
    u += scc_xor_lane_f64<4>(u);
    u += scc_xor_lane_f64<2>(u);
    return u + scc_xor_lane_f64<1>(u);
}

// one memory row (LDS or global, P = its packed lower row) of column i
__device__ __forceinline__ void tc_mem_row(double* P, int r, int s_lo, int lx, double vr, double vpr, double wpr,
                                  const double (&vs)[TC_NS], const double (&vps)[TC_NS],
                                  const double (&wps)[TC_NS], double (&cacc)[TC_NS], double& racc,
                                  double* xcol, int lane)
{
    double x[TC_MS];
#pragma unroll
    for (int s = 0; s < TC_MS; ++s)  // every load of the row in flight at once
        x[s] = (s >= s_lo && 64 * s <= r) ? P[min(64 * s + lane, r)] : 0.0;
#pragma unroll
    for (int s = 0; s < TC_MS; ++s) {
        if (s < s_lo || 64 * s > r) continue;
        const int c = 64 * s + lane;
        double v = fma(-vpr, wps[s], fma(-wpr, vps[s], x[s]));
        v = (c <= r) ? v : 0.0;
        if (c <= r) P[c] = v;
        if (s == s_lo && lane == lx) xcol[r] = v;
        racc = fma(v, vs[s], racc);
        cacc[s] = fma((c < r) ? v : 0.0, vr, cacc[s]);
    }
}

__global__ void __launch_bounds__(TC_T) k_tridiag_cu(TriCuArgs a)
{
    extern __shared__ __attribute__((aligned(16))) double sm[];
    const int n = a.n, lda = a.lda;
    const int tid = threadIdx.x, lane = tid & 63, w = scc_wave_id();
    const int nm = min(n, TC_RB);  // memory rows [0, nm)
    const int r1 = a.r1;
    double* xcol = sm;            // column i+1 of A^(i-1), rows >= i+1
    double* xbuf = xcol + n;      // x = column i+1 of A^(i) (the next reflector's source)
    double* wbuf = xbuf + n;      // w_i
    double* rowres = wbuf + n;    // row sums of the product
    double* yp = rowres + n;      // [8][n] column sums per wave
    double* red = yp + 8 * n;     // [32] reductions
    double* lrows = red + 32;     // packed LDS rows r1 .. nm-1
    const long lbase = (long)r1 * (r1 + 1) / 2;

    if (tid == 0) {
        u32 x;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
        __hip_atomic_store(&a.reg[0], (x & 0xfu) + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    for (int k = tid; k < 12 * n + 32; k += TC_T) sm[k] = 0.0;
    if (n == 1) {
        if (tid == 0) {
            a.d[0] = a.A[0];
            a.e[0] = 0.0;
            a.tau[0] = 0.0;
        }
        return;
    }

    // ---- load: register rows, memory rows, column 0
    double ra[TC_MR][TC_NS];
#pragma unroll
    for (int m = 0; m < TC_MR; ++m) {
        const int r = TC_RB + 8 * m + w;
        const int st = (TC_RB + 8 * m) / 64;
#pragma unroll
        for (int s = 0; s < TC_NS; ++s) {
            if (s > st) continue;
            const int c = 64 * s + lane;
            const bool ok = r < n && c <= r;
            const double x = a.A[(size_t)min(r, n - 1) * lda + min(c, n - 1)];
            ra[m][s] = ok ? x : 0.0;
        }
    }
    for (int r = r1 + w; r < nm; r += TC_W)
        for (int c = lane; c <= r; c += 64) lrows[(long)r * (r + 1) / 2 - lbase + c] = a.A[(size_t)r * lda + c];
    for (int r = w; r < r1; r += TC_W)
        for (int c = lane; c <= r; c += 64) a.grows[(long)r * (r + 1) / 2 + c] = a.A[(size_t)r * lda + c];
    __syncthreads();
    for (int j = tid; j < n; j += TC_T) xbuf[j] = a.A[j];  // column 0 (= row 0)
    __syncthreads();

    // ---- reflector 0 from column 0 (dlarfg)
    double tc, scal_c;
    {
        const int j = tid;
        const double xj = (j < n) ? xbuf[j] : 0.0;
        double q = (j >= 2 && j < n) ? xj * xj : 0.0;
        q = tc_sum(q);
        if (lane == 0) red[16 + w] = q;
        __syncthreads();
        double xn2 = 0.0;
#pragma unroll
        for (int q2 = 0; q2 < TC_W; ++q2) xn2 += red[16 + q2];
        const double alpha = xbuf[1];
        double beta = alpha;
        tc = 0.0;
        scal_c = 0.0;
        if (xn2 > 0.0) {
            beta = -copysign(sqrt(alpha * alpha + xn2), alpha);
            tc = (beta - alpha) / beta;
            scal_c = 1.0 / (alpha - beta);
        }
        if (tid == 0) {
            a.d[0] = xbuf[0];
            a.e[0] = beta;
            a.tau[0] = tc;
        }
        if (j >= 1 && j < n) a.refl[j] = (j == 1) ? 1.0 : xj * scal_c;
    }
    double vs[TC_NS], vps[TC_NS], wps[TC_NS], cacc[TC_NS];
#pragma unroll
    for (int s = 0; s < TC_NS; ++s) {
        const int c = 64 * s + lane;
        const double x = xbuf[min(c, n - 1)];
        vs[s] = (c == 1) ? 1.0 : ((c > 1 && c < n) ? x * scal_c : 0.0);
        vps[s] = 0.0;
        wps[s] = 0.0;
        cacc[s] = 0.0;
    }

    const bool stmp = a.stamps && tid == 0;
    u64 t_1a = 0, t_1b = 0, t_2a = 0, t_2b = 0, tm = 0;
    for (int i = 0; i <= n - 2; ++i) {
        const int s_lo = (i + 1) >> 6, lx = (i + 1) & 63;
        if (stmp) tm = __builtin_amdgcn_s_memtime();
        // ---- phase 1a: register rows, four at a time
#pragma unroll
        for (int grp = 0; grp < (TC_MR + 3) / 4; ++grp) {
            const int rmin = TC_RB + 32 * grp + w, rmax = rmin + 24;
            if (rmin >= n || rmax <= i) continue;  // uniform: no live row in the group
            double racc[4];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int m = 4 * grp + g;
                const int st = (TC_RB + 8 * m) / 64;
                const int r = TC_RB + 8 * m + w;
                racc[g] = 0.0;
                if (m >= TC_MR || r >= n || r <= i) continue;
                const int L = (TC_RB + 8 * m) % 64 + w;
                const double vr = tc_rl(vs[st], L), vpr = tc_rl(vps[st], L), wpr = tc_rl(wps[st], L);
#pragma unroll
                for (int s = 0; s < TC_NS; ++s) {
                    if (s > st || s < s_lo) continue;
                    const int c = 64 * s + lane;
                    double x = fma(-vpr, wps[s], fma(-wpr, vps[s], ra[m][s]));
                    if (s == st) x = (c <= r) ? x : 0.0;
                    ra[m][s] = x;
                    if (s == s_lo && lane == lx) xcol[r] = x;
                    racc[g] = fma(x, vs[s], racc[g]);
                    const double xc = (s == st) ? ((c < r) ? x : 0.0) : x;
                    cacc[s] = fma(xc, vr, cacc[s]);
                }
            }
            const double tot = tc_sum4(racc, lane);
            const int gl = (lane >> 4) & 3;
            const int r = rmin + 8 * gl;
            if ((lane & 15) == 0 && 4 * grp + gl < TC_MR && r < n && r > i) rowres[r] = tot;
        }
        if (stmp) {
            const u64 t1 = __builtin_amdgcn_s_memtime();
            t_1a += t1 - tm;
            tm = t1;
        }
        // ---- phase 1b: memory rows r = w + 8k > i, four at a time
        {
            int k = (i + 1 > w) ? (i + 1 - w + TC_W - 1) / TC_W : 0;
            for (; w + TC_W * k < nm; k += 4) {
                double racc[4];
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int r = w + TC_W * (k + g);
                    racc[g] = 0.0;
                    if (r >= nm) continue;
                    const double vr = tc_bcast<TC_MS>(vs, r), vpr = tc_bcast<TC_MS>(vps, r),
                                 wpr = tc_bcast<TC_MS>(wps, r);
                    if (r < r1)
                        tc_mem_row(a.grows + (long)r * (r + 1) / 2, r, s_lo, lx, vr, vpr, wpr, vs, vps, wps, cacc,
                                   racc[g], xcol, lane);
                    else
                        tc_mem_row(lrows + ((long)r * (r + 1) / 2 - lbase), r, s_lo, lx, vr, vpr, wpr, vs, vps, wps,
                                   cacc, racc[g], xcol, lane);
                }
                const double tot = tc_sum4(racc, lane);
                const int r = w + TC_W * (k + ((lane >> 4) & 3));
                if ((lane & 15) == 0 && r < nm) rowres[r] = tot;
            }
        }
#pragma unroll
        for (int s = 0; s < TC_NS; ++s) {
            const int c = 64 * s + lane;
            if (s >= s_lo && c < n) yp[w * n + c] = cacc[s];
            cacc[s] = 0.0;
        }
        __syncthreads();
        if (stmp) {
            const u64 t1 = __builtin_amdgcn_s_memtime();
            t_1b += t1 - tm;
            tm = t1;
        }

        // ---- phase 2: p = tau A v, w, column i+1 of A^(i), next reflector
        const int j = i + 1 + tid;
        const bool act = j < n;
        const int jc = act ? j : i + 1;
        double y = rowres[jc], y1 = rowres[i + 1];
#pragma unroll
        for (int q = 0; q < TC_W; ++q) {
            y += yp[q * n + jc];
            y1 += yp[q * n + i + 1];
        }
        const double p = tc * y, p1 = tc * y1;
        const double xo = xbuf[jc];
        const double vj = act ? ((j == i + 1) ? 1.0 : xo * scal_c) : 0.0;
        double part = act ? p * vj : 0.0;
        part = tc_sum(part);
        if (lane == 0) red[w] = part;
        __syncthreads();
        double K = 0.0;
#pragma unroll
        for (int q = 0; q < TC_W; ++q) K += red[q];
        const double a2 = -0.5 * tc * K;
        const double wj = (act && tc != 0.0) ? fma(a2, vj, p) : 0.0;
        const double w1 = (tc != 0.0) ? fma(a2, 1.0, p1) : 0.0;
        const double xj = act ? fma(-1.0, wj, fma(-w1, vj, xcol[jc])) : 0.0;
        if (act) {
            wbuf[j] = wj;
            xbuf[j] = xj;
        }
        double q2 = (act && j >= i + 3) ? xj * xj : 0.0;
        q2 = tc_sum(q2);
        if (lane == 0) red[8 + w] = q2;
        __syncthreads();
        if (stmp) {
            const u64 t1 = __builtin_amdgcn_s_memtime();
            t_2a += t1 - tm;
            tm = t1;
        }
        if (i + 1 <= n - 2) {
            double xn2 = 0.0;
#pragma unroll
            for (int q = 0; q < TC_W; ++q) xn2 += red[8 + q];
            const double alpha = xbuf[i + 2];
            double bn = alpha, tn = 0.0, scal = 0.0;
            if (xn2 > 0.0) {
                bn = -copysign(sqrt(alpha * alpha + xn2), alpha);
                tn = (bn - alpha) / bn;
                scal = 1.0 / (alpha - bn);
            }
            if (tid == 0) {
                a.d[i + 1] = xbuf[i + 1];
                a.e[i + 1] = bn;
                a.tau[i + 1] = tn;
            }
            if (act && j >= i + 2) a.refl[(size_t)(i + 1) * lda + j] = (j == i + 2) ? 1.0 : xj * scal;
#pragma unroll
            for (int s = 0; s < TC_NS; ++s) {
                const int c = 64 * s + lane, cc = min(c, n - 1);
                const double xv = xbuf[cc], wv = wbuf[cc];
                vps[s] = vs[s];
                wps[s] = (c > i && c < n) ? wv : 0.0;
                vs[s] = (c == i + 2) ? 1.0 : ((c > i + 2 && c < n) ? xv * scal : 0.0);
            }
            tc = tn;
            scal_c = scal;
        } else if (tid == 0) {
            a.d[n - 1] = xbuf[n - 1];
            a.e[n - 1] = 0.0;
            a.tau[n - 1] = 0.0;
        }
        if (stmp) t_2b += __builtin_amdgcn_s_memtime() - tm;
    }
    if (stmp) {
        a.stamps[0] = t_1a + t_1b;
        a.stamps[7] = t_1a;
        a.stamps[1] = t_2a;
        a.stamps[2] = t_2b;
    }
}

static int tc_r1(int n)
{
    const long cap = TC_LDS_BYTES / 8 - (12L * n + 32);
    const long nm = n < TC_RB ? n : TC_RB;
    long r1 = 0;
    while (nm * (nm + 1) / 2 - r1 * (r1 + 1) / 2 > cap) ++r1;
    return (int)r1;
}

extern "C" int scc_tridiag_cu_fits(int n) { return n >= 2 && n <= TC_NMAX; }

// grows: >= n (n + 1) / 2 doubles of scratch
extern "C" hipError_t scc_launch_tridiag_cu(const double* A, int n, int lda, double* grows, double* d, double* e,
                                            double* tau, double* refl, unsigned int* reg, unsigned long long* stamps,
                                            hipStream_t st)
{
    if (!scc_tridiag_cu_fits(n)) return hipErrorInvalidValue;
    TriCuArgs t;
    t.A = A;
    t.n = n;
    t.lda = lda;
    t.r1 = tc_r1(n);
    t.grows = grows;
    t.d = d;
    t.e = e;
    t.tau = tau;
    t.refl = refl;
    t.reg = reg;
    t.stamps = (u64*)stamps;
    hipError_t err = hipFuncSetAttribute((const void*)k_tridiag_cu, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         TC_LDS_BYTES);
    if (err != hipSuccess) return err;
    hipLaunchKernelGGL(k_tridiag_cu, dim3(1), dim3(TC_T), TC_LDS_BYTES, st, t);
    return hipGetLastError();
}
