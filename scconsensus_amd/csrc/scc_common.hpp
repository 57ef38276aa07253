// scc_common.hpp — device helpers shared by the scConsensus MI355X engine.
//
// Everything here is compiled with -ffp-contract=off: the compensated (double-
// double) sums and the R-order p-value arithmetic depend on un-fused rounding.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <atomic>
#include <map>
#include <mutex>
#include <utility>

typedef unsigned long long u64;
typedef long long i64;
typedef uint32_t u32;
typedef uint8_t u8;

#define SCC_WAVE 64

// clusters one engine run holds: 7-bit cluster codes (bit 7 of a sorted-code
// byte flags "equal to the next element" in the rank kernels)
#define SCC_MAX_K 128
#define SCC_CODE_BITS 7
#define SCC_CODE_MASK 127u

// ------------------------------------------------------------ launch attributes
// A kernel's dynamic-LDS limit, set once per (kernel, device) and raised only
// when a launch needs more: hipFuncSetAttribute costs ~23 us a call on this
// runtime (HIP API trace of the config-B bench: 134 calls, 3.1 ms over 12
// steps), and the per-call settings kept the host behind the GPU.
static inline hipError_t scc_set_lds(const void* fn, size_t bytes)
{
    static std::mutex mu;
    static std::map<std::pair<const void*, int>, size_t> set;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) {
        (void)hipGetLastError();
        dev = -1;
    }
    std::lock_guard<std::mutex> lk(mu);
    const auto key = std::make_pair(fn, dev);
    const auto it = set.find(key);
    if (it != set.end() && it->second >= bytes) return hipSuccess;
    const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e == hipSuccess) set[key] = bytes;
    return e;
}

// ------------------------------------------------------------ orderable keys
// Bijective map fp64 -> u64 whose unsigned order is the IEEE total order for
// finite values (-0 and +0 never reach it: zeros are the implicit tie group).
__host__ __device__ inline u64 scc_key_of(double v)
{
    u64 b = (u64)__double_as_longlong(v);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__host__ __device__ inline double scc_val_of(u64 k)
{
    u64 b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
    return __longlong_as_double((long long)b);
}

// ------------------------------------------------------------ double-double
struct dd {
    double hi, lo;
};
__device__ inline dd dd_two_sum(double a, double b)
{
    double s = a + b;
    double bb = s - a;
    double e = (a - (s - bb)) + (b - bb);
    return dd{s, e};
}
__device__ inline dd dd_fast_two_sum(double a, double b)
{
    double s = a + b;
    double e = b - (s - a);
    return dd{s, e};
}
__device__ inline dd dd_add_d(dd x, double y)
{
    dd s = dd_two_sum(x.hi, y);
    s.lo += x.lo;
    return dd_fast_two_sum(s.hi, s.lo);
}
__device__ inline dd dd_add(dd x, dd y)
{
    dd s = dd_two_sum(x.hi, y.hi);
    dd t = dd_two_sum(x.lo, y.lo);
    s.lo += t.hi;
    s = dd_fast_two_sum(s.hi, s.lo);
    s.lo += t.lo;
    return dd_fast_two_sum(s.hi, s.lo);
}
// exact product a * b as a double-double (FMA)
__device__ inline dd dd_two_prod(double a, double b)
{
    const double p = a * b;
    return dd{p, fma(a, b, -p)};
}
// x * y for a double-double x and a double y
__device__ inline dd dd_mul_d(dd x, double y)
{
    const dd p = dd_two_prod(x.hi, y);
    return dd_fast_two_sum(p.hi, fma(x.lo, y, p.lo));
}
// (hi + lo) / n rounded to double (one correction step; exact enough that the
// result is the correctly rounded mean except in measure-zero cases).
__device__ inline double dd_div_n(dd x, double n)
{
    double q = x.hi / n;
    double r = fma(-q, n, x.hi);  // exact remainder of hi - q*n
    r += x.lo;
    return q + r / n;
}

__device__ inline dd dd_shfl_xor(dd x, int m)
{
    return dd{__shfl_xor(x.hi, m, SCC_WAVE), __shfl_xor(x.lo, m, SCC_WAVE)};
}
// Deterministic butterfly: every lane ends with the same value.
__device__ inline dd dd_wave_sum(dd x)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) x = dd_add(x, dd_shfl_xor(x, m));
    return x;
}
__device__ inline u64 u64_wave_sum(u64 x)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) x += __shfl_xor(x, m, SCC_WAVE);
    return x;
}
__device__ inline u32 u32_wave_sum(u32 x)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) x += __shfl_xor(x, m, SCC_WAVE);
    return x;
}

// Value of lane (this lane ^ S) without an LDS round trip: DPP inside a
// 16-lane row, v_permlane16/32_swap across rows (gfx950).  Whole-wave only:
// every lane must be active.
template <int S>
__device__ inline u32 scc_xor_lane(u32 v)
{
    const int x = (int)v;
    if constexpr (S == 1) {
        return (u32)__builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, true);  // quad_perm [1,0,3,2]
    } else if constexpr (S == 2) {
        return (u32)__builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, true);  // quad_perm [2,3,0,1]
    } else if constexpr (S == 4) {
        const int up = __builtin_amdgcn_update_dpp(0, x, 0x104, 0xF, 0xF, true);  // row_shl:4
        const int dn = __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, true);  // row_shr:4
        return (u32)((__lane_id() & 4) ? dn : up);
    } else if constexpr (S == 8) {
        return (u32)__builtin_amdgcn_update_dpp(0, x, 0x128, 0xF, 0xF, true);  // row_ror:8
    } else if constexpr (S == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (__lane_id() & 16) ? r[0] : r[1];
    } else {
        static_assert(S == 32, "scc_xor_lane: stride");
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (__lane_id() & 32) ? r[0] : r[1];
    }
}
template <int S>
__device__ inline double scc_xor_lane_f64(double v)
{
    const u64 b = (u64)__double_as_longlong(v);
    const u64 r = ((u64)scc_xor_lane<S>((u32)(b >> 32)) << 32) | scc_xor_lane<S>((u32)b);
    return __longlong_as_double((long long)r);
}
template <int S>
__device__ inline dd dd_xor_lane(dd x)
{
    return dd{scc_xor_lane_f64<S>(x.hi), scc_xor_lane_f64<S>(x.lo)};
}
// dd_wave_sum / u32_wave_sum without LDS (same butterfly order, whole wave only)
__device__ inline dd dd_wave_sum_dpp(dd x)
{
    x = dd_add(x, dd_xor_lane<32>(x));
    x = dd_add(x, dd_xor_lane<16>(x));
    x = dd_add(x, dd_xor_lane<8>(x));
    x = dd_add(x, dd_xor_lane<4>(x));
    x = dd_add(x, dd_xor_lane<2>(x));
    return dd_add(x, dd_xor_lane<1>(x));
}
__device__ inline u32 u32_wave_sum_dpp(u32 x)
{
    x += scc_xor_lane<32>(x);
    x += scc_xor_lane<16>(x);
    x += scc_xor_lane<8>(x);
    x += scc_xor_lane<4>(x);
    x += scc_xor_lane<2>(x);
    return x + scc_xor_lane<1>(x);
}

// sqrt for s >= 0 from the hardware reciprocal square root (~2^-26
// relative) and one Newton correction y += (s - y^2) / (2 y), with 1 / (2 y)
// taken as g / 2: the error is ~delta^2 = 2^-52 relative plus the roundings,
// i.e. within ~2 ulp (the libm sequence adds denormal scaling and two more
// corrections; distance entries are far from the denormal range, and 0 maps
// to 0).  v_sqrt_f64 alone is only ~1e-8 relative.
__device__ inline double scc_sqrt_nr(double s)
{
    const double g = __builtin_amdgcn_rsq(s);  // s = 0: +inf, handled below
    const double y = s * g;
    const double e = fma(-y, y, s);
    const double r = fma(e, 0.5 * g, y);
    return s > 0.0 ? r : 0.0;
}

// wave index inside the workgroup, as a wave-uniform (SGPR) value: loops
// bounded by it stay scalar instead of being treated as divergent
__device__ inline int scc_wave_id() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }

// CU count of the current device, cached per device ordinal (host threads
// driving different devices or contexts may call this concurrently)
inline int scc_device_cus(int fallback)
{
    static std::atomic<int> cache[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return fallback;
    int v = cache[dev].load(std::memory_order_relaxed);
    if (v > 0) return v;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) {
        (void)hipGetLastError();
        return fallback;
    }
    cache[dev].store(v, std::memory_order_relaxed);
    return v;
}

__host__ __device__ inline int scc_next_pow2(int n)
{
    int m = 1;
    while (m < n) m <<= 1;
    return m;
}

// ------------------------------------------------------------ pair indexing
// Pairs (i<j) enumerated as R's nested loops: p = i*K - i*(i+1)/2 + (j-i-1).
__host__ __device__ inline int scc_pair_index(int i, int j, int K)
{
    return i * K - i * (i + 1) / 2 + (j - i - 1);
}

// ------------------------------------------------------------ pnorm (R)
// Two-sided normal p-value 2*min(pnorm(z), pnorm(z, lower.tail=FALSE)) with the
// same evaluation as R's nmath/pnorm.c (Cody 1993, ACM TOMS 715), including its
// underflow cut-offs (|z| >= 37.5193 -> 0).
__device__ inline double scc_pnorm_small_tail(double z)
{
    // returns min(pnorm(z), pnorm(-z)) i.e. the tail beyond |z|, NaN for NaN
    const double A[5] = {2.2352520354606839287, 161.02823106855587881, 1067.6894854603709582,
                         18154.981253343561249, 0.065682337918207449113};
    const double B[4] = {47.20258190468824187, 976.09855173777669322, 10260.932208618978205,
                         45507.789335026729956};
    const double C[9] = {0.39894151208813466764, 8.8831497943883759412, 93.506656132177855979,
                         597.27027639480026226, 2494.5375852903726711, 6848.1904505362823326,
                         11602.651437647350124, 9842.7148383839780218, 1.0765576773720192317e-8};
    const double D[8] = {22.266688044328115691, 235.38790178262499861, 1519.377599407554805,
                         6485.558298266760755, 18615.571640885098091, 34900.952721145977266,
                         38912.003286093271411, 19685.429676859990727};
    const double P[6] = {0.21589853405795699, 0.1274011611602473639, 0.022235277870649807,
                         0.001421619193227893466, 2.9112874951168792e-5, 0.02307344176494017303};
    const double Q[5] = {1.28426009614491121, 0.468238212480865118, 0.0659881378689285515,
                         0.00378239633202758244, 7.29751555083966205e-5};
    if (z != z) return z;
    // R evaluates pnorm(z) (lower) and pnorm(z, lower=FALSE) (upper) separately;
    // the smaller one is the tail on the far side of 0.  Restate each branch of
    // pnorm_both for that tail with the same operation order.
    double y = fabs(z);
    double cum, ccum, temp, xnum, xden, xsq, del;
    if (y <= 0.67448975) {
        const double eps = 1.1102230246251565e-16;  // DBL_EPSILON * 0.5
        if (y > eps) {
            xsq = z * z;
            xnum = A[4] * xsq;
            xden = xsq;
            for (int i = 0; i < 3; ++i) {
                xnum = (xnum + A[i]) * xsq;
                xden = (xden + B[i]) * xsq;
            }
        } else {
            xnum = xden = 0.0;
        }
        temp = z * (xnum + A[3]) / (xden + B[3]);
        cum = 0.5 + temp;
        ccum = 0.5 - temp;
        return cum < ccum ? cum : ccum;
    } else if (y <= 5.656854249492380195206754896838) {
        xnum = C[8] * y;
        xden = y;
        for (int i = 0; i < 7; ++i) {
            xnum = (xnum + C[i]) * y;
            xden = (xden + D[i]) * y;
        }
        temp = (xnum + C[7]) / (xden + D[7]);
        xsq = trunc(y * 16.0) / 16.0;
        del = (y - xsq) * (y + xsq);
        cum = exp(-xsq * xsq * 0.5) * exp(-del * 0.5) * temp;
        ccum = 1.0 - cum;
        // cum is the tail beyond |z| on the far side; R swaps for z > 0 so the
        // small tail is cum either way.
        return cum < ccum ? cum : ccum;
    } else {
        // lower tail of z<0 valid for -37.5193 < z; upper tail of z>0 valid for z < 37.5193
        if (!(y < 37.5193)) return 0.0;
        double x = z;
        xsq = 1.0 / (x * x);
        xnum = P[5] * xsq;
        xden = xsq;
        for (int i = 0; i < 4; ++i) {
            xnum = (xnum + P[i]) * xsq;
            xden = (xden + Q[i]) * xsq;
        }
        temp = xsq * (xnum + P[4]) / (xden + Q[4]);
        temp = (0.398942280401432677939946059934 - temp) / y;
        xsq = trunc(x * 16.0) / 16.0;
        del = (x - xsq) * (x + xsq);
        cum = exp(-xsq * xsq * 0.5) * exp(-del * 0.5) * temp;
        return cum;  // the small tail (R: cum for x<0, swapped into ccum for x>0)
    }
}
