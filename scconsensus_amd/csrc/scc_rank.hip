// scc_rank.hip — per-gene statistics and the all-pairs Wilcoxon rank-sum engine.
//
// Replaces the reference's per-(pair, gene) `wilcox.test(data.use[x, ] ~ group)`
// calls (R/reclusterDEConsensusFast.R:78-91; R/reclusterDEConsensus.R:99-103)
// and the per-cluster log-mean / detection statistics (Fast:229-271,
// slow:104-113).  Exact integer arithmetic throughout: R's statistic
// W = 2U/2 and its tie term sum(NTIES^3 - NTIES) are reproduced bit for bit.
//
// Kernels (one launch each, all on the nonzeros the ingest grouped by
// (gene, cluster); zeros are never materialised):
//   k_gene_stats   one workgroup per gene: per-cluster double-double sums of
//                  x and expm1(x), counts of x > 0 and x < 0, fixed reduction
//                  order (bitwise deterministic).
//   k_rank_classify  per gene: does any cluster pair test it (FAST filters
//                  ran before the rank stage, exactly as ComputePairWiseDE
//                  only tests the features that pass, Fast:242-291)?  Genes
//                  that fit a workgroup's LDS become work items; larger ones
//                  go to the splitter.
//   k_rank_split   one workgroup per large gene: 2048-bin histogram of the
//                  value key, bins packed into value-range buckets of <= cap
//                  elements, buckets scattered to their own ranges, and the
//                  cross-bucket part of every tested pair's rank sum from the
//                  per-bucket cluster histograms.  Equal values never straddle
//                  buckets, so ties stay inside one work item.
//   k_rank_item    one workgroup per work item (a gene or a bucket): stable
//                  LSD radix sort (8-bit digits, wave match-ranking, no atomic
//                  conflicts) on a 32-bit window of the orderable key with an
//                  exact fix-up of windows that merged distinct doubles; the
//                  sorted positions partitioned by cluster; for every tested
//                  pair (a, b) the within-item count #{x in a, y in b: x > y}
//                  by binary searches of the smaller cluster's positions in
//                  the larger's; tie groups (runs of equal values) give
//                  E_ab = sum c_a c_b, X_ab = sum c_a c_b (c_a + c_b) and
//                  F_a = sum (c_a^3 - c_a).  Everything is added with integer
//                  atomics into per-(pair, gene) accumulators (order-free).
// The pair-test kernel (scc_select.hip) adds the implicit zero group in closed
// form:  2U = 2 (S + z_a neg_b + pos_a z_b) + z_a z_b + E,
//        T  = F_a + F_b + f(z_a) + f(z_b) + 3 z_a z_b (z_a + z_b) + 3 X.
#include "scc_common.hpp"
#include "scc_kernels.hpp"

#include <algorithm>
#include <cstddef>
#include <cstdio>
#include <vector>
#include <type_traits>

__device__ inline u64 f_tie(u64 c) { return c * c * c - c; }

__device__ inline u32 lanes_below(u64 m)  // popcount of m over lanes < this lane
{
    return __builtin_amdgcn_mbcnt_hi((u32)(m >> 32), __builtin_amdgcn_mbcnt_lo((u32)m, 0u));
}

__device__ inline u64 shfl_xor_u64(u64 v, int m)
{
    const u32 lo = __shfl_xor((u32)v, m, 64), hi = __shfl_xor((u32)(v >> 32), m, 64);
    return ((u64)hi << 32) | lo;
}

__device__ inline void pair_decode(int p, int K, int& a, int& b)
{
    a = 0;
    int rem = p;
    while (rem >= K - 1 - a) {
        rem -= K - 1 - a;
        ++a;
    }
    b = a + 1 + rem;
}

// lanes whose value of the low `bits` bits of d equals this lane's (among `act`)
template <int BITS>
__device__ inline u64 match_bits(u32 d, u64 act)
{
    u64 peers = act;
#pragma unroll
    for (int b = 0; b < BITS; ++b) {
        const bool bit = (d >> b) & 1u;
        const u64 bb = __ballot(bit);
        peers &= bit ? bb : ~bb;
    }
    return peers;
}

// ===================================================================== stats
#define ST_T 256
#define ST_W (ST_T / 64)
#ifndef ST_U
#define ST_U 4
#endif

struct StatItem {
    double sx_hi, sx_lo, se_hi, se_lo;
    u32 pos, neg;
};

// FAST needs the per-cluster mean of expm1(x) (Fast:259-272), SLOW the mean
// of x (slow:105), the FAST t test (DiffTTest, Fast:185-196) both plus, in a
// second pass (VAR), R's two-pass variance sum((x - mean)^2) / (n - 1) over
// the cluster, zeros included.  Each pass accumulates only its own
// double-double sums.
template <bool EXPM1, bool SUMX, bool VAR>
__global__ void __launch_bounds__(ST_T) k_gene_stats(ScStatsLaunch A)
{
    __shared__ int off[SCC_MAX_K + 1];
    __shared__ StatItem item[SCC_MAX_K + ST_W + 4];
    const int g = A.glo + blockIdx.x, K = A.K, tid = threadIdx.x, lane = tid & 63, w = scc_wave_id();
    const i64 base = A.gstart[g];
    const int n = (int)(A.gstart[g + 1] - base);
    const u64* key = A.keys + base;
    if (tid <= K) off[tid] = (int)A.coff[(size_t)A.cl_cc[tid] * A.G + g];
    __syncthreads();
    // balanced pieces that never straddle clusters, combined in a fixed order
    const int Lp = max(64, (((n + ST_W - 1) / ST_W) + 63) & ~63);
    for (int it = w;; it += ST_W) {
        int a = 0, acc = 0, ni = 0;
        for (; a < K; ++a) {
            ni = (off[a + 1] - off[a] + Lp - 1) / Lp;
            if (it < acc + ni) break;
            acc += ni;
        }
        if (a == K) break;
        const int s0 = off[a] + (it - acc) * Lp, s1 = min(off[a + 1], s0 + Lp);
        const double ma = VAR ? A.mean_x[(size_t)a * A.G + g] : 0.0;
        dd sx{0.0, 0.0}, se{0.0, 0.0};
        u32 pos = 0, neg = 0;
        // ST_U loads in flight per lane (16 measured slower: B 0.18 -> 0.28 ms,
        // D 2.06 -> 2.75: the stage is VALU-bound on fp64 expm1 + double-double
        // adds, and the wider unroll cost occupancy); the per-lane summation
        // order (i, i + 64, i + 128, ...) does not depend on ST_U
        for (int i = s0 + lane; i < s1; i += 64 * ST_U) {
            double x[ST_U];  // past the end adds +0 (exact no-op)
#pragma unroll
            for (int q = 0; q < ST_U; ++q) {  // clamped unconditional load + select (i < s1)
                const double v = scc_val_of(key[min(i + 64 * q, s1 - 1)]);
                x[q] = (i + 64 * q < s1) ? v : 0.0;
            }
#pragma unroll
            for (int q = 0; q < ST_U; ++q) {
                if (EXPM1) se = dd_add_d(se, expm1(x[q]));
                if (SUMX) sx = dd_add_d(sx, x[q]);
                if (VAR && i + 64 * q < s1) sx = dd_add(sx, dd_two_prod(x[q] - ma, x[q] - ma));
                pos += (x[q] > 0.0);
                neg += (x[q] < 0.0);
            }
        }
        if (EXPM1) se = dd_wave_sum_dpp(se);
        if (SUMX || VAR) sx = dd_wave_sum_dpp(sx);
        pos = u32_wave_sum_dpp(pos);
        neg = u32_wave_sum_dpp(neg);
        if (lane == 0) item[it] = StatItem{sx.hi, sx.lo, se.hi, se.lo, pos, neg};
    }
    __syncthreads();
    if (tid < K) {
        const int a = tid;
        int first = 0;
        for (int b = 0; b < a; ++b) first += (off[b + 1] - off[b] + Lp - 1) / Lp;
        const int ni = (off[a + 1] - off[a] + Lp - 1) / Lp;
        dd sx{0.0, 0.0}, se{0.0, 0.0};
        u32 pos = 0, neg = 0;
        for (int q = first; q < first + ni; ++q) {
            sx = dd_add(sx, dd{item[q].sx_hi, item[q].sx_lo});
            se = dd_add(se, dd{item[q].se_hi, item[q].se_lo});
            pos += item[q].pos;
            neg += item[q].neg;
        }
        const double na = (double)A.n_clu[a];
        if (VAR) {  // + the zeros' (0 - mean)^2, then / (n - 1)
            const double m = A.mean_x[(size_t)a * A.G + g];
            const double z = na - (double)A.cnt_pos[(size_t)a * A.G + g] - (double)A.cnt_neg[(size_t)a * A.G + g];
            sx = dd_add(sx, dd_mul_d(dd_two_prod(m, m), z));
            A.var_x[(size_t)a * A.G + g] = dd_div_n(sx, na - 1.0);
            return;
        }
        if (EXPM1) A.mean_e[(size_t)a * A.G + g] = dd_div_n(se, na);
        if (SUMX) A.mean_x[(size_t)a * A.G + g] = dd_div_n(sx, na);
        A.cnt_pos[(size_t)a * A.G + g] = pos;
        A.cnt_neg[(size_t)a * A.G + g] = neg;
    }
}

extern "C" hipError_t scc_launch_gene_stats(const ScStatsLaunch* L, hipStream_t st)
{
    if (L->G <= 0 || L->gn <= 0 || L->glo < 0 || L->glo + L->gn > L->G) return hipSuccess;
    const dim3 grid(L->gn);
    if (L->mode == SCC_DE_FAST && L->test == SCC_TEST_T) {
        hipLaunchKernelGGL((k_gene_stats<true, true, false>), grid, dim3(ST_T), 0, st, *L);
        hipLaunchKernelGGL((k_gene_stats<false, false, true>), grid, dim3(ST_T), 0, st, *L);
    } else if (L->mode == SCC_DE_FAST) {
        hipLaunchKernelGGL((k_gene_stats<true, false, false>), grid, dim3(ST_T), 0, st, *L);
    } else {
        hipLaunchKernelGGL((k_gene_stats<false, true, false>), grid, dim3(ST_T), 0, st, *L);
    }
    return hipGetLastError();
}

// ===================================================================== classify
// counts: [0] small items, [1] medium items, [2] global-memory items, [3] split genes
#define SPLIT_BIG 32768
// split gene i of split_count(A) (the large ones first)
__device__ inline int split_count(const ScRankLaunch& A) { return A.counts[SCC_CNT_STRIDE * (3)] + A.counts[SCC_CNT_STRIDE * (13)]; }
// (nbig = A.counts[SCC_CNT_STRIDE * (13)], read once by the caller)
__device__ inline int split_gene_at(const ScRankLaunch& A, int nbig, int i)
{
    return i < nbig ? A.split_genes[A.G - 1 - i] : A.split_genes[i - nbig];
}

__global__ void k_rank_classify(ScRankLaunch A)
{
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= A.G) return;
    const i64 base = A.gstart[g];
    const i64 n = A.gstart[g + 1] - base;
    if (n <= 0) return;
    if (!A.all_pairs) {
        // 16 pairs' flags per round (clamped loads in flight together): an untested
        // gene costs P / 16 dependent rounds instead of P
        bool any = false;
        for (int p0 = 0; p0 < A.P && !any; p0 += 16) {
            u8 f[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) f[u] = A.flags[(size_t)min(p0 + u, A.P - 1) * A.G + g];
#pragma unroll
            for (int u = 0; u < 16; ++u) any |= (f[u] & 1) != 0;
        }
        if (!any) return;
    }
    // every ranked gene is split into value buckets; genes of >= SPLIT_BIG
    // values fill the list from its end (split_gene_at hands them out first:
    // the split's queue runs longest first, so a gene shard's largest genes
    // are not its tail)
    if (n >= SPLIT_BIG)
        A.split_genes[A.G - 1 - atomicAdd(&A.counts[SCC_CNT_STRIDE * (13)], 1)] = g;
    else
        A.split_genes[atomicAdd(&A.counts[SCC_CNT_STRIDE * (3)], 1)] = g;
}

extern "C" hipError_t scc_launch_rank_classify(const ScRankLaunch* L, hipStream_t st)
{
    hipLaunchKernelGGL(k_rank_classify, dim3((L->G + 255) / 256), dim3(256), 0, st, *L);
    return hipGetLastError();
}

// ===================================================================== radix
// LDS block state of the radix passes (W waves)
template <int W>
struct RadixLds {
    u32 hist[W * 256];
    u32 dtot[256 + W];
};

// One stable LSD pass of the digit dig(id) (< 2^BITS, BITS <= 8): in -> out.
// Each wave owns a contiguous range and per-(wave, digit) counters; inside a
// 64-element tile equal digits are ranked by lane (match by ballots), so one
// leader lane per distinct digit touches the counter: no LDS atomic ever
// conflicts.  Two tiles are in flight per wave; the returning adds of the
// scatter execute in tile order, which keeps the pass stable.
template <int W, int BITS, class IX, class DIG>
__device__ void radix_pass(DIG dig, const IX* in, IX* out, int n, RadixLds<W>& L)
{
    constexpr int U = 2;
    const int tid = threadIdx.x, lane = tid & 63, w = scc_wave_id();
    const int R = (((n + W - 1) / W) + 63) & ~63;
    const int lo = min(n, w * R), hi = min(n, lo + R);
    u32* hw = L.hist + w * 256;
    for (int d = lane; d < 256; d += 64) hw[d] = 0;
    __builtin_amdgcn_wave_barrier();
    for (int i0 = lo; i0 < hi; i0 += 64 * U) {
        u32 d[U];
        bool ok[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = i0 + 64 * u + lane;
            ok[u] = i < hi;
            d[u] = ok[u] ? dig(in[i]) : 0u;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const u64 peers = match_bits<BITS>(d[u], __ballot(ok[u]));
            if (ok[u] && lanes_below(peers) == 0)
                __hip_atomic_fetch_add(&hw[d[u]], (u32)__popcll(peers), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        }
    }
    __syncthreads();
    u32 tot = 0, incl = 0;
    if (tid < 256) {
        u32 c[W];
#pragma unroll
        for (int v = 0; v < W; ++v) c[v] = L.hist[v * 256 + tid];
        u32 s = 0;
#pragma unroll
        for (int v = 0; v < W; ++v) {
            L.hist[v * 256 + tid] = s;
            s += c[v];
        }
        tot = s;
        incl = s;
        for (int o = 1; o < 64; o <<= 1) {
            const u32 y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (lane == 63) L.dtot[256 + (tid >> 6)] = incl;
    }
    __syncthreads();
    if (tid < 256) {
        u32 base = incl - tot;
        for (int v = 0; v < (tid >> 6); ++v) base += L.dtot[256 + v];
#pragma unroll
        for (int v = 0; v < W; ++v) L.hist[v * 256 + tid] += base;
    }
    __syncthreads();
    for (int i0 = lo; i0 < hi; i0 += 64 * U) {
        u32 d[U];
        IX id[U];
        bool ok[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = i0 + 64 * u + lane;
            ok[u] = i < hi;
            id[u] = ok[u] ? in[i] : (IX)0;
            d[u] = ok[u] ? dig(id[u]) : 0u;
        }
        u32 b[U], rank[U];
        int leader[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const u64 peers = match_bits<BITS>(d[u], __ballot(ok[u]));
            rank[u] = lanes_below(peers);
            leader[u] = __builtin_ctzll(peers ? peers : 1ull);
            b[u] = 0;
            if (ok[u] && rank[u] == 0)
                b[u] = __hip_atomic_fetch_add(&hw[d[u]], (u32)__popcll(peers), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_WAVEFRONT);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const u32 bb = (u32)__shfl((int)b[u], leader[u], 64);
            if (ok[u]) out[bb + rank[u]] = id[u];
        }
    }
    __syncthreads();
}

// exact order of one mixed run (length <= 64) by (key, cluster, index): one wave
template <class KP, class IX>
__device__ void wave_sort_run(KP key, const u8* code, IX* ix, int s, int len)
{
    const int lane = threadIdx.x & 63;
    u64 k = ~0ull;
    u32 id = 0xffffffffu;
    if (lane < len) {
        id = (u32)ix[s + lane];
        k = key[id];
    }
    // secondary key: cluster code above the index (ties of equal doubles keep cluster order)
    u64 k2 = (lane < len) ? (((u64)code[id] << 32) | id) : ~0ull;
    for (int size = 2; size <= 64; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            const u64 ok = shfl_xor_u64(k, stride);
            const u64 ok2 = shfl_xor_u64(k2, stride);
            const bool up = (lane & size) == 0 || size == 64;
            const bool lower = (lane & stride) == 0;
            const bool other_less = (ok < k) || (ok == k && ok2 < k2);
            const bool take = (lower == up) ? other_less : !other_less;
            if (take) {
                k = ok;
                k2 = ok2;
            }
        }
    }
    if (lane < len) ix[s + lane] = (IX)(u32)k2;
}

// ===================================================================== item
#define RK_RUNS 256

template <int W>
struct ItemLds {
    RadixLds<W> rx;
    u32 m[SCC_MAX_K];       // nonzeros per cluster in this item
    u32 po[SCC_MAX_K + 1];  // position-list offsets
    u64 F[SCC_MAX_K];       // per-cluster tie term
    u64 red64[2 * W];  // min / max keys
    u32 redu[W + 1];
    int run_s[RK_RUNS], run_l[RK_RUNS];
    int nruns, flag, redo, anytie;
    int ntp, nchunk;
    u64 kmin, kmax;
    // tested pairs: packed (p | a << 16 | b << 23 | small-is-b << 30), chunk prefix
    u32 tp[1];  // dynamic tail: tp[ntp_max], cp[ntp_max + 1], eacc[ntp_max], xacc[ntp_max] (u64),
                // pmap[K * K] (u16: tested-pair slot + 1, 0 = untested)
};

__device__ inline int tp_p(u32 v) { return (int)(v & 0xffffu); }
__device__ inline int tp_a(u32 v) { return (int)((v >> 16) & 127u); }
__device__ inline int tp_b(u32 v) { return (int)((v >> 23) & 127u); }
__device__ inline bool tp_sb(u32 v) { return ((v >> 30) & 1u) != 0; }

// lower_bound of x in the ascending array s[0..len)
template <class IX>
__device__ inline u32 lower_bound_ix(const IX* s, u32 len, u32 x)
{
    u32 lo = 0;
    while (len > 0) {
        const u32 half = len >> 1;
        const bool lt = (u32)s[lo + half] < x;
        lo = lt ? lo + half + 1 : lo;
        len = lt ? len - half - 1 : half;
    }
    return lo;
}

// GLOBALMEM: every per-element array lives in HBM scratch (items too large
// for LDS); otherwise the key window, indices, codes and sorted codes are in
// LDS and the 64-bit keys stay in registers / L2.  KPT: keys per thread held
// in registers during the setup (LDS items: cap <= KPT * T).
template <int T, bool GLOBALMEM, int KPT>
__device__ void rank_one_item(const ScRankLaunch& A, const ScRankItem it, int item_no, char* smem)
{
    constexpr int W = T / 64;
    using IX = typename std::conditional<GLOBALMEM, u32, unsigned short>::type;
    const int K = A.K, P = A.P, G = A.G, g = it.gene, n = it.n;
    const int tid = threadIdx.x, lane = tid & 63, w = scc_wave_id();
    ItemLds<W>& L = *(ItemLds<W>*)smem;
    // tested-pair tables: in LDS after the fixed state, or (many tested pairs,
    // e.g. K > 64) in this workgroup's slice of an HBM scratch
    char* tab = A.tp_global ? (A.tp_scr + (size_t)blockIdx.x * A.tp_scr_stride) : (char*)L.tp;
    u32* tp = (u32*)tab;
    u32* cp = tp + A.ntp_max;
    u64* eacc = (u64*)(((uintptr_t)(cp + A.ntp_max + 1) + 7) & ~(uintptr_t)7);
    u64* xacc = eacc + A.ntp_max;
    unsigned short* pmap = (unsigned short*)(xacc + A.ntp_max);
    char* big = A.tp_global ? (char*)L.tp : (char*)(pmap + K * K);
    big = (char*)(((uintptr_t)big + 15) & ~(uintptr_t)15);
    u64* const stamps = A.stamps ? A.stamps + (size_t)item_no * 8 : nullptr;
#define ISTAMP(ph)                                                                   \
    do {                                                                             \
        if (stamps && threadIdx.x == 0) stamps[ph] = __builtin_amdgcn_s_memtime(); \
    } while (0)
    ISTAMP(0);
    // ---- per-element arrays
    const u64* key = (it.src ? A.keys2 : A.keys) + it.base;  // HBM / L2
    u32* win;
    u8 *code, *sc;
    IX *ix0, *ix1;
    if (GLOBALMEM) {
        win = A.gwin + it.base;
        code = it.src ? (A.codes2 + it.base) : (A.gcode + it.base);
        sc = A.gsc + it.base;
        ix0 = (IX*)(A.gix + it.base);
        ix1 = (IX*)(A.gix + A.nnz + it.base);
    } else {
        win = (u32*)big;
        ix0 = (IX*)(win + A.cap_lds);
        ix1 = ix0 + A.cap_lds;
        code = (u8*)(ix1 + A.cap_lds);
        sc = code + A.cap_lds;
    }
    // ---- setup: every global read issued before the first barrier
    int off_r = 0;
    if (it.src == 0 && tid <= K) off_r = (int)A.coff[(size_t)A.cl_cc[tid] * G + g];
    u64 kr[KPT];
    u64 kmn = ~0ull, kmx = 0;
    if (!GLOBALMEM) {
#pragma unroll
        for (int u = 0; u < KPT; ++u) {
            const int i = u * T + tid;
            kr[u] = (i < n) ? key[i] : 0ull;
        }
#pragma unroll
        for (int u = 0; u < KPT; ++u) {
            if (u * T + tid < n) {
                kmn = kr[u] < kmn ? kr[u] : kmn;
                kmx = kr[u] > kmx ? kr[u] : kmx;
            }
        }
    } else {
        for (int i = tid; i < n; i += T) {
            const u64 k = key[i];
            kmn = k < kmn ? k : kmn;
            kmx = k > kmx ? k : kmx;
        }
    }
    for (int m2 = 32; m2 >= 1; m2 >>= 1) {
        const u64 o1 = shfl_xor_u64(kmn, m2), o2 = shfl_xor_u64(kmx, m2);
        kmn = o1 < kmn ? o1 : kmn;
        kmx = o2 > kmx ? o2 : kmx;
    }
    if (tid < SCC_MAX_K) {
        L.m[tid] = 0;
        L.F[tid] = 0;
    }
    for (int i = tid; i < K * K; i += T) pmap[i] = 0;
    if (lane == 0) {
        L.red64[w] = kmn;
        L.red64[W + w] = kmx;
    }
    if (tid == 0) {
        L.nruns = 0;
        L.flag = 0;
        L.redo = 0;
        L.anytie = 0;
    }
    int* off = (int*)L.po;  // cluster offsets of a gene segment, until the position offsets exist
    if (it.src == 0 && tid <= K) off[tid] = off_r;
    // tested pairs of this gene, compacted in pair order (all of them in SLOW / test-all)
    {
        u32 basep = 0;
        for (int p0 = 0; p0 < P; p0 += T) {
            const int p = p0 + tid;
            const bool t = p < P && (A.all_pairs || (A.flags[(size_t)p * G + g] & 1));
            const u64 bal = __ballot(t);
            if (lane == 0) L.redu[w] = (u32)__popcll(bal);
            __syncthreads();
            u32 o = basep;
            for (int v = 0; v < w; ++v) o += L.redu[v];
            if (t) tp[o + lanes_below(bal)] = (u32)p;
            for (int v = 0; v < W; ++v) basep += L.redu[v];
            __syncthreads();
        }
        if (tid == 0) L.ntp = (int)basep;
    }
    // key range -> 32-bit window of (key - kmin)
    kmn = L.red64[0];
    kmx = L.red64[W];
    for (int v = 1; v < W; ++v) {
        kmn = L.red64[v] < kmn ? L.red64[v] : kmn;
        kmx = L.red64[W + v] > kmx ? L.red64[W + v] : kmx;
    }
    const u64 kmin = kmn, kmax = kmx;
    const u64 range = kmax - kmin;
    const int bits = range ? 64 - __clzll((long long)range) : 0;
    const int sh = bits > 32 ? bits - 32 : 0;
    if (!GLOBALMEM) {
#pragma unroll
        for (int u = 0; u < KPT; ++u) {
            const int i = u * T + tid;
            if (i < n) win[i] = (u32)((kr[u] - kmin) >> sh);
        }
    } else {
        for (int i = tid; i < n; i += T) win[i] = (u32)((key[i] - kmin) >> sh);
    }
    if (it.src == 0) {  // the ingest's cluster-grouped gene segment: codes from the offsets
        for (int a = 0; a < K; ++a) {
            const int s0 = off[a], s1 = off[a + 1];
            if (tid == 0) L.m[a] = (u32)(s1 - s0);
            for (int i = s0 + tid; i < s1; i += T) code[i] = (u8)a;
        }
    } else {
        for (int i0 = 0; i0 < n; i0 += T) {  // bucket: codes and cluster counts
            const int i = i0 + tid;
            const bool ok = i < n;
            const u32 c = ok ? A.codes2[it.base + i] : 0u;
            if (ok && !GLOBALMEM) code[i] = (u8)c;
            const u64 peers = match_bits<SCC_CODE_BITS>(c, __ballot(ok));
            if (ok && lanes_below(peers) == 0) atomicAdd(&L.m[c], (u32)__popcll(peers));
        }
    }
    __syncthreads();
    {
        // pack (pair, a, b, smaller side), one tested pair per thread, and chunk
        // the smaller side by 64 (chunk offsets: a workgroup exclusive scan)
        const int ntp0 = L.ntp;
        u32 basec = 0;
        for (int j0 = 0; j0 < ntp0; j0 += T) {
            const int j = j0 + tid;
            u32 nchk = 0;
            if (j < ntp0) {
                int a2, b2;
                pair_decode((int)tp[j], K, a2, b2);
                const u32 ma = L.m[a2], mb = L.m[b2];
                const bool sb = mb < ma;
                tp[j] = tp[j] | ((u32)a2 << 16) | ((u32)b2 << 23) | ((u32)sb << 30);
                pmap[a2 * K + b2] = (unsigned short)(j + 1);
                eacc[j] = 0;
                xacc[j] = 0;
                nchk = ((sb ? mb : ma) + 63) / 64;
            }
            u32 inc = nchk;
            for (int o = 1; o < 64; o <<= 1) {
                const u32 y = __shfl_up(inc, o, 64);
                if (lane >= o) inc += y;
            }
            if (lane == 63) L.redu[w] = inc;
            __syncthreads();
            u32 pre = basec;
            for (int v = 0; v < w; ++v) pre += L.redu[v];
            if (j < ntp0) cp[j] = pre + inc - nchk;
            for (int v = 0; v < W; ++v) basec += L.redu[v];
            __syncthreads();
        }
        if (tid == 0) {
        cp[ntp0] = basec;
        L.nchunk = (int)basec;
        u32 s2 = 0;
        for (int a3 = 0; a3 < K; ++a3) {
            L.po[a3] = s2;
            s2 += L.m[a3];
        }
        L.po[K] = s2;
        }
    }
    __syncthreads();
    const int ntp = L.ntp;
    if (it.bucket >= 0 && tid < K) A.hbg[(size_t)it.bucket * K + tid] = L.m[tid];
    ISTAMP(1);
    if (kmin == kmax) {
        // one distinct value: every pair is a tie, no order needed
        if (tid < K) {
            const u64 c = L.m[tid];
            if (c >= 2) atomicAdd((unsigned long long*)&A.accF[(size_t)tid * G + g], (unsigned long long)f_tie(c));
        }
        for (int j = tid; j < ntp; j += T) {
            const u32 v = tp[j];
            const u64 ca = L.m[tp_a(v)], cb = L.m[tp_b(v)];
            if (ca && cb) {
                atomicAdd((unsigned long long*)&A.accE[(size_t)tp_p(v) * G + g], (unsigned long long)(ca * cb));
                atomicAdd((unsigned long long*)&A.accX[(size_t)tp_p(v) * G + g],
                          (unsigned long long)(ca * cb * (ca + cb)));
            }
        }
        return;
    }
    // ---- stable sort by (value, cluster) on the 32-bit window
    for (int i = tid; i < n; i += T) ix0[i] = (IX)i;
    __syncthreads();
    IX* in = ix0;
    IX* out = ix1;
    if (it.src != 0) {  // bucket input is not cluster-grouped: stable pass on the cluster first
        radix_pass<W, SCC_CODE_BITS>([&](IX id) { return (u32)code[id]; }, in, out, n, L.rx);
        IX* t = in;
        in = out;
        out = t;
    }
    const int wbits = bits - sh;
    for (int p = 0; 8 * p < wbits; ++p) {
        const int s = 8 * p;
        radix_pass<W, 8>([&](IX id) { return (win[id] >> s) & 255u; }, in, out, n, L.rx);
        IX* t = in;
        in = out;
        out = t;
    }
    ISTAMP(2);
    if (sh > 0) {  // exact fix-up of windows that merged distinct doubles
        for (int i = tid; i + 1 < n; i += T) {
            const IX i0 = in[i], i1 = in[i + 1];
            if (win[i0] == win[i1] && key[i0] != key[i1]) L.flag = 1;
        }
        __syncthreads();
        if (L.flag) {
            for (int i = tid; i < n; i += T) {
                const u32 w0 = win[in[i]];
                const bool start = (i == 0 || win[in[i - 1]] != w0) && i + 1 < n && win[in[i + 1]] == w0;
                if (!start) continue;
                const u64 k0 = key[in[i]];
                int e = i + 1;
                bool mixed = false;
                while (e < n && win[in[e]] == w0) {
                    mixed |= key[in[e]] != k0;
                    ++e;
                }
                if (!mixed) continue;
                if (e - i <= 64) {
                    const int slot = atomicAdd(&L.nruns, 1);
                    if (slot < RK_RUNS) {
                        L.run_s[slot] = i;
                        L.run_l[slot] = e - i;
                    } else {
                        L.redo = 1;
                    }
                } else {
                    L.redo = 1;
                }
            }
            __syncthreads();
            if (L.redo) {  // pathological: exact LSD sort on every key bit (equal keys keep their order)
                for (int p = 0; 8 * p < bits; ++p) {
                    const int s = 8 * p;
                    radix_pass<W, 8>([&](IX id) { return (u32)((key[id] - kmin) >> s) & 255u; }, in, out, n, L.rx);
                    IX* t = in;
                    in = out;
                    out = t;
                }
            } else {
                // a mixed run holds one window: sort it exactly on (key, cluster, index)
                for (int r = w; r < L.nruns; r += W) wave_sort_run(key, code, in, L.run_s[r], L.run_l[r]);
                __syncthreads();
            }
        }
    }
    // sorted codes; bit 7: equal to the next element (a tie group continues)
    bool tie = false;
    for (int i = tid; i < n; i += T) {
        const IX id = in[i];
        bool eqn = false;
        if (i + 1 < n) {
            const IX id1 = in[i + 1];
            eqn = win[id1] == win[id] && (sh == 0 || key[id1] == key[id]);
        }
        tie |= eqn;
        sc[i] = (u8)(code[id] | (eqn ? 128 : 0));
    }
    if (__ballot(tie) && lane == 0) L.anytie = 1;
    __syncthreads();
    ISTAMP(3);
    // ---- positions partitioned by cluster (stable: ascending inside a cluster)
    IX* pl = out;  // the free index buffer
    {
        const int R = (((n + W - 1) / W) + 63) & ~63;
        const int lo = min(n, w * R), hi = min(n, lo + R);
        u32* hw = L.rx.hist + w * 256;
        for (int d = lane; d < SCC_MAX_K; d += 64) hw[d] = 0;
        __builtin_amdgcn_wave_barrier();
        for (int i0 = lo; i0 < hi; i0 += 64) {
            const int i = i0 + lane;
            const bool ok = i < hi;
            const u32 d = ok ? (sc[i] & SCC_CODE_MASK) : 0u;
            const u64 peers = match_bits<SCC_CODE_BITS>(d, __ballot(ok));
            if (ok && lanes_below(peers) == 0) hw[d] += (u32)__popcll(peers);
            __builtin_amdgcn_wave_barrier();
        }
        __syncthreads();
        if (tid < SCC_MAX_K) {  // per-(wave, cluster) start offsets
            u32 s = (tid < K) ? L.po[tid] : 0u;
            for (int v = 0; v < W; ++v) {
                const u32 c = L.rx.hist[v * 256 + tid];
                L.rx.hist[v * 256 + tid] = s;
                s += c;
            }
        }
        __syncthreads();
        for (int i0 = lo; i0 < hi; i0 += 64) {
            const int i = i0 + lane;
            const bool ok = i < hi;
            const u32 d = ok ? (sc[i] & SCC_CODE_MASK) : 0u;
            const u64 peers = match_bits<SCC_CODE_BITS>(d, __ballot(ok));
            if (ok) {
                const u32 rank = lanes_below(peers);
                const u32 b = hw[d];
                pl[b + rank] = (IX)i;
                if (rank == 0) hw[d] = b + (u32)__popcll(peers);
            }
            __builtin_amdgcn_wave_barrier();
        }
        __syncthreads();
    }
    ISTAMP(4);
    // ---- within-item S_ab for every tested pair: the smaller cluster's
    // positions binary-searched in the larger one's (positions are distinct)
    {
        const int nch = L.nchunk;
        int cur = -1;
        u64 acc = 0;
        for (int c = w; c < nch; c += W) {
            int lo = 0, hi = ntp;  // last j with cp[j] <= c (wave-uniform)
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if ((int)cp[mid] <= c) lo = mid;
                else hi = mid;
            }
            const int j = lo;
            if (j != cur) {
                if (cur >= 0) {
                    const u64 s = u64_wave_sum(acc);
                    if (lane == 0 && s)
                        atomicAdd((unsigned long long*)&A.accS[(size_t)tp_p(tp[cur]) * G + g], (unsigned long long)s);
                }
                cur = j;
                acc = 0;
            }
            const u32 v = tp[j];
            const int a = tp_a(v), b = tp_b(v);
            const bool sb = tp_sb(v);
            const int s = sb ? b : a, lg = sb ? a : b;
            const u32 ms = L.m[s];
            const u32 e = (u32)(c - (int)cp[j]) * 64u + (u32)lane;
            const u32 mlg = L.m[lg];
            const IX* lst = pl + L.po[lg];
            u32 x = 0;
            if (e < ms) x = (u32)pl[L.po[s] + e];
            const u32 lb = lower_bound_ix(lst, mlg, x);
            if (e < ms) acc += sb ? (u64)(mlg - lb) : (u64)lb;
        }
        if (cur >= 0) {
            const u64 s = u64_wave_sum(acc);
            if (lane == 0 && s)
                atomicAdd((unsigned long long*)&A.accS[(size_t)tp_p(tp[cur]) * G + g], (unsigned long long)s);
        }
    }
    ISTAMP(5);
    // ---- tie groups: runs of equal (value, cluster) inside groups of equal value
    if (L.anytie) {
        IX* rs = in;  // sorted order no longer needed: run starts
        // run start flags -> exclusive scan (per-thread contiguous chunks)
        const int chunk = (n + T - 1) / T;
        const int c0 = min(n, tid * chunk), c1 = min(n, c0 + chunk);
        u32 cnt = 0;
        for (int i = c0; i < c1; ++i) {
            const bool st = (i == 0) || !(sc[i - 1] & 128) || ((sc[i - 1] & SCC_CODE_MASK) != (sc[i] & SCC_CODE_MASK));
            cnt += st;
        }
        u32 incl = cnt;
        for (int o = 1; o < 64; o <<= 1) {
            const u32 y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (lane == 63) L.redu[w] = incl;
        __syncthreads();
        u32 basev = incl - cnt;
        for (int v = 0; v < w; ++v) basev += L.redu[v];
        if (tid == T - 1) L.redu[W] = basev + cnt;  // number of runs
        __syncthreads();
        const u32 nr = L.redu[W];
        // rs aliases the sorted-order buffer that is no longer read; the
        // starts are written after every thread finished reading it above
        for (int i = c0; i < c1; ++i) {
            const bool st = (i == 0) || !(sc[i - 1] & 128) || ((sc[i - 1] & SCC_CODE_MASK) != (sc[i] & SCC_CODE_MASK));
            if (st) rs[basev++] = (IX)i;
        }
        if (tid == 0) rs[nr] = (IX)n;
        __syncthreads();
        for (u32 r = tid; r < nr; r += T) {
            const u32 s0 = rs[r], len = (u32)rs[r + 1] - s0;
            const int a = sc[s0] & SCC_CODE_MASK;
            if (len >= 2) atomicAdd((unsigned long long*)&L.F[a], (unsigned long long)f_tie(len));
            // earlier runs of the same value: their clusters are smaller (codes
            // increase inside a group), each gives a cross-cluster tie block
            u32 q = r;
            while (q > 0 && (sc[(u32)rs[q] - 1] & 128)) {
                --q;
                const u32 ps = rs[q];
                const u64 lb = (u32)rs[q + 1] - ps, la = len;
                const int b = sc[ps] & SCC_CODE_MASK;  // b < a
                const int slot = pmap[b * K + a];
                if (slot) {
                    atomicAdd((unsigned long long*)&eacc[slot - 1], (unsigned long long)(la * lb));
                    atomicAdd((unsigned long long*)&xacc[slot - 1], (unsigned long long)(la * lb * (la + lb)));
                }
            }
        }
        __syncthreads();
        if (tid < K && L.F[tid])
            atomicAdd((unsigned long long*)&A.accF[(size_t)tid * G + g], (unsigned long long)L.F[tid]);
        for (int j = tid; j < ntp; j += T) {
            const int pp = tp_p(tp[j]);
            if (eacc[j]) atomicAdd((unsigned long long*)&A.accE[(size_t)pp * G + g], (unsigned long long)eacc[j]);
            if (xacc[j]) atomicAdd((unsigned long long*)&A.accX[(size_t)pp * G + g], (unsigned long long)xacc[j]);
        }
    }
    ISTAMP(6);
#undef ISTAMP
}

template <int T, bool GLOBALMEM, int KPT>
__global__ void __launch_bounds__(T, 4) k_rank_item(ScRankLaunch A, int cls)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int cnt = A.counts[SCC_CNT_STRIDE * (cls)];
    for (int i = blockIdx.x; i < cnt; i += gridDim.x) {
        const ScRankItem it = A.items[(size_t)cls * A.item_cap + i];
        rank_one_item<T, GLOBALMEM, KPT>(A, it, i + A.stamp_base[cls], smem);
        __syncthreads();
    }
}

#define RW_SLOTS_MAX 16  // tested pairs per gene the wave kernel holds: 64 * slots (2, 4, 8 or 16)
#define RW_PAIRS_MAX (8 * 64 * RW_SLOTS_MAX)  // genes past 1024 tested pairs: one 16-slot pass per 1024
#define RS_ACC_MAX (SCC_MAX_K * (SCC_MAX_K - 1) / 2)  // re-split: in-parent cross terms of every tested pair sum in LDS
#define RS_T 256          // re-split: threads per workgroup
#define RS_SLICES 8       // re-split: workgroups sharing one gene's large parents
#define RS_KPT 8          // keys per thread (held in registers: the scatter is in place)
#define RS_CAP (RS_T * RS_KPT)
#define RS_LOG2B 9
#define RS_BINS (1 << RS_LOG2B)
#define RS_BMAX (2 * RS_BINS + 1)
#define RS_HCAP 2048      // sub-bucket x cluster histogram entries held in LDS
#define RSW_LOG2B 8       // wave re-split: parents of <= RSW_CAP elements, 256 bins
#define RSW_BINS (1 << RSW_LOG2B)
#define RSW_CAP 256
#define RSW_HCAP 512
#define RSW_PACC 1280     // genes with <= this many tested pairs keep them (and their sums) in registers
#define RSW_TS_SMALL 8    // the wave re-split's launch for genes with <= 512 tested pairs

// ===================================================================== split
#define SP_T 1024
#define SP_W (SP_T / 64)
#define SP_BINS 2048
#define SP_BMAX (2 * SP_BINS + 1)  // a bucket starts at a bin, or right after a fat bin
#define SP_KPT 8                    // keys per thread held in registers across the passes
#define SP_CHUNK (SP_T * SP_KPT)
#define SP_SUP 4096  // two-level scatter: group width (a group holds < 2 * SP_SUP = SP_CHUNK values)
#define SP_NSUP 1022 // groups a gene may have (three [SP_NSUP + 1] u32 tables fit the excl table)

struct SplitLds {
    u32 hist[SP_BINS];
    u32 excl[SP_BINS];
    u32 bid[SP_BINS];   // bucket of each bin
    u32 bcur[SP_BMAX];  // bucket cursors
    u32 boff[SP_BMAX + 1];
    u64 rep[SP_BINS];      // one key of each bin (any: the last leader's store wins)
    u8 bdiff[SP_BMAX + 3]; // bucket holds two different keys
    u32 wsum[SP_W + 1];
    u32 wsum2[SP_W + 1];
    u64 rmn[SP_W], rmx[SP_W];
    u32 cdf[SP_BINS + 1];  // the linear window's counts, scanned: the equalized bins' map
    int off[SCC_MAX_K + 1];
    int nb, bk0, next;
    int nfat, fat0, nwav, wav0;
    int nsup;
};
// the split's LDS: its tables, then the bucket-order staging of a gene that
// fits one register chunk (SP_CHUNK keys + codes)
static constexpr size_t kSplitStageOff = (sizeof(SplitLds) + 15) & ~(size_t)15;
static_assert(kSplitStageOff + (size_t)SP_CHUNK * 9 <= 160 * 1024, "split LDS");


// One ranked gene: 2048-bin histogram of its key window, bins packed into
// value buckets of < 2 * target elements (a bin of more than `target` is a
// bucket of its own), elements scattered into bucket order (keys2 / codes2
// over the gene's own range).  Buckets of <= 64 elements go to the wave
// kernel, larger ones (fat bins) to the LDS item kernel.  Every bucket gets a
// global id: its cluster histogram row in hbg, written by whoever ranks it.
__device__ void split_one_gene(const ScRankLaunch& A, int g, SplitLds& L)
{
    const int K = A.K, G = A.G;
    const int tid = threadIdx.x, lane = tid & 63, w = scc_wave_id();
    const i64 base = A.gstart[g];
    const int n = (int)(A.gstart[g + 1] - base);
    const u64* key = A.keys + base;
    if (tid <= K) L.off[tid] = (int)A.coff[(size_t)A.cl_cc[tid] * G + g];
    for (int i = tid; i < SP_BINS; i += SP_T) L.hist[i] = 0;
    // tested pairs of the gene (the wave kernel holds at most 64 * A.rw_slots),
    // compacted in pair order into gene_tp[g] as p | a << 16 | b << 24
    u32 ntested = 0;
    for (int p0 = 0; p0 < A.P; p0 += SP_T) {
        const int p = p0 + tid;
        const bool t = p < A.P && (A.all_pairs || (A.flags[(size_t)p * G + g] & 1));
        const u64 bal = __ballot(t);
        if (lane == 0) L.wsum2[w] = (u32)__popcll(bal);
        __syncthreads();
        u32 o = ntested;
        for (int v = 0; v < w; ++v) o += L.wsum2[v];
        if (t) {
            int a2, b2;
            pair_decode(p, K, a2, b2);
            A.gene_tp[(size_t)g * A.P + o + lanes_below(bal)] = (u32)p | ((u32)a2 << 16) | ((u32)b2 << 24);
        }
        for (int v = 0; v < SP_W; ++v) ntested += L.wsum2[v];
        __syncthreads();
    }
    if (tid == 0) A.gene_nt[g] = (int)ntested;
    const bool waves_ok = ntested <= (A.rw_slots >= RW_SLOTS_MAX ? (u32)RW_PAIRS_MAX : 64u * (u32)A.rw_slots);
    // the gene's keys stay in registers when they fit (SP_KPT per thread);
    // larger genes re-read each chunk in every pass (from L2)
    u64 kr[SP_KPT];
    auto load_chunk = [&](int c0) {
#pragma unroll
        for (int q = 0; q < SP_KPT; ++q) {
            const int i = c0 + q * SP_T + tid;
            kr[q] = i < n ? key[i] : 0ull;
        }
    };
    load_chunk(0);
    // key range of the gene (min / max over its nonzeros)
    u64 kmn = ~0ull, kmx = 0;
    for (int c0 = 0; c0 < n; c0 += SP_CHUNK) {
        if (c0) load_chunk(c0);
#pragma unroll
        for (int q = 0; q < SP_KPT; ++q) {
            if (c0 + q * SP_T + tid < n) {
                kmn = kr[q] < kmn ? kr[q] : kmn;
                kmx = kr[q] > kmx ? kr[q] : kmx;
            }
        }
    }
    for (int m2 = 32; m2 >= 1; m2 >>= 1) {
        const u64 o1 = shfl_xor_u64(kmn, m2), o2 = shfl_xor_u64(kmx, m2);
        kmn = o1 < kmn ? o1 : kmn;
        kmx = o2 > kmx ? o2 : kmx;
    }
    if (lane == 0) {
        L.rmn[w] = kmn;
        L.rmx[w] = kmx;
    }
    __syncthreads();
    kmn = L.rmn[0];
    kmx = L.rmx[0];
    for (int v = 1; v < SP_W; ++v) {
        kmn = L.rmn[v] < kmn ? L.rmn[v] : kmn;
        kmx = L.rmx[v] > kmx ? L.rmx[v] : kmx;
    }
    const u64 range = kmx - kmn;
    const int bits = range ? 64 - __clzll((long long)range) : 0;
    const int sh = bits > 11 ? bits - 11 : 0;
    if (tid == 0) A.gkmin[g] = bits <= 64 - SCC_CODE_BITS ? kmn : ~0ull;  // wave kernel: (key - kmin) << 7 | cluster
    // ---- 1. equalized bins.  A linear 2048-bin window over the gene's whole
    // key range puts hundreds of distinct values into one bin where the values
    // crowd (at 200k cells: the count-1 band of a dense gene), and every such
    // bin cost a re-split (k_rank_resplit*: 8 ms of config D's rank stage).
    // So the linear histogram is a first look: where a bin holds more than 64
    // elements, its scan (cdf) maps a key
    // to  floor(2048 (cdf[j] + f h_j) / n)  (j its linear bin, f its place in
    // it, h_j the bin's count) -- the gene's empirical CDF, interpolated --
    // and the buckets are cut on those bins.  The map is non-decreasing in the
    // key (every operation is a correctly rounded monotone one), so a bin is a
    // key interval: equal values never straddle bins and order is kept.
    // A gene whose linear bins all hold <= 64 elements keeps them (no second pass).
    for (int c0 = 0; c0 < n; c0 += SP_CHUNK) {
        if (n > SP_CHUNK) load_chunk(c0);
#pragma unroll
        for (int q = 0; q < SP_KPT; ++q) {
            if (c0 + q * SP_T + tid < n) {
                const u32 d = (u32)((kr[q] - kmn) >> sh);
                atomicAdd(&L.hist[d], 1u);
                L.rep[d] = kr[q];
            }
        }
    }
    __syncthreads();
    const bool equalize = __syncthreads_or(L.hist[2 * tid] > 64u || L.hist[2 * tid + 1] > 64u) != 0;
    if (equalize) {
        const u32 h0 = L.hist[2 * tid], h1 = L.hist[2 * tid + 1];
        const u32 v = h0 + h1;
        u32 incl = v;
        for (int o = 1; o < 64; o <<= 1) {
            const u32 y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (lane == 63) L.wsum[w] = incl;
        __syncthreads();
        u32 b = incl - v;
        for (int q = 0; q < w; ++q) b += L.wsum[q];
        L.cdf[2 * tid] = b;
        L.cdf[2 * tid + 1] = b + h0;
        if (tid == SP_T - 1) L.cdf[SP_BINS] = (u32)n;
        L.hist[2 * tid] = 0;
        L.hist[2 * tid + 1] = 0;
    }
    __syncthreads();
    const double inv_w = ldexp(1.0, -sh), bin_scale = (double)SP_BINS / (double)max(n, 1);
    auto binof = [&](u64 k) -> u32 {
        const u64 x = k - kmn;
        const u32 j = (u32)(x >> sh);
        if (!equalize) return j;
        const u32 lo = L.cdf[j], h = L.cdf[j + 1] - lo;
        const double f = (double)(x - ((u64)j << sh)) * inv_w;
        const u32 d = (u32)(((double)lo + f * (double)h) * bin_scale);
        return d < SP_BINS ? d : SP_BINS - 1;
    };
    // histogram of the equalized bins (one LDS atomic per element; any key of
    // a bin is kept as its representative)
    for (int c0 = 0; c0 < n && equalize; c0 += SP_CHUNK) {
        if (n > SP_CHUNK) load_chunk(c0);
#pragma unroll
        for (int q = 0; q < SP_KPT; ++q) {
            if (c0 + q * SP_T + tid < n) {
                const u32 d = binof(kr[q]);
                atomicAdd(&L.hist[d], 1u);
                L.rep[d] = kr[q];
            }
        }
    }
    __syncthreads();
    // ---- 2. exclusive scan of the bins (2 per thread)
    {
        const u32 h0 = L.hist[2 * tid], h1 = L.hist[2 * tid + 1];
        const u32 v = h0 + h1;
        u32 incl = v;
        for (int o = 1; o < 64; o <<= 1) {
            const u32 y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (lane == 63) L.wsum[w] = incl;
        __syncthreads();
        u32 b = incl - v;
        for (int q = 0; q < w; ++q) b += L.wsum[q];
        L.excl[2 * tid] = b;
        L.excl[2 * tid + 1] = b + h0;
    }
    __syncthreads();
    // ---- 3. buckets: runs of bins with equal floor(excl / target); a bin of
    // more than `target` elements is a bucket of its own
    const u32 target = (u32)A.wave_target;
    {
        u32 st[2];
        for (int q = 0; q < 2; ++q) {
            const int d = 2 * tid + q;
            const bool fat = L.hist[d] > target;
            const bool pfat = d > 0 && L.hist[d - 1] > target;
            st[q] = (d == 0) || fat || pfat || (L.excl[d] / target != L.excl[d - 1] / target);
        }
        const u32 v = st[0] + st[1];
        u32 incl = v;
        for (int o = 1; o < 64; o <<= 1) {
            const u32 y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (lane == 63) L.wsum2[w] = incl;
        __syncthreads();
        u32 b = incl - v;
        for (int q = 0; q < w; ++q) b += L.wsum2[q];
        L.bid[2 * tid] = b + st[0] - 1;
        L.bid[2 * tid + 1] = b + st[0] + st[1] - 1;
        if (st[0]) L.boff[b] = L.excl[2 * tid];
        if (st[1]) L.boff[b + st[0]] = L.excl[2 * tid + 1];
        if (tid == SP_T - 1) {
            L.nb = (int)(b + v);
            L.boff[b + v] = (u32)n;
            L.bk0 = atomicAdd(&A.counts[SCC_CNT_STRIDE * (5)], (int)(b + v));
            A.gene_bk[2 * g] = L.bk0;
            A.gene_bk[2 * g + 1] = (int)(b + v);
        }
    }
    __syncthreads();
    const int nb = L.nb, bk0 = L.bk0;
    for (int q = tid; q < nb; q += SP_T) {
        L.bcur[q] = L.boff[q];
        L.bdiff[q] = 0;
    }
    __syncthreads();
    // ---- 4. scatter into bucket order (keys2 / codes2 over the gene's own range);
    // the order inside a bucket is arbitrary (its ranker sorts by key and cluster).
    // A gene of one register chunk is ordered in LDS and leaves as whole lines
    // (scattered 8-byte / 1-byte stores wrote each line several times over:
    // 3.8x the keys2 + codes2 bytes at config D).  A larger gene goes in two
    // levels: its buckets grouped into super-buckets (runs of buckets whose
    // starts share floor(offset / SP_SUP); a bucket of more than SP_SUP values
    // alone, so a group holds < SP_CHUNK), the values scattered into group
    // order (a chunk's values land in a few dozen runs: whole lines), then each
    // group of two or more buckets reloaded, ordered in LDS and written back.
    // The one-level scatter's scattered stores were ~2/3 of a large gene's
    // split time (8.4 -> 3.0 cycles per value without them at config D).
    // A gene past SP_NSUP groups: the one-level scatter.
    const bool staged = n <= SP_CHUNK;
    u64* stk = (u64*)((char*)&L + kSplitStageOff);
    u8* stc = (u8*)(stk + SP_CHUNK);
    // group tables over the bin tables the layout no longer needs (hist and
    // excl, adjacent: 4096 words): the bins' group ids in the first 1024, then
    // three [SP_NSUP + 1] tables
    static_assert(offsetof(SplitLds, excl) == offsetof(SplitLds, hist) + sizeof(u32) * SP_BINS, "hist | excl");
    static_assert(SP_BINS / 2 + 3 * (SP_NSUP + 1) <= 2 * SP_BINS, "group tables");
    unsigned short* supbin = (unsigned short*)L.hist;  // [SP_BINS] group of each bin
    u32* sbeg = L.hist + SP_BINS / 2;                  // [SP_NSUP + 1] group starts (offsets)
    u32* sbk = sbeg + (SP_NSUP + 1);                   // [SP_NSUP + 1] first bucket of each group
    u32* scur = sbk + (SP_NSUP + 1);                   // [SP_NSUP] group cursors
    bool two = !staged;
    if (two) {
        // group starts over the bins, 2 per thread (the bucket rule's scan)
        auto big = [&](u32 b) { return L.boff[b + 1] - L.boff[b] > (u32)SP_SUP; };
        u32 st[2], bq[2];
        for (int q = 0; q < 2; ++q) {
            const int d = 2 * tid + q;
            const u32 b = L.bid[d];
            bq[q] = b;
            const u32 bp = d > 0 ? L.bid[d - 1] : b;
            st[q] = (d == 0) || (bp != b && (big(b) || big(bp) || L.boff[b] / SP_SUP != L.boff[bp] / SP_SUP));
        }
        const u32 v = st[0] + st[1];
        u32 incl = v;
        for (int o = 1; o < 64; o <<= 1) {
            const u32 y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (lane == 63) L.wsum2[w] = incl;
        __syncthreads();
        u32 sb = incl - v;
        for (int q = 0; q < w; ++q) sb += L.wsum2[q];
        const u32 ns = [&] {
            u32 t = 0;
            for (int q = 0; q < SP_W; ++q) t += L.wsum2[q];
            return t;
        }();
        if (ns <= SP_NSUP) {
            for (int q = 0; q < 2; ++q) {
                sb += st[q];
                if (st[q]) {
                    sbeg[sb - 1] = L.boff[bq[q]];
                    sbk[sb - 1] = bq[q];
                    scur[sb - 1] = L.boff[bq[q]];
                }
            }
            // (the writes above use the per-thread running index; store the bin's group after)
        }
        __syncthreads();  // every thread has read the bin tables' old contents (hist / excl no longer read)
        if (ns <= SP_NSUP) {
            u32 sb2 = incl - v;
            for (int q = 0; q < w; ++q) sb2 += L.wsum2[q];
            for (int q = 0; q < 2; ++q) {
                sb2 += st[q];
                supbin[2 * tid + q] = (unsigned short)(sb2 - 1);
            }
            if (tid == 0) {
                sbeg[ns] = (u32)n;
                sbk[ns] = (u32)nb;
            }
        }
        two = ns <= SP_NSUP;  // (block-uniform)
        if (tid == 0) L.nsup = (int)ns;
        __syncthreads();
    }
    if (two) {  // first level: straight to the group cursors
        // (staging each chunk in LDS by group first, for whole-line stores,
        // measured no faster at config D for genes from 32k, 64k or 128k values)
        for (int c0 = 0; c0 < n; c0 += SP_CHUNK) {
            load_chunk(c0);
            int a = 0;
#pragma unroll
            for (int q = 0; q < SP_KPT; ++q) {
                const int i = c0 + q * SP_T + tid;
                if (i < n) {
                    while (a + 1 < K && L.off[a + 1] <= i) ++a;
                    const u64 k = kr[q];
                    const u32 d = binof(k);
                    const u32 pos = atomicAdd(&scur[supbin[d]], 1u);
                    A.keys2[base + pos] = k;
                    A.codes2[base + pos] = (u8)a;
                    if (k != L.rep[d]) L.bdiff[L.bid[d]] = 1;
                }
            }
        }
    }
    for (int c0 = 0; c0 < n && !two; c0 += SP_CHUNK) {
        if (n > SP_CHUNK) load_chunk(c0);
        int a = 0;
#pragma unroll
        for (int q = 0; q < SP_KPT; ++q) {
            const int i = c0 + q * SP_T + tid;
            if (i < n) {
                while (a + 1 < K && L.off[a + 1] <= i) ++a;
                const u64 k = kr[q];
                const u32 d = binof(k);
                const u32 bk = L.bid[d];
                const u32 pos = atomicAdd(&L.bcur[bk], 1u);
                if (staged) {
                    stk[pos] = k;
                    stc[pos] = (u8)a;
                } else if (A.dbg != 10) {  // (SCC_RW_DEBUG=10: timing cut, no unstaged stores; results invalid)
                    A.keys2[base + pos] = k;
                    A.codes2[base + pos] = (u8)a;
                }
                if (k != L.rep[d]) L.bdiff[bk] = 1;
            }
        }
    }
    __syncthreads();
    if (staged) {
        for (int i = tid; i < n; i += SP_T) {
            A.keys2[base + i] = stk[i];
            A.codes2[base + i] = stc[i];
        }
    }
    if (two) {  // second level: each group of >= 2 buckets ordered in LDS, in place
        const int ns = L.nsup;
        for (int sg = 0; sg < ns; ++sg) {
            if (sbk[sg + 1] - sbk[sg] < 2) continue;  // one bucket: in place already (block-uniform)
            const u32 o0 = sbeg[sg], m = sbeg[sg + 1] - o0;  // m < SP_CHUNK
            if (m == 0) continue;
            u64 kv[SP_KPT];
            u8 cv[SP_KPT];
#pragma unroll
            for (int q = 0; q < SP_KPT; ++q) {  // clamped unconditional loads (all in flight)
                const u32 j = (u32)(q * SP_T + tid);
                const u32 jc = j < m ? j : m - 1;
                kv[q] = A.keys2[base + o0 + jc];
                cv[q] = A.codes2[base + o0 + jc];
            }
#pragma unroll
            for (int q = 0; q < SP_KPT; ++q) {
                if ((u32)(q * SP_T + tid) < m) {
                    const u32 d = binof(kv[q]);
                    const u32 p = atomicAdd(&L.bcur[L.bid[d]], 1u) - o0;
                    stk[p] = kv[q];
                    stc[p] = cv[q];
                }
            }
            __syncthreads();
            for (u32 j = tid; j < m; j += SP_T) {
                A.keys2[base + o0 + j] = stk[j];
                A.codes2[base + o0 + j] = stc[j];
            }
            __syncthreads();
        }
    }
    // ---- 5. one work unit per bucket (empty buckets: a zero histogram row).
    // Wave buckets and re-split parents are reserved once per gene (one global
    // atomic each, not one per bucket) and placed with LDS cursors.
    auto kind = [&](int q) {  // 0 none, 1 wave bucket, 2 re-split parent, 3 LDS item
        const int c = (int)(L.boff[q + 1] - L.boff[q]);
        if (c <= 0) return 0;
        const bool ties_only = c > 64 && !L.bdiff[q];
        if ((c <= 64 || ties_only) && waves_ok) return 1;
        if (waves_ok && c <= RS_CAP && A.fatbk) return 2;
        return 3;
    };
    if (tid == 0) {
        L.nfat = 0;
        L.nwav = 0;
    }
    __syncthreads();
    for (int q = tid; q < nb; q += SP_T) {
        const int k = kind(q);
        if (k == 1) atomicAdd(&L.nwav, 1);
        if (k == 2) atomicAdd(&L.nfat, 1);
    }
    __syncthreads();
    if (tid == 0) {
        L.wav0 = L.nwav ? atomicAdd(&A.counts[SCC_CNT_STRIDE * (4)], L.nwav) : 0;
        L.fat0 = -1;
        if (L.nfat) {
            const int f0 = atomicAdd(&A.counts[SCC_CNT_STRIDE * (8)], L.nfat);
            if (f0 + L.nfat <= A.fat_cap) {
                L.fat0 = f0;
                A.fatg[atomicAdd(&A.counts[SCC_CNT_STRIDE * (11)], 1)] = int4{g, f0, L.nfat, 0};
            }
        }
        L.nfat = 0;
        L.nwav = 0;
    }
    __syncthreads();
    for (int q = tid; q < nb; q += SP_T) {
        const int c = (int)(L.boff[q + 1] - L.boff[q]);
        const int bid = bk0 + q;
        const int k = kind(q);
        if (k == 0) {
            for (int k2 = 0; k2 < K; ++k2) A.hbg[(size_t)bid * K + k2] = 0;
            continue;
        }
        // a bucket of one repeated key (a fat bin of ties): closed form in the wave kernel
        const bool ties_only = c > 64 && !L.bdiff[q];
        const ScRankItem itm{base + L.boff[q], c, g, ties_only ? 2 : 1, bid};
        if (k == 1) {
            A.sbuckets[L.wav0 + atomicAdd(&L.nwav, 1)] = itm;
        } else if (k == 2 && L.fat0 >= 0) {
            // > 64 distinct values in one bin: re-split on a finer window (k_rank_resplit)
            A.fatbk[L.fat0 + atomicAdd(&L.nfat, 1)] = itm;
        } else {
            const int cls = (c <= A.cap_s) ? 0 : ((c <= A.cap_m) ? 1 : 2);
            A.items[(size_t)cls * A.item_cap + atomicAdd(&A.counts[SCC_CNT_STRIDE * (cls)], 1)] = itm;
        }
    }
    __syncthreads();
}

// SCC_RW_DEBUG=9: per split gene (stored values, cycles) of the first
// SPLIT_DIAG_MAX genes, printed as a distribution (scc_rank_split_diag)
#define SPLIT_DIAG_MAX 65536
__device__ unsigned long long g_split_diag[SPLIT_DIAG_MAX][2];

__global__ void __launch_bounds__(SP_T) k_rank_split(ScRankLaunch A)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    SplitLds& L = *(SplitLds*)smem;
    const int cnt = split_count(A), nbig = A.counts[SCC_CNT_STRIDE * (13)];
    for (;;) {  // genes from a queue (their sizes vary by orders of magnitude)
        if (threadIdx.x == 0) L.next = atomicAdd(&A.counts[SCC_CNT_STRIDE * (6)], 1);
        __syncthreads();
        const int i = L.next;
        if (i >= cnt) break;
        const u64 t0 = A.dbg >= 9 ? __builtin_amdgcn_s_memtime() : 0;
        split_one_gene(A, split_gene_at(A, nbig, i), L);
        if (A.dbg >= 9 && threadIdx.x == 0 && i < SPLIT_DIAG_MAX) {
            const int g = split_gene_at(A, nbig, i);
            g_split_diag[i][0] = (unsigned long long)(A.gstart[g + 1] - A.gstart[g]);
            g_split_diag[i][1] = __builtin_amdgcn_s_memtime() - t0;
        }
    }
}

extern "C" void scc_rank_split_diag(hipStream_t st, int ngenes)
{
    static unsigned long long h[SPLIT_DIAG_MAX][2];
    const int n = ngenes < SPLIT_DIAG_MAX ? ngenes : SPLIT_DIAG_MAX;
    if (n <= 0 || hipStreamSynchronize(st) != hipSuccess ||
        hipMemcpyFromSymbol(h, HIP_SYMBOL(g_split_diag), sizeof(unsigned long long) * 2 * n, 0,
                            hipMemcpyDeviceToHost) != hipSuccess)
        return;
    std::vector<int> ix(n);
    for (int i = 0; i < n; ++i) ix[i] = i;
    std::sort(ix.begin(), ix.end(), [&](int a, int b) { return h[a][1] > h[b][1]; });
    unsigned long long tot = 0, totn = 0;
    for (int i = 0; i < n; ++i) {
        tot += h[i][1];
        totn += h[i][0];
    }
    fprintf(stderr, "[scc split diag] genes %d values %llu cycles %llu (mean %.0f per gene, %.1f per value); slowest:", n,
            totn, tot, (double)tot / n, (double)tot / std::max(1ull, totn));
    for (int q = 0; q < std::min(n, 12); ++q) fprintf(stderr, " %llu/%llu", h[ix[q]][0], h[ix[q]][1]);
    fprintf(stderr, "\n");
}

// ===================================================================== re-split
// A bucket the split left with > 64 distinct values (a dense stretch of the
// value axis: at 100k+ cells a 2048-bin window over the gene's whole range
// puts hundreds of values in one bin) is split again on its own key window:
// 512 bins, the same packing rule, elements scattered in place (all of them
// are in registers first).  The sub-buckets go to the wave kernel; the
// parent keeps its cluster histogram row (the gene-level cross term of
// k_rank_cross) and records its sub-bucket range, whose in-parent cross term
// k_rank_cross_seg adds from the sub-buckets' rows.
struct ResplitLds {
    u32 hist[RS_BINS];
    u32 excl[RS_BINS];
    u32 bid[RS_BINS];
    u64 rep[RS_BINS];
    u32 bcur[RS_BMAX];
    u32 boff[RS_BMAX + 1];
    u8 bdiff[RS_BMAX + 3];
    u32 m[SCC_MAX_K];
    u32 wsum[RS_T / 64 + 1];
    u32 wsum2[RS_T / 64 + 1];
    u64 rmn[RS_T / 64], rmx[RS_T / 64];
    u32 hs[RS_HCAP];  // [sub-bucket][cluster] counts (in-parent cross term), when nb * K fits
    u32 bs[RS_HCAP];  // [sub-bucket][cluster] elements of the cluster in lower sub-buckets
    int nb, bk0, next, ovf, nw, w0;
};

// A sub-bucket that still holds > 64 distinct values goes to the second
// re-split level (k_rank_resplit_w with rs_level 1) while its list has room.
__device__ inline bool push_fat2(const ScRankLaunch& A, const ScRankItem& itm)
{
    const int f = atomicAdd(&A.counts[SCC_CNT_STRIDE * (12)], 1);
    if (f >= A.fat2_cap) return false;
    A.fat2[f] = itm;
    return true;
}

__device__ void resplit_one(const ScRankLaunch& A, const ScRankItem it, ResplitLds& L, u64* __restrict__ acc)
{
    constexpr int W = RS_T / 64, BPT = RS_BINS / RS_T;
    const int K = A.K, g = it.gene, n = it.n;
    const int tid = threadIdx.x, lane = tid & 63, w = scc_wave_id();
    u64 t_prev = A.stamps ? __builtin_amdgcn_s_memtime() : 0;
#define RSTAMP(ph)                                                                         \
    do {                                                                                   \
        if (A.stamps && tid == 0) {                                                        \
            const u64 t_now = __builtin_amdgcn_s_memtime();                               \
            atomicAdd((unsigned long long*)&A.stamps[ph], (unsigned long long)(t_now - t_prev)); \
            t_prev = t_now;                                                                \
        }                                                                                  \
    } while (0)
    u64 kr[RS_KPT];
    u8 cd[RS_KPT];
#pragma unroll
    for (int q = 0; q < RS_KPT; ++q) {
        const int i = q * RS_T + tid;
        kr[q] = i < n ? A.keys2[it.base + i] : 0ull;
        cd[q] = i < n ? A.codes2[it.base + i] : (u8)0;
    }
    for (int d = tid; d < RS_BINS; d += RS_T) L.hist[d] = 0;
    if (tid < SCC_MAX_K) L.m[tid] = 0;
    u64 kmn = ~0ull, kmx = 0;
#pragma unroll
    for (int q = 0; q < RS_KPT; ++q) {
        if (q * RS_T + tid < n) {
            kmn = kr[q] < kmn ? kr[q] : kmn;
            kmx = kr[q] > kmx ? kr[q] : kmx;
        }
    }
    for (int m2 = 32; m2 >= 1; m2 >>= 1) {
        const u64 o1 = shfl_xor_u64(kmn, m2), o2 = shfl_xor_u64(kmx, m2);
        kmn = o1 < kmn ? o1 : kmn;
        kmx = o2 > kmx ? o2 : kmx;
    }
    if (lane == 0) {
        L.rmn[w] = kmn;
        L.rmx[w] = kmx;
    }
    __syncthreads();
    kmn = L.rmn[0];
    kmx = L.rmx[0];
    for (int v = 1; v < W; ++v) {
        kmn = L.rmn[v] < kmn ? L.rmn[v] : kmn;
        kmx = L.rmx[v] > kmx ? L.rmx[v] : kmx;
    }
    RSTAMP(0);
    const u64 range = kmx - kmn;
    const int bits = range ? 64 - __clzll((long long)range) : 0;
    const int sh = bits > RS_LOG2B ? bits - RS_LOG2B : 0;
#pragma unroll
    for (int q = 0; q < RS_KPT; ++q) {
        if (q * RS_T + tid < n) {
            const u32 d = (u32)((kr[q] - kmn) >> sh);
            atomicAdd(&L.hist[d], 1u);
            L.rep[d] = kr[q];
            atomicAdd(&L.m[cd[q]], 1u);
        }
    }
    __syncthreads();
    // exclusive scan of the bins (BPT consecutive bins per thread)
    {
        u32 h[BPT], v = 0;
#pragma unroll
        for (int q = 0; q < BPT; ++q) {
            h[q] = L.hist[BPT * tid + q];
            v += h[q];
        }
        u32 incl = v;
        for (int o = 1; o < 64; o <<= 1) {
            const u32 y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (lane == 63) L.wsum[w] = incl;
        __syncthreads();
        u32 b = incl - v;
        for (int q = 0; q < w; ++q) b += L.wsum[q];
#pragma unroll
        for (int q = 0; q < BPT; ++q) {
            L.excl[BPT * tid + q] = b;
            b += h[q];
        }
    }
    __syncthreads();
    // buckets: runs of bins with equal floor(excl / target); a bin of more
    // than `target` elements is a bucket of its own (the split's rule)
    const u32 target = (u32)A.wave_target;
    {
        u32 st[BPT], v = 0;
#pragma unroll
        for (int q = 0; q < BPT; ++q) {
            const int d = BPT * tid + q;
            const bool fat = L.hist[d] > target;
            const bool pfat = d > 0 && L.hist[d - 1] > target;
            st[q] = (d == 0) || fat || pfat || (L.excl[d] / target != L.excl[d - 1] / target);
            v += st[q];
        }
        u32 incl = v;
        for (int o = 1; o < 64; o <<= 1) {
            const u32 y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (lane == 63) L.wsum2[w] = incl;
        __syncthreads();
        u32 b = incl - v;
        for (int q = 0; q < w; ++q) b += L.wsum2[q];
#pragma unroll
        for (int q = 0; q < BPT; ++q) {
            const int d = BPT * tid + q;
            if (st[q]) L.boff[b] = L.excl[d];
            b += st[q];
            L.bid[d] = b - 1;
        }
        if (tid == RS_T - 1) {
            L.nb = (int)b;
            L.boff[b] = (u32)n;
            const int bk0 = atomicAdd(&A.counts[SCC_CNT_STRIDE * (5)], (int)b);
            L.ovf = bk0 + (int)b > A.bucket_cap;
            L.bk0 = bk0;
        }
    }
    __syncthreads();
    const int nb = L.nb, bk0 = L.bk0;
    RSTAMP(1);
    if (L.ovf) {  // out of bucket ids: rank the parent as one LDS item
        if (tid == 0) {
            const int cls = (n <= A.cap_s) ? 0 : ((n <= A.cap_m) ? 1 : 2);
            A.items[(size_t)cls * A.item_cap + atomicAdd(&A.counts[SCC_CNT_STRIDE * (cls)], 1)] = it;
        }
        return;
    }
    const bool hist_lds = nb * K <= RS_HCAP;
    for (int q = tid; q < nb; q += RS_T) {
        L.bcur[q] = L.boff[q];
        L.bdiff[q] = 0;
    }
    if (hist_lds)
        for (int e = tid; e < nb * K; e += RS_T) L.hs[e] = 0;
    __syncthreads();
    // in-place scatter into sub-bucket order (every element is in registers)
#pragma unroll
    for (int q = 0; q < RS_KPT; ++q) {
        if (q * RS_T + tid < n) {
            const u32 d = (u32)((kr[q] - kmn) >> sh);
            const u32 bk = L.bid[d];
            const u32 pos = atomicAdd(&L.bcur[bk], 1u);
            A.keys2[it.base + pos] = kr[q];
            A.codes2[it.base + pos] = cd[q];
            if (kr[q] != L.rep[d]) L.bdiff[bk] = 1;
            if (hist_lds) atomicAdd(&L.hs[bk * K + cd[q]], 1u);
        }
    }
    __syncthreads();
    RSTAMP(2);
    if (tid < K) A.hbg[(size_t)it.bucket * K + tid] = L.m[tid];  // the parent's row (gene-level cross)
    // sub-buckets for the wave kernel: one list reservation per parent
    {
        u32 wv[(RS_BMAX + RS_T - 1) / RS_T];
        u32 cntw = 0;
        for (int q0 = 0, r = 0; q0 < nb; q0 += RS_T, ++r) {
            const int q = q0 + tid;
            const int c = q < nb ? (int)(L.boff[q + 1] - L.boff[q]) : 0;
            const bool tw = c > 0 && (c <= 64 || !L.bdiff[q]);
            wv[r] = tw;
            cntw += tw;
        }
        cntw = u32_wave_sum(cntw);
        if (lane == 0) L.wsum[w] = cntw;
        __syncthreads();
        if (tid == 0) {
            u32 t = 0;
            for (int v = 0; v < W; ++v) t += L.wsum[v];
            L.nw = (int)t;
            L.w0 = t ? atomicAdd(&A.counts[SCC_CNT_STRIDE * (4)], (int)t) : 0;
        }
        __syncthreads();
        u32 o = (u32)L.w0;
        for (int q0 = 0, r = 0; q0 < nb; q0 += RS_T, ++r) {  // ordered slots: wave prefix per round
            const int q = q0 + tid;
            const u64 bal = __ballot(wv[r] != 0);
            if (lane == 0) L.wsum2[w] = (u32)__popcll(bal);
            __syncthreads();
            u32 ow = o;
            for (int v = 0; v < w; ++v) ow += L.wsum2[v];
            if (q < nb) {
                const int c = (int)(L.boff[q + 1] - L.boff[q]);
                const int bid = bk0 + q;
                if (c <= 0) {
                    for (int k2 = 0; k2 < K; ++k2) A.hbg[(size_t)bid * K + k2] = 0;
                } else {
                    const bool ties_only = c > 64 && !L.bdiff[q];
                    const ScRankItem itm{it.base + L.boff[q], c, g, ties_only ? 2 : 1, bid};
                    if (wv[r]) {
                        A.sbuckets[ow + lanes_below(bal)] = itm;
                    } else if (A.fat2 && c <= RSW_CAP && push_fat2(A, itm)) {
                        // still > 64 distinct values: a second re-split level
                    } else {
                        const int cls = (c <= A.cap_s) ? 0 : ((c <= A.cap_m) ? 1 : 2);
                        A.items[(size_t)cls * A.item_cap + atomicAdd(&A.counts[SCC_CNT_STRIDE * (cls)], 1)] = itm;
                    }
                }
            }
            for (int v = 0; v < W; ++v) o += L.wsum2[v];
            __syncthreads();
        }
    }
    RSTAMP(3);
    if (!hist_lds) {  // many sub-buckets: k_rank_cross_seg adds the in-parent cross term
        if (tid == 0) A.rsseg[atomicAdd(&A.counts[SCC_CNT_STRIDE * (10)], 1)] = int4{g, bk0, nb, 0};
        return;
    }
    // in-parent cross term: S_ab += sum_s hs[s][a] * bs[s][b], bs = #(b in
    // sub-buckets < s) (a column scan per cluster first: the pair sums are
    // then independent loads, not a dependent chain)
    for (int c = tid; c < K; c += RS_T) {
        u32 run = 0;
        for (int q = 0; q < nb; ++q) {
            L.bs[q * K + c] = run;
            run += L.hs[q * K + c];
        }
    }
    __syncthreads();
    const int ntp = A.gene_nt[g];
    const bool lds_acc = ntp <= A.P;  // always: the dynamic LDS array holds P entries
    for (int j = tid; j < ntp; j += RS_T) {
        const u32 v = A.gene_tp[(size_t)g * A.P + j];
        const int a = (int)((v >> 16) & 0xffu), b = (int)(v >> 24);
        if (!L.m[a] || !L.m[b]) continue;
        u64 sacc = 0;
#pragma unroll 4
        for (int q = 0; q < nb; ++q) sacc += (u64)L.hs[q * K + a] * L.bs[q * K + b];
        if (lds_acc)
            acc[j] += sacc;  // thread j owns tested pair j for the whole gene
        else if (sacc)
            atomicAdd((unsigned long long*)&A.accS[(size_t)(v & 0xffffu) * A.G + g], (unsigned long long)sacc);
    }
    RSTAMP(4);
    if (A.stamps && tid == 0) atomicAdd((unsigned long long*)&A.stamps[7], 1ull);
#undef RSTAMP
}

__global__ void __launch_bounds__(RS_T) k_rank_resplit(ScRankLaunch A)
{
    __shared__ ResplitLds L;
    // the gene's in-parent cross terms per tested pair: P entries of dynamic LDS
    // (8 B x 66 at config B, x 4950 at E), so no gene falls back to one global
    // atomic per (parent, pair)
    extern __shared__ __attribute__((aligned(16))) u64 racc[];
    const int ng = A.counts[SCC_CNT_STRIDE * (11)];
    // work items from a queue: slice sl of gene i takes the gene's parents
    // ge.y + sl, ge.y + sl + RS_SLICES, ... (a contiguous run of fatbk), so the
    // large parents of one heavy gene spread over RS_SLICES workgroups (one
    // workgroup per gene left the kernel waiting on its heaviest gene: ~1.5 ms
    // for 1/8 of config D's genes as for all of them).  Every slice adds its
    // in-parent cross terms with integer atomics: order-free.
    for (;;) {
        if (threadIdx.x == 0) L.next = atomicAdd(&A.counts[SCC_CNT_STRIDE * (9)], 1);
        __syncthreads();
        const int wi = L.next;
        if (wi >= ng * RS_SLICES) break;
        const int i = wi / RS_SLICES, sl = wi - i * RS_SLICES;
        const int4 ge = A.fatg[i];
        const int g = ge.x;
        const int ntp = A.gene_nt[g];
        for (int j = threadIdx.x; j < ntp; j += RS_T) racc[j] = 0;
        __syncthreads();
        for (int f = ge.y + sl; f < ge.y + ge.z; f += RS_SLICES) {
            const ScRankItem it = A.fatbk[f];
            if (it.n <= RSW_CAP) continue;  // k_rank_resplit_w (one wave per parent)
            resplit_one(A, it, L, racc);
            __syncthreads();
        }
        for (int j = threadIdx.x; j < ntp; j += RS_T) {
            if (racc[j]) {
                const u32 v = A.gene_tp[(size_t)g * A.P + j];
                atomicAdd((unsigned long long*)&A.accS[(size_t)(v & 0xffffu) * A.G + g], (unsigned long long)racc[j]);
            }
        }
        __syncthreads();
    }
}

// One wave per re-split parent of <= RSW_CAP elements (most of them): the
// same binning, packing, in-place scatter and in-parent cross term as
// resplit_one, with wave-level ordering only (no workgroup barriers) and four
// parents per workgroup in flight.
struct ResplitWLds {  // (offsets and running counts <= RSW_CAP: 16 bits; 12.3 KB a wave, three workgroups per CU)
    u32 hist[RSW_BINS];
    u32 excl[RSW_BINS];
    u32 bid[RSW_BINS];
    u64 rep[RSW_BINS];
    u32 bcur[2 * RSW_BINS + 1];
    uint16_t boff[2 * RSW_BINS + 2];
    u8 bdiff[2 * RSW_BINS + 4];
    u32 m[SCC_MAX_K];
    u32 hs[RSW_HCAP];
    uint16_t bs[RSW_HCAP];
};
static_assert(4 * sizeof(ResplitWLds) <= 160 * 1024 / 3, "wave re-split: three workgroups per CU");

__device__ inline void wsync()
{
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// TS: tested-pair slots held in registers (64 pairs each).  Two launches
// split the genes: TS = RSW_TS_SMALL takes those with <= 64 * RSW_TS_SMALL
// tested pairs (config D FAST: all of them; 3 waves per SIMD instead of 2),
// RSW_PACC / 64 the others (SLOW at K = 50: 1225 pairs).
template <int TS>
__global__ void __launch_bounds__(256) k_rank_resplit_w(ScRankLaunch A)
{
    __shared__ ResplitWLds Ls[4];
    const int lane = threadIdx.x & 63, wv = scc_wave_id();
    ResplitWLds& L = Ls[wv];
    const int K = A.K;
    const ScRankItem* list = A.rs_level ? A.fat2 : A.fatbk;
    const int cnt = A.rs_level ? min(A.counts[SCC_CNT_STRIDE * (12)], A.fat2_cap) : min(A.counts[SCC_CNT_STRIDE * (8)], A.fat_cap);
    constexpr int EPL = RSW_CAP / 64, BPL = RSW_BINS / 64;
    // Bucket ids and wave-list slots come from wave-private chunks: one global
    // atomic per chunk, not per parent (same-address atomics serialise in L2:
    // two per parent cost 48 of this kernel's 54 ms at config D).  Unused
    // list slots are filled with empty descriptors the wave kernel skips.
    const ScRankItem nullit{0, 0, 0, 1, -1};
    const int chunk = A.rsw_chunk;
    int id_cur = 0, id_end = 0, sl_cur = 0, sl_end = 0;
    auto fill_null = [&](int a, int b) {
        for (int q = a + lane; q < b; q += 64) A.sbuckets[q] = nullit;
    };
    // Each wave takes a contiguous run of the parent list.  The list holds a
    // gene's parents together, so the gene's tested pairs are loaded into
    // registers once per run (lane l: pairs l, l + 64, ...) and the in-parent
    // cross terms of consecutive parents add up there, reaching accS with one
    // atomic per (run of one gene, pair) instead of one per (parent, pair).
    // The consecutive sub-buckets also keep the wave kernel's register
    // accumulation on one gene.
    constexpr int PACC = 64 * TS;  // genes past it: per-(parent, pair) atomics (as past RSW_PACC before)
    constexpr bool SMALL = TS < RSW_PACC / 64;
    const int nw = gridDim.x * 4, w = blockIdx.x * 4 + wv;
    const int f0 = (int)((long long)cnt * w / nw), f1 = (int)((long long)cnt * (w + 1) / nw);
    u32 tpr[TS], par[TS];
#pragma unroll
    for (int s = 0; s < TS; ++s) tpr[s] = par[s] = 0;
    int pg = -1, pnt = 0, pn = 0;
    auto flush_par = [&]() {
        if (pg >= 0 && pn > 0 && pnt <= PACC) {
#pragma unroll
            for (int s = 0; s < TS; ++s) {
                if (s * 64 >= pnt) break;
                if (par[s])
                    atomicAdd((unsigned long long*)&A.accS[(size_t)(tpr[s] & 0xffffu) * A.G + pg], (unsigned long long)par[s]);
                par[s] = 0;
            }
        }
        pn = 0;
    };
    for (int f = f0; f < f1; ++f) {
        const ScRankItem it = list[f];
        const int n = it.n, g = it.gene;
        if (!A.rsw_all) {  // this launch's genes (a gene's parents are together in the list)
            const int nt_g = A.gene_nt[g];
            if (SMALL ? nt_g > PACC : nt_g <= 64 * RSW_TS_SMALL) continue;
        }
        // a parent adds at most 128 * 128 to one pair: flush before u32 could wrap
        if (g != pg || pn >= 65536) {
            flush_par();
            if (g != pg) {
                pg = g;
                pnt = A.gene_nt[g];
                if (pnt > 0 && pnt <= PACC) {
                    const u32* tl = A.gene_tp + (size_t)g * A.P;
#pragma unroll
                    for (int s = 0; s < TS; ++s) tpr[s] = tl[min(s * 64 + lane, pnt - 1)];
                }
            }
        }
        if (n > RSW_CAP) continue;  // k_rank_resplit (a workgroup per parent)
        u64 kr[EPL];
        u32 cd[EPL];
        u64 kmn = ~0ull, kmx = 0;
#pragma unroll
        for (int q = 0; q < EPL; ++q) {
            const int i = q * 64 + lane;
            kr[q] = i < n ? A.keys2[it.base + i] : 0ull;
            cd[q] = i < n ? (u32)A.codes2[it.base + i] : 0u;
            if (i < n) {
                kmn = kr[q] < kmn ? kr[q] : kmn;
                kmx = kr[q] > kmx ? kr[q] : kmx;
            }
        }
        for (int m2 = 32; m2 >= 1; m2 >>= 1) {
            const u64 o1 = shfl_xor_u64(kmn, m2), o2 = shfl_xor_u64(kmx, m2);
            kmn = o1 < kmn ? o1 : kmn;
            kmx = o2 > kmx ? o2 : kmx;
        }
        const u64 range = kmx - kmn;
        const int bits = range ? 64 - __clzll((long long)range) : 0;
        const int sh = bits > RSW_LOG2B ? bits - RSW_LOG2B : 0;
#pragma unroll
        for (int q = 0; q < BPL; ++q) L.hist[q * 64 + lane] = 0;
        for (int c = lane; c < SCC_MAX_K; c += 64) L.m[c] = 0;
        wsync();
#pragma unroll
        for (int q = 0; q < EPL; ++q) {
            if (q * 64 + lane < n) {
                const u32 d = (u32)((kr[q] - kmn) >> sh);
                atomicAdd(&L.hist[d], 1u);
                L.rep[d] = kr[q];
                atomicAdd(&L.m[cd[q]], 1u);
            }
        }
        wsync();
        // exclusive scan of the bins, BPL consecutive bins per lane
        {
            u32 h[BPL], v = 0;
#pragma unroll
            for (int q = 0; q < BPL; ++q) {
                h[q] = L.hist[BPL * lane + q];
                v += h[q];
            }
            u32 incl = v;
            for (int o = 1; o < 64; o <<= 1) {
                const u32 y = __shfl_up(incl, o, 64);
                if (lane >= o) incl += y;
            }
            u32 b = incl - v;
#pragma unroll
            for (int q = 0; q < BPL; ++q) {
                L.excl[BPL * lane + q] = b;
                b += h[q];
            }
        }
        wsync();
        const u32 target = (u32)A.wave_target;
        int nb;
        {
            u32 st[BPL], v = 0;
#pragma unroll
            for (int q = 0; q < BPL; ++q) {
                const int d = BPL * lane + q;
                const bool fat = L.hist[d] > target;
                const bool pfat = d > 0 && L.hist[d - 1] > target;
                st[q] = (d == 0) || fat || pfat || (L.excl[d] / target != L.excl[d - 1] / target);
                v += st[q];
            }
            u32 incl = v;
            for (int o = 1; o < 64; o <<= 1) {
                const u32 y = __shfl_up(incl, o, 64);
                if (lane >= o) incl += y;
            }
            u32 b = incl - v;
#pragma unroll
            for (int q = 0; q < BPL; ++q) {
                const int d = BPL * lane + q;
                if (st[q]) L.boff[b] = L.excl[d];
                b += st[q];
                L.bid[d] = b - 1;
            }
            nb = __shfl((int)incl, 63, 64);
            if (lane == 0) L.boff[nb] = (u32)n;
        }
        bool ovf = false;
        if (nb > id_end - id_cur) {
            const int grab = max(nb, 2 * chunk);
            int b0 = 0;
            if (lane == 0) b0 = atomicAdd(&A.counts[SCC_CNT_STRIDE * (5)], grab);
            b0 = __shfl(b0, 0, 64);
            ovf = b0 + grab > A.bucket_cap;
            id_cur = b0;
            id_end = ovf ? b0 : b0 + grab;
        }
        const int bk0 = id_cur;
        if (!ovf) id_cur += nb;
        if (ovf) {  // out of bucket ids: rank the parent as one LDS item
            if (lane == 0) {
                const int cls = (n <= A.cap_s) ? 0 : ((n <= A.cap_m) ? 1 : 2);
                A.items[(size_t)cls * A.item_cap + atomicAdd(&A.counts[SCC_CNT_STRIDE * (cls)], 1)] = it;
            }
            continue;
        }
        const bool hist_lds = nb * K <= RSW_HCAP;
        wsync();
        for (int q = lane; q < nb; q += 64) {
            L.bcur[q] = L.boff[q];
            L.bdiff[q] = 0;
        }
        if (hist_lds)
            for (int e = lane; e < nb * K; e += 64) L.hs[e] = 0;
        wsync();
#pragma unroll
        for (int q = 0; q < EPL; ++q) {
            if (q * 64 + lane < n) {
                const u32 d = (u32)((kr[q] - kmn) >> sh);
                const u32 bk = L.bid[d];
                const u32 pos = atomicAdd(&L.bcur[bk], 1u);
                A.keys2[it.base + pos] = kr[q];
                A.codes2[it.base + pos] = (u8)cd[q];
                if (kr[q] != L.rep[d]) L.bdiff[bk] = 1;
                if (hist_lds) atomicAdd(&L.hs[bk * K + cd[q]], 1u);
            }
        }
        wsync();
        for (int c = lane; c < K; c += 64) A.hbg[(size_t)it.bucket * K + c] = L.m[c];  // the parent's row (gene-level cross)
        // sub-buckets: one list reservation per parent, slots in sub-bucket order
        {
            u32 cw = 0;
            for (int q = lane; q < nb; q += 64) {
                const int c = (int)(L.boff[q + 1] - L.boff[q]);
                cw += (c > 0 && (c <= 64 || !L.bdiff[q])) ? 1u : 0u;
            }
            cw = u32_wave_sum(cw);
            bool to_items = false;
            if ((int)cw > sl_end - sl_cur) {
                fill_null(sl_cur, sl_end);
                const int grab = max((int)cw, chunk);
                int s0 = 0;
                if (lane == 0) s0 = atomicAdd(&A.counts[SCC_CNT_STRIDE * (4)], grab);
                s0 = __shfl(s0, 0, 64);
                if (s0 + grab > A.bucket_cap) {  // list full: these sub-buckets go to the LDS items
                    fill_null(min(s0, A.bucket_cap), A.bucket_cap);
                    to_items = true;
                    sl_cur = sl_end = 0;
                } else {
                    sl_cur = s0;
                    sl_end = s0 + grab;
                }
            }
            u32 o = (u32)sl_cur;
            if (!to_items) sl_cur += (int)cw;
            for (int q0 = 0; q0 < nb; q0 += 64) {
                const int q = q0 + lane;
                int c = 0;
                bool tw = false;
                if (q < nb) {
                    c = (int)(L.boff[q + 1] - L.boff[q]);
                    tw = c > 0 && (c <= 64 || !L.bdiff[q]);
                }
                if (to_items) tw = false;
                const u64 bal = __ballot(tw);
                if (q < nb) {
                    const int bid = bk0 + q;
                    if (c <= 0) {
                        for (int k2 = 0; k2 < K; ++k2) A.hbg[(size_t)bid * K + k2] = 0;
                    } else {
                        const bool ties_only = c > 64 && !L.bdiff[q];
                        const ScRankItem itm{it.base + L.boff[q], c, g, ties_only ? 2 : 1, bid};
                        if (tw) {
                            A.sbuckets[o + lanes_below(bal)] = itm;
                        } else if (A.rs_level == 0 && A.fat2 && push_fat2(A, itm)) {
                            // still > 64 distinct values: a second re-split level
                        } else {
                            const int cls = (c <= A.cap_s) ? 0 : ((c <= A.cap_m) ? 1 : 2);
                            A.items[(size_t)cls * A.item_cap + atomicAdd(&A.counts[SCC_CNT_STRIDE * (cls)], 1)] = itm;
                        }
                    }
                }
                o += (u32)__popcll(bal);
            }
        }
        if (!hist_lds) {  // many sub-buckets: k_rank_cross_seg adds the in-parent cross term
            if (lane == 0) A.rsseg[atomicAdd(&A.counts[SCC_CNT_STRIDE * (10)], 1)] = int4{g, bk0, nb, 0};
            continue;
        }
        for (int c = lane; c < K; c += 64) {
            u32 run = 0;
            for (int q = 0; q < nb; ++q) {
                L.bs[q * K + c] = run;
                run += L.hs[q * K + c];
            }
        }
        wsync();
        const int ntp = pnt;
        if (ntp <= PACC) {
            // m[a] = 0 or m[b] = 0 makes every product zero: no test needed
            ++pn;
#pragma unroll
            for (int s = 0; s < TS; ++s) {
                if (s * 64 >= ntp) break;
                const u32 v = tpr[s];
                const int a = (int)((v >> 16) & 0xffu), b = (int)(v >> 24);
                u32 sacc = 0;  // <= m[a] * m[b] <= 128 * 128
                for (int q = 0; q < nb; ++q) sacc += L.hs[q * K + a] * L.bs[q * K + b];
                par[s] += (s * 64 + lane < ntp) ? sacc : 0u;
            }
        } else {
            const u32* tl = A.gene_tp + (size_t)g * A.P;
            for (int j = lane; j < ntp; j += 64) {
                const u32 v = tl[j];
                const int a = (int)((v >> 16) & 0xffu), b = (int)(v >> 24);
                if (!L.m[a] || !L.m[b]) continue;
                u64 sacc = 0;
                for (int q = 0; q < nb; ++q) sacc += (u64)L.hs[q * K + a] * L.bs[q * K + b];
                if (sacc) atomicAdd((unsigned long long*)&A.accS[(size_t)(v & 0xffffu) * A.G + g], (unsigned long long)sacc);
            }
        }
        wsync();
    }
    flush_par();
    fill_null(sl_cur, sl_end);
}

// ===================================================================== waves
// One wave per bucket of <= 64 elements: bitonic sort of (key, cluster) across
// the lanes (DPP / permlane swaps, no LDS), one ballot mask per cluster over
// the sorted lanes, then every lane computes its own tested pair's S (and the
// tie terms E, X) from the two masks (pair_counts).  Buckets of one repeated
// key (fat bins of ties) need only their cluster histogram.  Consecutive
// buckets of one gene accumulate in registers (lane j: tested pair j) and are
// flushed with one integer atomic per pair when the gene changes.

// Wave sum through DPP (no LDS round trip): quad butterflies, half-row and
// row mirrors give every lane its 16-lane row total, row_bcast15 / row_bcast31
// carry the totals up; lane 63 ends with the sum.
__device__ inline u32 wave_sum_u32(u32 v)
{
    int x = (int)v;
    x += __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, true);    // quad_perm [1,0,3,2]
    x += __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, true);    // quad_perm [2,3,0,1]
    x += __builtin_amdgcn_update_dpp(0, x, 0x141, 0xF, 0xF, true);   // row_half_mirror
    x += __builtin_amdgcn_update_dpp(0, x, 0x140, 0xF, 0xF, true);   // row_mirror
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);  // row_bcast15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);  // row_bcast31 -> rows 2, 3
    return (u32)__builtin_amdgcn_readlane(x, 63);
}

// The same merge on one combined key (key - gene minimum) << 7 | cluster.
// The lanes that keep the minimum at stride ST of a merge whose direction
// bit is UPBIT (0: ascending everywhere) form a compile-time lane mask KM, so
// a compare-exchange is two lane moves, one 64-bit compare into a lane mask,
// one scalar XNOR with KM and two selects (the min / max / direction selects
// the compiler made of `keep_min ? min : max` took 14 instructions a step,
// the per-lane direction masks spilled to SGPR lanes).  take = lt XNOR KM:
// a keep-min lane takes the partner's key when it is smaller, a keep-max lane
// when it is not smaller (equal keys: either is the same key).
__host__ __device__ constexpr u64 bitonic_km(int ST, int UPBIT)
{
    u64 m = 0;
    for (int l = 0; l < 64; ++l)
        if (((l & ST) == 0) == (UPBIT == 0 || (l & UPBIT) == 0)) m |= 1ull << l;
    return m;
}

// per-lane select by a lane mask held in scalar registers (bit set: b)
__device__ inline u32 lane_select(u64 mask, u32 a, u32 b)
{
    u32 r;
    asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(mask));
    return r;
}

template <int ST, int UPBIT>
__device__ inline void bitonic_merge_ck(u64& ck)
{
    const u32 olo = scc_xor_lane<ST>((u32)ck), ohi = scc_xor_lane<ST>((u32)(ck >> 32));
    const u64 o = ((u64)ohi << 32) | olo;
    constexpr u64 KM = bitonic_km(ST, UPBIT);
    const u64 lt = __ballot(o < ck);
    const u64 take = ~(lt ^ KM);
    ck = ((u64)lane_select(take, (u32)(ck >> 32), ohi) << 32) | lane_select(take, (u32)ck, olo);
    if constexpr (ST > 1) bitonic_merge_ck<ST / 2, UPBIT>(ck);
}

__device__ inline u64 shfl_u64(u64 v, int src)
{
    const u32 lo = (u32)__shfl((int)(u32)v, src, 64), hi = (u32)__shfl((int)(u32)(v >> 32), src, 64);
    return ((u64)hi << 32) | lo;
}

// One pair's counts over a sorted bucket from its cluster masks, walking the
// set bits of the smaller one: S_ab = sum_{i in a} #b below i = sum_{j in b}
// #a above j; with ties (gst: lanes starting a group of equal keys, n: valid
// lanes) E_ab = sum over groups c_a c_b and X_ab = sum c_a c_b (c_a + c_b).
__device__ inline void pair_counts(u64 ma, u64 mb, bool ties, u64 gst, int n, u32& S, u32& E, u32& X)
{
    const bool walk_a = __popcll(ma) <= __popcll(mb);
    u64 m = walk_a ? ma : mb;
    const u64 self = m, other = walk_a ? mb : ma;
    S = E = X = 0;
    while (m) {
        const int i = __builtin_ctzll(m);
        m &= m - 1;
        const u64 le = (2ull << i) - 1;  // lanes <= i (all of them for i = 63)
        S += (u32)__popcll(other & (walk_a ? (le >> 1) : ~le));
        if (ties) {
            const int gsl = 63 - __clzll((long long)(gst & le));
            const u64 aft = gst & ~le;
            const int ge = aft ? __builtin_ctzll(aft) : n;
            const u64 grp = ((ge >= 64) ? ~0ull : ((1ull << ge) - 1)) & ~((1ull << gsl) - 1);
            const u32 co = (u32)__popcll(other & grp), cs = (u32)__popcll(self & grp);
            E += co;
            X += co * (co + cs);
        }
    }
}

// One bitonic merge level of (key, code) across the lanes, strides ST .. 1.
template <int ST>
__device__ inline void bitonic_merge(u64& key, u32& code, bool up, int lane)
{
    const u64 ok = ((u64)scc_xor_lane<ST>((u32)(key >> 32)) << 32) | (u64)scc_xor_lane<ST>((u32)key);
    const u32 oc = scc_xor_lane<ST>(code);
    const bool lower = (lane & ST) == 0;
    const bool other_less = (ok < key) || (ok == key && oc < code);
    if ((lower == up) ? other_less : !other_less) {
        key = ok;
        code = oc;
    }
    if constexpr (ST > 1) bitonic_merge<ST / 2>(key, code, up, lane);
}

template <int RW_SLOTS>
__global__ void __launch_bounds__(256) k_rank_waves(ScRankLaunch A)
{
    __shared__ u64 cms[4][SCC_MAX_K];  // per-wave cluster masks (K > 16)
    const int lane = threadIdx.x & 63, wv = scc_wave_id();
    const int W = blockIdx.x * 4 + wv, NW = gridDim.x * 4;
    const int cnt = min(A.counts[SCC_CNT_STRIDE * (4)], A.bucket_cap);
    const int K = A.K, G = A.G, P = A.P;
    constexpr int CH = 16;  // consecutive buckets per wave visit (gene locality; 8 / 32 / 64 measured no better)
    int cur = -1, ntp = 0;
    u64 xbud = 0;  // a bound on the largest slot sum of the current run
    u64 gk = ~0ull;
    // per slot: the tested pair as the split packed it (p | a << 16 | b << 24)
    // and its sums over the buckets of the current run of one gene, in 32 bits
    // (a wave bucket adds S <= 32 * 32, E <= 32 * 32, X <= 32 * 32 * 64 to one
    // pair, a ties-only bucket of n values E <= n^2 / 4, X <= n^3 / 4: a run is
    // cut before the bound passes 2^32; a ties-only bucket past 2048 values
    // goes straight out in 64 bits):
    // half the registers of u64 sums and three pair words, so the 16-slot
    // variant fits two waves per SIMD
    u32 tp[RW_SLOTS];
    u32 aS[RW_SLOTS], aE[RW_SLOTS], aX[RW_SLOTS];
#pragma unroll
    for (int q = 0; q < RW_SLOTS; ++q) {
        tp[q] = 0;
        aS[q] = aE[q] = aX[q] = 0;
    }
    for (int c0 = W * CH; c0 < cnt; c0 += NW * CH) {
        const int c1 = min(cnt, c0 + CH);
        // the chunk's descriptors, one per lane, and the first bucket's elements:
        // every bucket's loads are issued one bucket ahead
        ScRankItem D{0, 0, 0, 0, 0};
        if (lane < c1 - c0) D = A.sbuckets[c0 + lane];
        // this launch ranks the buckets of genes with wv_lo < tested pairs <= wv_hi
        // (the slot count of each launch fits its genes: fewer registers, more waves)
        // (one class launched: no filter, and no dependent load before the first bucket)
        u64 rem;
        if (A.wv_filter) {
            const int ntg = (lane < c1 - c0 && D.n > 0) ? A.gene_nt[D.gene] : -1;  // n = 0: an unused re-split slot
            rem = __ballot(ntg > A.wv_lo && ntg <= A.wv_hi);
        } else {
            rem = __ballot(lane < c1 - c0 && D.n > 0);
        }
        if (!rem) continue;
        const u32 dlo = (u32)(u64)D.base, dhi = (u32)((u64)D.base >> 32);
        auto dbase = [&](int li) {
            return (i64)(((u64)(u32)__builtin_amdgcn_readlane((int)dhi, li) << 32) |
                         (u32)__builtin_amdgcn_readlane((int)dlo, li));
        };
        u64 nkey;
        u32 ncode;
        {
            const int l0 = __builtin_ctzll(rem);
            const i64 b0 = dbase(l0);
            const int n0 = __builtin_amdgcn_readlane(D.n, l0);
            nkey = lane < n0 ? A.keys2[b0 + lane] : ~0ull;
            ncode = lane < n0 ? (u32)A.codes2[b0 + lane] : 255u;
        }
        while (rem) {
            const int li = __builtin_ctzll(rem);
            rem &= rem - 1;
            const int g = __builtin_amdgcn_readlane(D.gene, li);
            const int n = __builtin_amdgcn_readlane(D.n, li);
            const int bucket = __builtin_amdgcn_readlane(D.bucket, li);
            const int src = __builtin_amdgcn_readlane(D.src, li);
            const i64 bbase = dbase(li);
            u64 key = nkey;
            u32 code = ncode;
            if (rem) {
                const int l1 = __builtin_ctzll(rem);
                const i64 b1 = dbase(l1);
                const int n1 = __builtin_amdgcn_readlane(D.n, l1);
                nkey = lane < n1 ? A.keys2[b1 + lane] : ~0ull;
                ncode = lane < n1 ? (u32)A.codes2[b1 + lane] : 255u;
            }
            const bool big_ties = src == 2 && n > 2048;
            const u64 xadd = src == 2 ? (big_ties ? 0ull : (u64)n * n * n / 4 + 1) : 65536ull;
            if (g != cur || xbud + xadd > 0xffffffffull) {
                // flush the previous run's sums: one integer atomic per pair
                if (cur >= 0) {
#pragma unroll
                    for (int q = 0; q < RW_SLOTS; ++q) {
                        if (q * 64 + lane < ntp) {
                            const size_t o = (size_t)(tp[q] & 0xffffu) * G + cur;
                            if (aS[q]) atomicAdd((unsigned long long*)&A.accS[o], (unsigned long long)aS[q]);
                            if (aE[q]) atomicAdd((unsigned long long*)&A.accE[o], (unsigned long long)aE[q]);
                            if (aX[q]) atomicAdd((unsigned long long*)&A.accX[o], (unsigned long long)aX[q]);
                        }
                        aS[q] = aE[q] = aX[q] = 0;
                    }
                }
                xbud = 0;
            }
            xbud += xadd;
            if (g != cur) {
                cur = g;
                gk = A.gkmin[g];
                // tested pairs of g in pair order (compacted by the split)
                // this launch's window of the gene's tested pairs (wv_base > 0: the
                // second pass over a gene with more than 64 * RW_SLOTS of them)
                ntp = max(0, min(A.gene_nt[g] - A.wv_base, 64 * RW_SLOTS));
                const u32* tl = A.gene_tp + (size_t)g * P + A.wv_base;
#pragma unroll
                for (int q = 0; q < RW_SLOTS; ++q) {
                    const int j = q * 64 + lane;
                    const u32 v = tl[j < ntp ? j : 0];
                    if (j < ntp) tp[q] = v;
                }
            }
            if (src == 2) {
                // one repeated key: only the cluster histogram matters.  Inside
                // the bucket S_ab = 0 (a < b: ties ordered by cluster),
                // E_ab = c_a c_b, X_ab = c_a c_b (c_a + c_b), F_a = f(c_a).
                u32 myc = 0, myc1 = 0;  // lane c: cluster c's count, and cluster c + 64's
                for (int i0 = 0; i0 < n; i0 += 256) {
                    u32 cd[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int i = i0 + u * 64 + lane;
                        cd[u] = i < n ? (u32)A.codes2[bbase + i] : 255u;
                    }
                    for (int c = 0; c < K; ++c) {
                        u32 t = 0;
#pragma unroll
                        for (int u = 0; u < 4; ++u) t += (u32)__popcll(__ballot(cd[u] == (u32)c));
                        if (lane == c) myc += t;
                        if (lane + 64 == c) myc1 += t;
                    }
                }
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int c = lane + 64 * h;
                    const u32 mc = h ? myc1 : myc;
                    if (c < K) {
                        A.hbg[(size_t)bucket * K + c] = mc;
                        if (mc >= 2 && A.wv_base == 0)  // per cluster: once, not per pair window
                            atomicAdd((unsigned long long*)&A.accF[(size_t)c * G + g], (unsigned long long)f_tie(mc));
                    }
                }
                // (past 2048 values its counts can pass 32 bits: straight out in 64)
#pragma unroll
                for (int q = 0; q < RW_SLOTS; ++q) {
                    const u32 pa = (tp[q] >> 16) & 0xffu, pb = tp[q] >> 24;
                    u64 ca = (u32)__shfl((int)myc, (int)(pa & 63u), 64);
                    u64 cb = (u32)__shfl((int)myc, (int)(pb & 63u), 64);
                    if (K > 64) {
                        const u64 ca1 = (u32)__shfl((int)myc1, (int)(pa & 63u), 64);
                        const u64 cb1 = (u32)__shfl((int)myc1, (int)(pb & 63u), 64);
                        ca = pa >= 64 ? ca1 : ca;
                        cb = pb >= 64 ? cb1 : cb;
                    }
                    if (q * 64 + lane < ntp && ca && cb) {
                        if (big_ties) {
                            const size_t o = (size_t)(tp[q] & 0xffffu) * G + g;
                            atomicAdd((unsigned long long*)&A.accE[o], (unsigned long long)(ca * cb));
                            atomicAdd((unsigned long long*)&A.accX[o], (unsigned long long)(ca * cb * (ca + cb)));
                        } else {
                            aE[q] += (u32)(ca * cb);
                            aX[q] += (u32)(ca * cb * (ca + cb));
                        }
                    }
                }
                continue;
            }
            // ---- load and bitonic sort by (key, code) across the lanes (invalid lanes last)
            const bool vl = lane < n;
            if (A.dbg == 2) {
            } else if (gk != ~0ull) {  // one 64-bit sort key: (key - gene minimum) << 7 | cluster
                u64 ck = vl ? (((key - gk) << SCC_CODE_BITS) | code) : ~0ull;
                // levels up to the next power of two >= n (lanes past it hold only ~0)
                if (n > 1) bitonic_merge_ck<1, 2>(ck);
                if (n > 2) bitonic_merge_ck<2, 4>(ck);
                if (n > 4) bitonic_merge_ck<4, 8>(ck);
                if (n > 8) bitonic_merge_ck<8, 16>(ck);
                if (n > 16) bitonic_merge_ck<16, 32>(ck);
                if (n > 32) bitonic_merge_ck<32, 0>(ck);
                key = ck >> SCC_CODE_BITS;  // order-equivalent for the tie tests below
                code = vl ? (u32)(ck & SCC_CODE_MASK) : 255u;
            } else {
                if (n > 1) bitonic_merge<1>(key, code, (lane & 2) == 0, lane);
                if (n > 2) bitonic_merge<2>(key, code, (lane & 4) == 0, lane);
                if (n > 4) bitonic_merge<4>(key, code, (lane & 8) == 0, lane);
                if (n > 8) bitonic_merge<8>(key, code, (lane & 16) == 0, lane);
                if (n > 16) bitonic_merge<16>(key, code, (lane & 32) == 0, lane);
                if (n > 32) bitonic_merge<32>(key, code, true, lane);
            }
            // ---- cluster masks over the sorted lanes (lane c holds cluster c's, cm1
            // cluster c + 64's) and the hbg row
            u64 cm = 0, cm1 = 0;
            if (K <= 16) {  // one ballot per cluster
                for (int c = 0; c < K; ++c) {
                    const u64 m = __ballot(code == (u32)c);
                    if (lane == c) cm = m;
                }
            } else {  // many clusters: 7 ballots match equal codes, each cluster's leader posts its mask
                const u64 peers = match_bits<SCC_CODE_BITS>(code & SCC_CODE_MASK, __ballot(vl));
                cms[wv][lane] = 0;
                if (K > 64) cms[wv][lane + 64] = 0;
                wsync();
                if (vl && lanes_below(peers) == 0) cms[wv][code] = peers;
                wsync();
                cm = cms[wv][lane];
                if (K > 64) cm1 = cms[wv][lane + 64];
            }
            if (lane < K) A.hbg[(size_t)bucket * K + lane] = (u32)__popcll(cm);
            if (lane + 64 < K) A.hbg[(size_t)bucket * K + lane + 64] = (u32)__popcll(cm1);
            // ---- tie groups (equal keys) and runs (equal key and cluster)
            const u64 kp = ((u64)(u32)__shfl_up((int)(u32)(key >> 32), 1, 64) << 32) |
                           (u64)(u32)__shfl_up((int)(u32)key, 1, 64);
            const u32 cpv = (u32)__shfl_up((int)code, 1, 64);
            const u64 vmask = (n >= 64) ? ~0ull : ((1ull << n) - 1);
            const bool gs_me = (lane == 0) || (kp != key);
            const u64 gst = __ballot(gs_me && vl);
            const bool anytie = ((~gst) & vmask & ~1ull) != 0;
            if (anytie) {
                // within-cluster runs: F_a += len^3 - len per run of >= 2
                const u64 le = (lane == 63) ? ~0ull : ((2ull << lane) - 1);  // lanes <= me
                const bool rs_me = (lane == 0) || (kp != key) || (cpv != code);
                const u64 rst = __ballot(rs_me && vl);
                if (rs_me && vl) {
                    const u64 raft = rst & ~le;
                    const int re = raft ? __builtin_ctzll(raft) : n;
                    const u64 len = (u64)(re - lane);
                    if (len >= 2 && A.wv_base == 0)
                        atomicAdd((unsigned long long*)&A.accF[(size_t)code * G + g], (unsigned long long)f_tie(len));
                }
            }
            // ---- tested pairs: lane l of slot q owns pair q * 64 + l
#pragma unroll
            for (int q = 0; q < RW_SLOTS; ++q) {
                if (q * 64 >= ntp || A.dbg == 1) break;
                u64 ma, mb;
                const u32 pa = (tp[q] >> 16) & 0xffu, pb = tp[q] >> 24;
                if (K > 16) {  // the pair's masks straight from the leaders' LDS posts (two reads, no lane moves;
                               // clusters 64..127 too: 8 lane moves a slot before at K > 64)
                    ma = cms[wv][pa];
                    mb = cms[wv][pb];
                } else {
                    ma = shfl_u64(cm, (int)(pa & 63u));
                    mb = shfl_u64(cm, (int)(pb & 63u));
                }
                if (q * 64 + lane < ntp && ma && mb) {
                    u32 S, E, X;
                    pair_counts(ma, mb, anytie, gst, n, S, E, X);
                    aS[q] += S;
                    aE[q] += E;
                    aX[q] += X;
                }
            }
            if (K > 16) wsync();  // the masks are reposted by the next bucket
        }
    }
    if (cur >= 0) {
#pragma unroll
        for (int q = 0; q < RW_SLOTS; ++q) {
            if (q * 64 + lane < ntp) {
                const size_t o = (size_t)(tp[q] & 0xffffu) * G + cur;
                if (aS[q]) atomicAdd((unsigned long long*)&A.accS[o], (unsigned long long)aS[q]);
                if (aE[q]) atomicAdd((unsigned long long*)&A.accE[o], (unsigned long long)aE[q]);
                if (aX[q]) atomicAdd((unsigned long long*)&A.accX[o], (unsigned long long)aX[q]);
            }
        }
    }
}

// ===================================================================== waves on MFMA
// The bucket walk of k_rank_waves with the pair counting on the int8 matrix
// cores (K <= 64).  After the bitonic sort, with O the bucket's one-hot
// (element x cluster) matrix and L the strict lower triangle of positions,
//   M = L O        M[i][b]: b-elements sorted below element i
//   S += O^T M     S[a][b] = sum over i in a of #b below i (for a < b the
//                  positional count is the strict one: equal keys sort by cluster)
// and, in a bucket with ties, with Eq[i][j] = [j in i's tie group],
// Q = Eq O (Q[i][b] = t_b of i's group) and D_i = t_{c_i} of i's group:
//   E += O^T Q                     sum over groups t_a t_b
//   X += (D O)^T Q + Q^T (D O)     sum over groups t_a^2 t_b + t_a t_b^2
// Every operand is 0/1 or a count <= 64 (int8) and one bucket's products fit
// int32.  A gene's sums stay in the accumulator tiles (the upper 16 x 16 tiles
// of the K x K matrices hold every pair a < b) and leave with one integer
// atomic per tested pair when the gene changes: at K <= 64 (NC = 4 cluster
// tiles) 26 MFMAs 16x16x64 per bucket without ties, 72 with, whatever the
// number of tested pairs (the per-pair walk of k_rank_waves ran 16 slots of 64
// pairs per bucket at config D).  Same bucket list, same hbg rows and F terms,
// same integers.
typedef int rk_v4i __attribute__((ext_vector_type(4)));
// bytes [base + q < x], q = 0..3 (0 / 1 each)
__device__ inline u32 rk_lt_bytes(int x, int base)
{
    int v = x - base;
    v = v < 0 ? 0 : (v > 4 ? 4 : v);
    return (u32)((0x01010101ull << (8 * v)) >> 32);
}

// bytes of w equal to c (0 / 1 each)
__device__ inline u32 rk_eq_bytes(u32 w, u32 c)
{
    const u32 x = w ^ (c * 0x01010101u);
    const u32 nz = ((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x;  // bit 7 of a byte: the byte is not zero
    return (~nz >> 7) & 0x01010101u;
}

__device__ unsigned long long g_rk_stamps[8];  // SCC_RK_STAMPS diagnostics: summed phase cycles
extern "C" void scc_rank_mfma_stamps(hipStream_t st, int print)
{
    unsigned long long h[8];
    if (print) {
        hipStreamSynchronize(st);
        hipMemcpyFromSymbol(h, HIP_SYMBOL(g_rk_stamps), sizeof(h), 0, hipMemcpyDeviceToHost);
        fprintf(stderr, "[scc rk stamps] buckets %llu flush %llu: per bucket sort %.0f operands %.0f products %.0f ties %.0f "
                "flush %.0f fat %.0f\n", h[6], h[7], h[0] / (double)(h[6] + 1), h[1] / (double)(h[6] + 1),
                h[2] / (double)(h[6] + 1), h[3] / (double)(h[6] + 1), h[4] / (double)(h[6] + 1), h[5] / (double)(h[6] + 1));
    }
    const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    hipMemcpyToSymbolAsync(HIP_SYMBOL(g_rk_stamps), z, sizeof(z), 0, hipMemcpyHostToDevice, st);
    hipStreamSynchronize(st);
}

struct RkWaveLds {
    u8 code[64];  // sorted codes at their operand slots
    u8 dcnt[64];  // D_i at their operand slots
    u32 cnt[64];  // a fat bin's cluster counts
    u64 F[64];    // within-cluster tie terms of the current gene, per cluster
};

// The products on 16 x 16 x 64 tiles (K <= 16 * NC): one MFMA covers a
// bucket's 64 elements, a cluster tile is 4 accumulator registers, so the
// kernel keeps two waves per SIMD even at K = 64 (a 32 x 32 x 32 form of the
// same products held 1 wave at 422 registers: D SLOW rank 60.8 ms against
// 42.3 ms for this one, round 6).  Slots: lane l holds
// row / column l & 15 and, in byte t of its 16-byte fragment (lane group
// g = l >> 4), element e(g, t) = 16 (t >> 2) + 4 g + (t & 3): the row the
// accumulator layout puts in register t & 3 of lane group g of row tile
// t >> 2, so four packed accumulator tiles are the next product's operand.
__device__ inline rk_v4i rk_mfma16(rk_v4i a, rk_v4i b, rk_v4i c)
{
    return __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
}

template <int NC>
__device__ constexpr int rk_tile16(int ma, int nb)  // upper tiles (ma <= nb) in row order
{
    return ma * NC - ma * (ma - 1) / 2 + (nb - ma);
}

template <int NC>
__global__ void __launch_bounds__(256, NC >= 3 ? 2 : 1) k_rank_mfma16(ScRankLaunch A)  // NC >= 3: 2 waves / SIMD (NC = 4: 23 VGPRs spill)
{
    constexpr int NTL = NC * (NC + 1) / 2;
    constexpr int TL = NC == 1 ? 2 : NC == 2 ? 8 : 32;  // tested-pair list entries per lane (P <= 120 / 496 / 2016)
    __shared__ __attribute__((aligned(16))) RkWaveLds Ls[4];
    __shared__ u32 Lbuf[4][NTL * 256];   // one accumulator matrix of a flush, [tile][a & 15][b & 15]
    const int lane = threadIdx.x & 63, wv = scc_wave_id();
    RkWaveLds& Lw = Ls[wv];
    u32* buf = Lbuf[wv];
    const int NW = gridDim.x * 4, W = blockIdx.x * 4 + wv;
    const int cnt = min(A.counts[SCC_CNT_STRIDE * (4)], A.bucket_cap);
    const int K = A.K, G = A.G, P = A.P;
    const int CH = max(16, min(512, cnt / (4 * NW)));
    const int g4 = lane >> 4, r16 = lane & 15;
    const rk_v4i zero = {0, 0, 0, 0};
    // L rows 16 mt + r16: bytes [e(g4, t) < i] (formed where used: held for the
    // whole kernel they were 16 registers of the 2-waves-per-SIMD budget at NC = 4)
    auto Lrow = [&](int mt) {
        rk_v4i l;
#pragma unroll
        for (int d = 0; d < 4; ++d) l[d] = (int)rk_lt_bytes(16 * mt + r16, 16 * d + 4 * g4);
        return l;
    };
    rk_v4i R[NTL], X[NTL];
#pragma unroll
    for (int t = 0; t < NTL; ++t) R[t] = X[t] = zero;
    Lw.F[lane] = 0;
    int cur = -1, ntp = 0, nrun = 0;
    bool rtie = false;
    u64 gk = ~0ull;
    const bool stm = A.dbg == 7;  // SCC_RW_DEBUG=7: phase clocks into g_rk_stamps
    u64 tph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tprev = stm ? __builtin_amdgcn_s_memtime() : 0;
    auto stamp = [&](int ph) {
        if (stm) {
            const u64 t = __builtin_amdgcn_s_memtime();
            tph[ph] += t - tprev;
            tprev = t;
        }
    };
    auto flush = [&]() {
        ++tph[7];
        const u32* tl = A.gene_tp + (size_t)cur * P;
        // the tested-pair list in register chunks of <= 8 entries a lane (a
        // whole 2016-pair list in registers would cost the kernel its occupancy)
        constexpr int TLC = TL < 8 ? TL : 8;
        auto out = [&](rk_v4i* Mx, unsigned long long* acc) {
#pragma unroll
            for (int ma = 0; ma < NC; ++ma)
#pragma unroll
                for (int nb = ma; nb < NC; ++nb) {
                    const int t = rk_tile16<NC>(ma, nb);
#pragma unroll
                    for (int r = 0; r < 4; ++r) buf[t * 256 + (4 * g4 + r) * 16 + r16] = (u32)Mx[t][r];
                    Mx[t] = zero;
                }
            wsync();
            for (int q0 = 0; q0 < TL; q0 += TLC) {
                if (q0 * 64 >= ntp) break;
                u32 tv[TLC];
#pragma unroll
                for (int q = 0; q < TLC; ++q) tv[q] = tl[min((q0 + q) * 64 + lane, max(ntp - 1, 0))];
#pragma unroll
                for (int q = 0; q < TLC; ++q) {
                    if ((q0 + q) * 64 >= ntp) break;
                    const u32 v = tv[q];
                    const int a = (int)((v >> 16) & 0xffu), b = (int)(v >> 24);
                    const u32 x = buf[rk_tile16<NC>(a >> 4, b >> 4) * 256 + (a & 15) * 16 + (b & 15)];
                    if ((q0 + q) * 64 + lane < ntp && x)
                        atomicAdd(&acc[(size_t)(v & 0xffffu) * G + cur], (unsigned long long)x);
                }
            }
            wsync();
        };
        out(R, (unsigned long long*)A.accE);
        if (rtie) {
            out(X, (unsigned long long*)A.accX);
            const u64 f = Lw.F[lane];
            if (lane < K && f) atomicAdd((unsigned long long*)&A.accF[(size_t)lane * G + cur], (unsigned long long)f);
            Lw.F[lane] = 0;
            wsync();
        }
        nrun = 0;
        rtie = false;
    };
    for (int c0 = W * CH; c0 < cnt; c0 += NW * CH) {
        const int c1 = min(cnt, c0 + CH);
        for (int s0 = c0; s0 < c1; s0 += 64) {
            const int s1 = min(c1, s0 + 64);
            ScRankItem D{0, 0, 0, 0, 0};
            if (lane < s1 - s0) D = A.sbuckets[s0 + lane];
            u64 rem;
            if (A.wv_filter) {
                const int ntg = (lane < s1 - s0 && D.n > 0) ? A.gene_nt[D.gene] : -1;
                rem = __ballot(ntg > A.wv_lo && ntg <= A.wv_hi);
            } else {
                rem = __ballot(lane < s1 - s0 && D.n > 0);
            }
            if (!rem) continue;
            const u32 dlo = (u32)(u64)D.base, dhi = (u32)((u64)D.base >> 32);
            auto dbase = [&](int li) {
                return (i64)(((u64)(u32)__builtin_amdgcn_readlane((int)dhi, li) << 32) |
                             (u32)__builtin_amdgcn_readlane((int)dlo, li));
            };
            u64 nkey;
            u32 ncode;
            {
                const int l0 = __builtin_ctzll(rem);
                const i64 b0 = dbase(l0);
                const int n0 = __builtin_amdgcn_readlane(D.n, l0);
                nkey = lane < n0 ? A.keys2[b0 + lane] : ~0ull;
                ncode = lane < n0 ? (u32)A.codes2[b0 + lane] : 255u;
            }
            while (rem) {
                const int li = __builtin_ctzll(rem);
                rem &= rem - 1;
                const int g = __builtin_amdgcn_readlane(D.gene, li);
                const int n = __builtin_amdgcn_readlane(D.n, li);
                const int bucket = __builtin_amdgcn_readlane(D.bucket, li);
                const int src = __builtin_amdgcn_readlane(D.src, li);
                const i64 bbase = dbase(li);
                u64 key = nkey;
                u32 code = ncode;
                if (rem) {
                    const int l1 = __builtin_ctzll(rem);
                    const i64 b1 = dbase(l1);
                    const int n1 = __builtin_amdgcn_readlane(D.n, l1);
                    nkey = lane < n1 ? A.keys2[b1 + lane] : ~0ull;
                    ncode = lane < n1 ? (u32)A.codes2[b1 + lane] : 255u;
                }
                if (g != cur || nrun >= 16384) {
                    if (cur >= 0) flush();
                    if (g != cur) {
                        cur = g;
                        gk = A.gkmin[g];
                        ntp = A.gene_nt[g];
                    }
                }
                ++nrun;
                ++tph[6];
                stamp(4);
                if (src == 2) {  // one repeated key: only the cluster histogram matters (as in k_rank_waves)
                    u32 myc = 0;
                    for (int i00 = 0; i00 < n; i00 += 256) {
                        u32 cd[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const int i = i00 + u * 64 + lane;
                            cd[u] = i < n ? (u32)A.codes2[bbase + i] : 255u;
                        }
                        for (int c = 0; c < K; ++c) {
                            u32 t = 0;
#pragma unroll
                            for (int u = 0; u < 4; ++u) t += (u32)__popcll(__ballot(cd[u] == (u32)c));
                            if (lane == c) myc += t;
                        }
                    }
                    if (lane < K) {
                        A.hbg[(size_t)bucket * K + lane] = myc;
                        if (myc >= 2) Lw.F[lane] += f_tie(myc);
                    }
                    rtie = true;
                    Lw.cnt[lane] = myc;
                    wsync();
                    const u32* tl = A.gene_tp + (size_t)g * P;
                    for (int j = lane; j < ntp; j += 64) {
                        const u32 v = tl[j];
                        const u64 ca = Lw.cnt[(v >> 16) & 0xffu], cb = Lw.cnt[v >> 24];
                        if (ca && cb) {
                            const size_t o = (size_t)(v & 0xffffu) * G + g;
                            atomicAdd((unsigned long long*)&A.accE[o], (unsigned long long)(ca * cb));
                            atomicAdd((unsigned long long*)&A.accX[o], (unsigned long long)(ca * cb * (ca + cb)));
                        }
                    }
                    wsync();
                    stamp(5);
                    continue;
                }
                const bool vl = lane < n;
                if (gk != ~0ull) {
                    u64 ck = vl ? (((key - gk) << SCC_CODE_BITS) | code) : ~0ull;
                    if (n > 1) bitonic_merge_ck<1, 2>(ck);
                    if (n > 2) bitonic_merge_ck<2, 4>(ck);
                    if (n > 4) bitonic_merge_ck<4, 8>(ck);
                    if (n > 8) bitonic_merge_ck<8, 16>(ck);
                    if (n > 16) bitonic_merge_ck<16, 32>(ck);
                    if (n > 32) bitonic_merge_ck<32, 0>(ck);
                    key = ck >> SCC_CODE_BITS;
                    code = vl ? (u32)(ck & SCC_CODE_MASK) : 255u;
                } else {
                    if (n > 1) bitonic_merge<1>(key, code, (lane & 2) == 0, lane);
                    if (n > 2) bitonic_merge<2>(key, code, (lane & 4) == 0, lane);
                    if (n > 4) bitonic_merge<4>(key, code, (lane & 8) == 0, lane);
                    if (n > 8) bitonic_merge<8>(key, code, (lane & 16) == 0, lane);
                    if (n > 16) bitonic_merge<16>(key, code, (lane & 32) == 0, lane);
                    if (n > 32) bitonic_merge<32>(key, code, true, lane);
                }
                stamp(0);
                // ---- one-hot operand: sorted codes at their slots, element i at
                // byte 16 ((i >> 2) & 3) + 4 (i >> 4) + (i & 3)
                const int sg = (((lane >> 2) & 3) << 4) | ((lane >> 4) << 2) | (lane & 3);
                Lw.code[sg] = (u8)code;
                wsync();
                const rk_v4i cw = *(const rk_v4i*)(Lw.code + 16 * g4);
                rk_v4i ob[NC];
#pragma unroll
                for (int t = 0; t < NC; ++t)
#pragma unroll
                    for (int d = 0; d < 4; ++d) ob[t][d] = (int)rk_eq_bytes((u32)cw[d], (u32)(r16 + 16 * t));
#pragma unroll
                for (int t = 0; t < NC; ++t) {  // the bucket's cluster histogram row
                    u32 sm = (u32)ob[t][0] + (u32)ob[t][1] + (u32)ob[t][2] + (u32)ob[t][3];
                    u32 c = (sm * 0x01010101u) >> 24;
                    c += (u32)__shfl_xor((int)c, 16, 64);
                    c += (u32)__shfl_xor((int)c, 32, 64);
                    if (g4 == 0 && r16 + 16 * t < K) A.hbg[(size_t)bucket * K + r16 + 16 * t] = c;
                }
                stamp(1);
                // ---- M = L O (row tiles of 16 elements), R += O^T (2 M)
                const int nmt = (n + 15) >> 4;
                rk_v4i mb[NC];
#pragma unroll
                for (int t = 0; t < NC; ++t) mb[t] = zero;
#pragma unroll
                for (int mt = 0; mt < 4; ++mt) {
                    if (mt >= nmt) break;
                    const rk_v4i Lmt = Lrow(mt);
#pragma unroll
                    for (int t = 0; t < NC; ++t) {
                        const rk_v4i m = rk_mfma16(Lmt, ob[t], zero);
                        mb[t][mt] = (int)((u32)(2 * m[0]) | ((u32)(2 * m[1]) << 8) | ((u32)(2 * m[2]) << 16) |
                                          ((u32)(2 * m[3]) << 24));
                    }
                }
#pragma unroll
                for (int ma = 0; ma < NC; ++ma)
#pragma unroll
                    for (int nb = ma; nb < NC; ++nb) {
                        const int t = rk_tile16<NC>(ma, nb);
                        R[t] = rk_mfma16(ob[ma], mb[nb], R[t]);
                    }
                stamp(2);
                // ---- tie groups and runs
                const u64 kp = ((u64)(u32)__shfl_up((int)(u32)(key >> 32), 1, 64) << 32) |
                               (u64)(u32)__shfl_up((int)(u32)key, 1, 64);
                const u32 cpv = (u32)__shfl_up((int)code, 1, 64);
                const u64 vmask = (n >= 64) ? ~0ull : ((1ull << n) - 1);
                const bool gs_me = (lane == 0) || (kp != key);
                const u64 gst = __ballot(gs_me && vl);
                const bool anytie = ((~gst) & vmask & ~1ull) != 0;
                if (anytie) {
                    rtie = true;
                    const u64 le = (lane == 63) ? ~0ull : ((2ull << lane) - 1);
                    const bool rs_me = (lane == 0) || (kp != key) || (cpv != code);
                    const u64 rst = __ballot(rs_me && vl);
                    const u64 raft = rst & ~le;
                    const int re = raft ? __builtin_ctzll(raft) : n;
                    const int rs = 63 - __clzll((long long)((rst & le) | 1ull));
                    if (rs_me && vl && re - lane >= 2)
                        atomicAdd((unsigned long long*)&Lw.F[code], (unsigned long long)f_tie((u64)(re - lane)));
                    const int gs = 63 - __clzll((long long)((gst & le) | 1ull));
                    const u64 gaft = gst & ~le;
                    const int ge = gaft ? __builtin_ctzll(gaft) : n;
                    Lw.dcnt[sg] = (u8)(vl ? re - rs : 0);
                    wsync();
                    const rk_v4i dw = *(const rk_v4i*)(Lw.dcnt + 16 * g4);
                    rk_v4i odb[NC], qb[NC];
#pragma unroll
                    for (int t = 0; t < NC; ++t) {
                        qb[t] = zero;
#pragma unroll
                        for (int d = 0; d < 4; ++d) odb[t][d] = (int)(((u32)ob[t][d] * 0xffu) & (u32)dw[d]);
                    }
#pragma unroll
                    for (int mt = 0; mt < 4; ++mt) {
                        if (mt >= nmt) break;
                        const int gsr = __shfl(gs, 16 * mt + r16, 64), ger = __shfl(ge, 16 * mt + r16, 64);
                        rk_v4i eq;
#pragma unroll
                        for (int d = 0; d < 4; ++d)
                            eq[d] = (int)(rk_lt_bytes(ger, 16 * d + 4 * g4) - rk_lt_bytes(gsr, 16 * d + 4 * g4));
#pragma unroll
                        for (int t = 0; t < NC; ++t) {
                            const rk_v4i q = rk_mfma16(eq, ob[t], zero);
                            qb[t][mt] = (int)((u32)q[0] | ((u32)q[1] << 8) | ((u32)q[2] << 16) | ((u32)q[3] << 24));
                        }
                    }
#pragma unroll
                    for (int ma = 0; ma < NC; ++ma)
#pragma unroll
                        for (int nb = ma; nb < NC; ++nb) {
                            const int t = rk_tile16<NC>(ma, nb);
                            R[t] = rk_mfma16(ob[ma], qb[nb], R[t]);
                            X[t] = rk_mfma16(odb[ma], qb[nb], X[t]);
                            X[t] = rk_mfma16(qb[ma], odb[nb], X[t]);
                        }
                    wsync();
                }
                wsync();
                stamp(3);
            }
        }
    }
    if (cur >= 0) flush();
    stamp(4);
    if (stm && lane == 0)
        for (int q = 0; q < 8; ++q) atomicAdd(&g_rk_stamps[q], (unsigned long long)tph[q]);
}

// ===================================================================== cross
// Cross-bucket rank sums: for tested pair (a, b) of gene g,
//   S_ab += sum over buckets beta of h_beta[a] * #(b-elements in buckets < beta)
// one wave per (gene, pair), lanes over buckets (inclusive scan per 64).
// SEG: the same over the sub-buckets of each re-split parent (k_rank_resplit).
template <bool SEG>
__global__ void __launch_bounds__(256) k_rank_cross(ScRankLaunch A)
{
    const int lane = threadIdx.x & 63;
    const int W = blockIdx.x * 4 + scc_wave_id(), NW = gridDim.x * 4;
    const int ng = SEG ? A.counts[SCC_CNT_STRIDE * (10)] : split_count(A), P = A.P, nbig = A.counts[SCC_CNT_STRIDE * (13)];
    for (int f = W; f < ng * P; f += NW) {
        const int gi = f / P, p = f - gi * P;
        int g, bk0, nb;
        if (SEG) {
            const int4 sg = A.rsseg[gi];
            g = sg.x;
            bk0 = sg.y;
            nb = sg.z;
        } else {
            g = split_gene_at(A, nbig, gi);
            bk0 = A.gene_bk[2 * g];
            nb = A.gene_bk[2 * g + 1];
        }
        if (!A.all_pairs && !(A.flags[(size_t)p * A.G + g] & 1)) continue;
        int a, b;
        pair_decode(p, A.K, a, b);
        const unsigned int* h = A.hbg + (size_t)bk0 * A.K;
        u64 s = 0, carry = 0;
        for (int q0 = 0; q0 < nb; q0 += 64) {
            const int q = q0 + lane;
            const u32 ha = (q < nb) ? h[(size_t)q * A.K + a] : 0u;
            const u32 hb = (q < nb) ? h[(size_t)q * A.K + b] : 0u;
            u32 inc = hb;
            for (int o = 1; o < 64; o <<= 1) {
                const u32 y = __shfl_up(inc, o, 64);
                if (lane >= o) inc += y;
            }
            s += (u64)ha * (carry + inc - hb);
            carry += (u32)__shfl((int)inc, 63, 64);
        }
        s = u64_wave_sum(s);
        if (lane == 0 && s) atomicAdd((unsigned long long*)&A.accS[(size_t)p * A.G + g], (unsigned long long)s);
    }
}

// Gene-level cross terms, one workgroup per split gene:
//   S_ab += sum_q H[q][a] * C[q][b],  C[q][b] = #(b-elements in buckets < q)
// over the gene's buckets q in value order.  The gene's histogram rows are
// read once, 64 buckets at a time, into LDS (coalesced: rows are [bucket][K]),
// C comes from a column scan with a carry, and each thread accumulates its
// tested pairs (<= XC_J per thread) in registers: one atomic per (gene, pair).
// (The per-(gene, pair) wave version re-read the rows once per pair.)
#define XC_T 256
#define XC_Q 64                 // buckets per LDS round
#define XC_KC SCC_MAX_K         // cluster columns held
#define XC_J 8                  // tested pairs per thread per pass over the rows (2048)
#define XC_PF ((XC_Q * XC_KC + XC_T - 1) / XC_T)  // histogram words a thread prefetches per round
// SEG: the same sum over the sub-buckets of each re-split parent (the
// in-parent cross term; segments from k_rank_resplit*, rsseg).
// Each round's rows are loaded into registers while the previous round is
// summed (its latency off the per-gene chain), and every pair's sum over a
// round runs as four independent partial sums (the LDS reads in flight
// together): one workgroup walks a gene's buckets in order, so the per-round
// chain is what its time was (config D: 2.5 ms, D SLOW 7.8 ms before).
template <bool SEG>
__global__ void __launch_bounds__(XC_T) k_rank_cross_gene(ScRankLaunch A)
{
    // cluster-major: a pair's rows of one round are contiguous, read 4 at a time
    // (16-B LDS reads; the row stride XC_Q + 4 words spreads the clusters over banks)
    __shared__ __attribute__((aligned(16))) u32 Hs[XC_KC][XC_Q + 4];
    __shared__ __attribute__((aligned(16))) u32 Cs[XC_KC][XC_Q + 4];
    __shared__ u32 seg[XC_T / XC_KC][XC_KC];
    __shared__ u32 carry[XC_KC];
    constexpr int NPART = XC_T / XC_KC, RPP = XC_Q / NPART;  // column-scan parts, rows per part
    const int tid = threadIdx.x, K = A.K, G = A.G, P = A.P;
    const int ng = SEG ? A.counts[SCC_CNT_STRIDE * (10)] : split_count(A), nbig = A.counts[SCC_CNT_STRIDE * (13)];
    for (int gi = blockIdx.x; gi < ng; gi += gridDim.x) {
        int g, bk0, nb;
        if (SEG) {
            const int4 sg = A.rsseg[gi];
            g = sg.x;
            bk0 = sg.y;
            nb = sg.z;
        } else {
            g = split_gene_at(A, nbig, gi);
            bk0 = A.gene_bk[2 * g];
            nb = A.gene_bk[2 * g + 1];
        }
        const int ntp = min(A.gene_nt[g], P);
        const u32* tl = A.gene_tp + (size_t)g * P;
        const int nw = XC_Q * K;  // histogram words of a full round
        // one round's rows into registers (clamped loads, masked past the gene)
        u32 hv[XC_PF];
        auto prefetch = [&](int q0) {
            const unsigned int* h = A.hbg + (size_t)(bk0 + q0) * K;
            const int lim = (min(XC_Q, nb - q0)) * K;
#pragma unroll
            for (int r = 0; r < XC_PF; ++r) {
                const int e = r * XC_T + tid;
                hv[r] = h[min(e, max(lim - 1, 0))];
                if (e >= lim) hv[r] = 0u;
            }
        };
        for (int j0 = 0; j0 < ntp; j0 += XC_J * XC_T) {  // windows of 2048 tested pairs
            u32 pv[XC_J];
            u64 acc[XC_J];
#pragma unroll
            for (int u = 0; u < XC_J; ++u) {
                const int j = j0 + u * XC_T + tid;
                pv[u] = j < ntp ? tl[j] : 0u;
                acc[u] = 0;
            }
            if (nb > 0) prefetch(0);
            __syncthreads();
            if (tid < XC_KC) carry[tid] = 0;
            for (int q0 = 0; q0 < nb; q0 += XC_Q) {
                const int nq = min(XC_Q, nb - q0);
                __syncthreads();
#pragma unroll
                for (int r = 0; r < XC_PF; ++r) {
                    const int e = r * XC_T + tid;
                    if (e < nw) {
                        const int q = e / K, c = e - q * K;
                        Hs[c][q] = hv[r];
                    }
                }
                if (q0 + XC_Q < nb) prefetch(q0 + XC_Q);  // the next round's rows, in flight meanwhile
                __syncthreads();
                // column scan: thread (c, part) sums RPP rows, parts combined through LDS
                const int c = tid % XC_KC, part = tid / XC_KC;
                u32 ssum = 0;
                if (c < K)
                    for (int q = part * RPP; q < part * RPP + RPP; ++q) ssum += Hs[c][q];
                seg[part][c] = ssum;
                __syncthreads();
                if (c < K) {
                    u32 run = carry[c];
                    for (int v = 0; v < part; ++v) run += seg[v][c];
                    for (int q = part * RPP; q < part * RPP + RPP; ++q) {
                        Cs[c][q] = run;
                        run += Hs[c][q];
                    }
                }
                __syncthreads();
                if (tid < K)
                    for (int v = 0; v < NPART; ++v) carry[tid] += seg[v][tid];
#pragma unroll
                for (int u = 0; u < XC_J; ++u) {
                    if (j0 + u * XC_T + tid < ntp) {
                        const int a = (int)((pv[u] >> 16) & 0xffu), b = (int)(pv[u] >> 24);
                        u64 s0 = 0, s1 = 0, s2 = 0, s3 = 0;  // (rows past nq are zero)
                        const uint4* ha = (const uint4*)Hs[a];
                        const uint4* cb = (const uint4*)Cs[b];
#pragma unroll 4
                        for (int q4 = 0; q4 < XC_Q / 4; ++q4) {
                            const uint4 hx = ha[q4], cx = cb[q4];
                            s0 += (u64)hx.x * cx.x;
                            s1 += (u64)hx.y * cx.y;
                            s2 += (u64)hx.z * cx.z;
                            s3 += (u64)hx.w * cx.w;
                        }
                        acc[u] += (s0 + s1) + (s2 + s3);
                    }
                }
                (void)nq;
            }
#pragma unroll
            for (int u = 0; u < XC_J; ++u) {
                if (j0 + u * XC_T + tid < ntp && acc[u])
                    atomicAdd((unsigned long long*)&A.accS[(size_t)(pv[u] & 0xffffu) * G + g], (unsigned long long)acc[u]);
            }
        }
        __syncthreads();
    }
}

// ===================================================================== host
// bytes of an item's tested-pair tables (tp, cp, eacc, xacc, pmap)
static size_t item_tables_bytes(int ntp_max, int K)
{
    const size_t s = sizeof(u32) * (2 * (size_t)ntp_max + 1) + 8 + 16 * (size_t)ntp_max + 2 * (size_t)K * K;
    return (s + 31) & ~(size_t)15;
}

// tables past 24 KB (many tested pairs per gene, K > ~40) live in HBM scratch
extern "C" int scc_rank_tables_global(int ntp_max, int K) { return item_tables_bytes(ntp_max, K) > 24 * 1024; }
extern "C" size_t scc_rank_tables_stride(int ntp_max, int K) { return (item_tables_bytes(ntp_max, K) + 255) & ~(size_t)255; }

template <int W>
static size_t item_lds_fixed(int ntp_max, int K)
{
    const size_t s = sizeof(ItemLds<W>) + (scc_rank_tables_global(ntp_max, K) ? 16 : item_tables_bytes(ntp_max, K));
    return (s + 31) & ~(size_t)15;
}

#define RK_T0 256   // small items
#define RK_T1 512   // medium items (two workgroups per CU)
#define RK_T2 1024  // HBM-resident items

extern "C" size_t scc_rank_item_lds(int cls, int cap, int ntp_max, int K)
{
    if (cls == 0) return item_lds_fixed<RK_T0 / 64>(ntp_max, K) + (size_t)cap * (4 + 2 + 2 + 1 + 1);
    if (cls == 1) return item_lds_fixed<RK_T1 / 64>(ntp_max, K) + (size_t)cap * (4 + 2 + 2 + 1 + 1);
    return item_lds_fixed<RK_T2 / 64>(ntp_max, K);
}

// largest LDS-resident item capacity (multiple of 64) of class cls within lim bytes
#define RK_KPT0 8   // cap_s <= 8 * 256
#define RK_KPT1 8  // cap_m <= 8 * 512

extern "C" int scc_rank_item_cap(int cls, int want, int ntp_max, int K, int lim)
{
    int cap = want & ~63;
    if (cls == 0 && cap > RK_KPT0 * RK_T0) cap = RK_KPT0 * RK_T0;
    if (cls == 1 && cap > RK_KPT1 * RK_T1) cap = RK_KPT1 * RK_T1;
    while (cap > 64 && scc_rank_item_lds(cls, cap, ntp_max, K) > (size_t)lim) cap -= 64;
    if (cap > 65535) cap = 65535 & ~63;
    return cap;
}

extern "C" size_t scc_rank_split_lds(int K)
{
    (void)K;
    return kSplitStageOff + (size_t)SP_CHUNK * (sizeof(u64) + 1);
}

// Launches that may run concurrently taken round st0, side[0], side[1], ...:
// a side stream waits on the fork event (recorded on st0 before the first
// launch: a record costs no wait) when it first gets a launch, and st0 waits on
// its join event at the end.  nside 0: everything on st0.
struct SideStreams {
    hipStream_t st0;
    const hipStream_t* side;
    int nside;
    hipEvent_t fork;
    const hipEvent_t* join;
    bool used[4] = {false, false, false, false};
    int turn = 0;
    SideStreams(hipStream_t s, const hipStream_t* sd, int n, hipEvent_t f, const hipEvent_t* j)
        : st0(s), side(sd), nside((f && j && sd) ? std::min(n, 4) : 0), fork(f), join(j)
    {
        if (nside > 0) hipEventRecord(fork, st0);
    }
    hipStream_t next()
    {
        const int t = turn++;
        if (nside <= 0 || t % (nside + 1) == 0) return st0;
        return pick(t % (nside + 1) - 1);
    }
    hipStream_t pick(int i)  // -1: st0; i: side[i] (st0 when there are fewer sides)
    {
        if (i < 0 || i >= nside) return st0;
        if (!used[i]) hipStreamWaitEvent(side[i], fork, 0);
        used[i] = true;
        return side[i];
    }
    void end()
    {
        for (int i = 0; i < nside; ++i)
            if (used[i]) {
                hipEventRecord(join[i], side[i]);
                hipStreamWaitEvent(st0, join[i], 0);
                used[i] = false;
            }
    }
};

static hipError_t rank_waves_launches(const ScRankLaunch* L, int grid, SideStreams& ss);

extern "C" hipError_t scc_launch_rank_waves(const ScRankLaunch* L, int grid, hipStream_t st0, const hipStream_t* side,
                                            int nside, hipEvent_t fork, const hipEvent_t* join)
{
    SideStreams ss(st0, side, nside, fork, join);
    const hipError_t e = rank_waves_launches(L, grid, ss);
    ss.end();
    return e != hipSuccess ? e : hipGetLastError();
}

static hipError_t rank_waves_launches(const ScRankLaunch* L, int grid, SideStreams& ss)
{
    // the launches below touch disjoint genes' accumulator cells (each gene is
    // in one class) or, for the windows of one gene, disjoint pair rows, and
    // read only what the split wrote: they may run concurrently, so each takes
    // the next stream in turn and their tails overlap (a gene shard's grid is
    // an eighth of the whole job's and each launch ended on a long tail)
    // With two sides (the runtime passes {a side stream, the LDS items'
    // stream}: three hardware queues) the launches take fixed places, longest
    // chains apart (config D timeline, profiles/r06_timeline_rank_d_*.txt):
    // matrix-core genes on side 1 ahead of the items, <= 128 tested pairs on
    // side 0 (the largest class), <= 256 then <= 512 on st0.  Otherwise round robin.
    auto next_stream = [&]() { return ss.next(); };
    auto place = [&](int role) {  // 0..3: slot class, 4: matrix cores, 5: windows
        if (ss.nside < 2) return ss.next();
        static const int where[6] = {0, -1, -1, 1, 1, -1};
        return ss.pick(where[role]);
    };
    hipStream_t st = ss.st0;
    // one launch per slot class present: genes with <= 128 tested pairs on the
    // 2-slot kernel, <= 256 on 4, <= 512 on 8, <= 1024 on 16
    // the matrix-core kernel (K <= 64) counts all K^2 pairs of a bucket at a
    // fixed cost: it takes the genes with more than 512 tested pairs (SLOW at
    // config D: every gene, 1225 pairs), the slot kernels the others
    // (SCC_RANK_MFMA=2: every gene on the matrix cores, 0: none)
    // (from 256 or 128 tested pairs, or every gene, measured slower at config D: rank
    // 22.6 / 29.0 / 31.9 vs 20.2 ms, round 6)
    constexpr int mfma_min = 512;  // the tested-pair count past which a gene goes there
    const int hi[4] = {128, 256, 512, 1024};
    const bool mfma = L->rw_mfma && L->K <= 64 && (L->rw_mfma == 2 || 64 * L->rw_slots > mfma_min);
    if (mfma) {
        ScRankLaunch M = *L;
        M.wv_filter = L->rw_mfma == 2 ? 0 : 1;
        M.wv_lo = mfma_min;
        st = place(4);
        M.wv_hi = 1 << 30;
        if (L->K <= 16)
            hipLaunchKernelGGL(k_rank_mfma16<1>, dim3(grid), dim3(256), 0, st, M);
        else if (L->K <= 32)
            hipLaunchKernelGGL(k_rank_mfma16<2>, dim3(grid), dim3(256), 0, st, M);
        else if (L->K <= 48)
            hipLaunchKernelGGL(k_rank_mfma16<3>, dim3(grid), dim3(256), 0, st, M);
        else
            hipLaunchKernelGGL(k_rank_mfma16<4>, dim3(grid), dim3(256), 0, st, M);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess || L->rw_mfma == 2) return e;
    }
    ScRankLaunch A = *L;
    // the 16-wide matrix-core kernel for the genes the slot kernels would take:
    // by default at K <= 16 (four waves per SIMD; config B rank 0.785 -> 0.744
    // ms), SCC_RANK_MFMA16=1 also at K <= 32 (two waves: config C 8.6 -> 10.2 ms)
    if (L->rw_mfma16 > 0 ? L->K <= 32 : (L->rw_mfma16 < 0 && L->K <= 16)) {
        ScRankLaunch M = *L;
        M.wv_filter = mfma ? 1 : 0;
        M.wv_lo = -1;
        M.wv_hi = mfma ? mfma_min : (1 << 30);
        if (L->K <= 16)
            hipLaunchKernelGGL(k_rank_mfma16<1>, dim3(grid), dim3(256), 0, st, M);
        else
            hipLaunchKernelGGL(k_rank_mfma16<2>, dim3(grid), dim3(256), 0, st, M);
        return hipGetLastError();
    }
    for (int c = 0; c < 4; ++c) {
        if (c > 0 && 64 * L->rw_slots < hi[c]) break;
        if (mfma && hi[c] > mfma_min) return hipSuccess;  // the genes past mfma_min: done on the matrix cores
        A.wv_lo = c ? hi[c - 1] : -1;
        A.wv_hi = hi[c];
        A.wv_base = 0;
        A.wv_filter = L->rw_slots > 2 ? 1 : 0;  // rw_slots 2: class 0 is the only launch and holds every gene
        st = place(c);
        if (c == 0)
            hipLaunchKernelGGL(k_rank_waves<2>, dim3(grid), dim3(256), 0, st, A);
        else if (c == 1)
            hipLaunchKernelGGL(k_rank_waves<4>, dim3(grid), dim3(256), 0, st, A);
        else if (c == 2)
            hipLaunchKernelGGL(k_rank_waves<8>, dim3(grid), dim3(256), 0, st, A);
        else
            hipLaunchKernelGGL(k_rank_waves<RW_SLOTS_MAX>, dim3(grid), dim3(256), 0, st, A);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    // genes with more than 1024 tested pairs (SLOW at K > 45, K > 64 runs): one
    // 16-slot pass per window of 1024 pairs, window k over the genes that reach it
    if (L->rw_slots >= RW_SLOTS_MAX) {
        const int per = 64 * RW_SLOTS_MAX;
        const int npass = (std::min(L->ntp_max, RW_PAIRS_MAX) + per - 1) / per;
        st = place(5);  // (the windows in one stream)
        for (int k = 0; k < npass; ++k) {
            A.wv_lo = std::max(per, k * per);
            A.wv_hi = RW_PAIRS_MAX;
            A.wv_base = k * per;
            A.wv_filter = 1;
            hipLaunchKernelGGL(k_rank_waves<RW_SLOTS_MAX>, dim3(grid), dim3(256), 0, st, A);
            const hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
    }
    return hipSuccess;
}

extern "C" hipError_t scc_launch_rank_cross(const ScRankLaunch* L, int grid, hipStream_t st)
{
    // per-gene workgroups pay off once genes have many tested pairs (at P = 66 the
    // per-(gene, pair) waves are 12 us faster; at P >= 435 the gene kernel wins)
    if (L->P > 128 && !L->cross_wave)
        hipLaunchKernelGGL(k_rank_cross_gene<false>, dim3(grid), dim3(XC_T), 0, st, *L);
    else  // one wave per (gene, pair) (SCC_CROSS_WAVE=1 selects it for comparisons)
        hipLaunchKernelGGL(k_rank_cross<false>, dim3(grid), dim3(256), 0, st, *L);
    return hipGetLastError();
}

extern "C" hipError_t scc_launch_rank_cross_seg(const ScRankLaunch* L, int grid, hipStream_t st)
{
    if (!L->fatbk) return hipSuccess;
    if (L->P > 128 && !L->cross_wave)  // one workgroup per segment, its rows read once (as the gene level)
        hipLaunchKernelGGL(k_rank_cross_gene<true>, dim3(grid), dim3(XC_T), 0, st, *L);
    else
        hipLaunchKernelGGL(k_rank_cross<true>, dim3(grid), dim3(256), 0, st, *L);
    return hipGetLastError();
}

extern "C" hipError_t scc_launch_rank_resplit(const ScRankLaunch* L, int grid, hipStream_t st0, const hipStream_t* side,
                                              int nside, hipEvent_t fork, const hipEvent_t* join)
{
    if (!L->fatbk || grid <= 0) return hipSuccess;
    // the first level's three launches take disjoint parents (<= RSW_CAP
    // elements by tested-pair class, larger ones) and meet only in atomic
    // allocation counters: concurrent; the second level reads the first's fat2
    SideStreams ss(st0, side, nside, fork, join);
    hipStream_t st = st0;
    // wave-private allocation chunks sized so that the unused tails of all
    // waves stay a small part of the bucket capacity
    ScRankLaunch W = *L;
    const long long waves = 2LL * grid * 4;
    W.rsw_chunk = (int)std::max(8LL, std::min(128LL, (long long)L->bucket_cap / (16 * waves)));
    W.rs_level = 0;
    // K > 64 (config E): most genes hold more than 512 tested pairs, one launch
    // of the wide variant takes every parent (a second pass over the list cost more)
    W.rsw_all = L->K > 64 ? 1 : 0;
    if (!W.rsw_all) hipLaunchKernelGGL(k_rank_resplit_w<RSW_TS_SMALL>, dim3(2 * grid), dim3(256), 0, ss.next(), W);
    if (L->P > 64 * RSW_TS_SMALL)
        hipLaunchKernelGGL(k_rank_resplit_w<RSW_PACC / 64>, dim3(2 * grid), dim3(256), 0, ss.next(), W);
    const size_t acc_lds = sizeof(u64) * (size_t)std::max(L->P, 1);
    scc_set_lds((const void*)k_rank_resplit, (int)acc_lds);
    hipLaunchKernelGGL(k_rank_resplit, dim3(grid), dim3(RS_T), acc_lds, ss.next(), *L);
    ss.end();
    if (L->fat2) {  // sub-buckets the first level left with > 64 distinct values
        W.rs_level = 1;
        if (!W.rsw_all) hipLaunchKernelGGL(k_rank_resplit_w<RSW_TS_SMALL>, dim3(2 * grid), dim3(256), 0, st, W);
        if (L->P > 64 * RSW_TS_SMALL)
            hipLaunchKernelGGL(k_rank_resplit_w<RSW_PACC / 64>, dim3(2 * grid), dim3(256), 0, st, W);
    }
    return hipGetLastError();
}

extern "C" hipError_t scc_launch_rank_split(const ScRankLaunch* L, int grid, hipStream_t st)
{
    if (grid <= 0) return hipSuccess;
    const size_t lds = scc_rank_split_lds(L->K);
    scc_set_lds((const void*)k_rank_split, (int)lds);
    hipLaunchKernelGGL(k_rank_split, dim3(grid), dim3(SP_T), lds, st, *L);
    return hipGetLastError();
}

extern "C" hipError_t scc_launch_rank_items(const ScRankLaunch* L, int cls, int grid, hipStream_t st)
{
    if (grid <= 0) return hipSuccess;
    ScRankLaunch A = *L;
    if (cls == 0) {
        A.cap_lds = L->cap_s;
        const size_t lds = scc_rank_item_lds(0, L->cap_s, L->ntp_max, L->K);
        scc_set_lds((const void*)k_rank_item<RK_T0, false, RK_KPT0>, (int)lds);
        hipLaunchKernelGGL((k_rank_item<RK_T0, false, RK_KPT0>), dim3(grid), dim3(RK_T0), lds, st, A, 0);
    } else if (cls == 1) {
        A.cap_lds = L->cap_m;
        const size_t lds = scc_rank_item_lds(1, L->cap_m, L->ntp_max, L->K);
        scc_set_lds((const void*)k_rank_item<RK_T1, false, RK_KPT1>, (int)lds);
        hipLaunchKernelGGL((k_rank_item<RK_T1, false, RK_KPT1>), dim3(grid), dim3(RK_T1), lds, st, A, 1);
    } else {
        A.cap_lds = 0;
        const size_t lds = scc_rank_item_lds(2, 0, L->ntp_max, L->K);
        scc_set_lds((const void*)k_rank_item<RK_T2, true, 1>, (int)lds);
        hipLaunchKernelGGL((k_rank_item<RK_T2, true, 1>), dim3(grid), dim3(RK_T2), lds, st, A, 2);
    }
    return hipGetLastError();
}
